#!/bin/bash
# Isolated per-stage times and the headline for several context-option sets
# (VARIANTS: ';'-separated, each a space-separated list of key=value).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/variants
mkdir -p $OUT
STEPS=${STEPS:-8}
i=0
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
  opts=""
  for kv in $v; do opts="$opts --ctx-opt $kv"; done
  timeout -k 10 400 python bench.py --steps $STEPS --warmup 2 --serial-steps 3 --no-cpu-baseline --e2e-steps 0 \
    --one-threads 0 $opts ${EXTRA:-} --out $OUT/v$i.json > $OUT/v$i.log 2>&1 || { tail -5 $OUT/v$i.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/v$i.json'));s=d['roofline_isolated']['stages_ms'];print('[$v]','value',d['value'],'sync',s['huff_sync'],'write',s['huff_write'],'h1',s['resize_h1'],'idct',s['idct'],'v1',s['resize_v1'],'stats',d['stats'],'wg',d.get('wg_timing_us'))"
  i=$((i+1))
done
