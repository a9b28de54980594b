#!/bin/bash
# Headline bench over context-option variants ($OPTS: ';'-separated lists of --ctx-opt k=v).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/optsweep
mkdir -p $OUT
i=0
IFS=';' read -ra CFGS <<< "$OPTS"
for cfg in "${CFGS[@]}"; do
  i=$((i + 1))
  args=""
  for kv in $cfg; do [ "$kv" = "-" ] || args="$args --ctx-opt $kv"; done
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e-steps 0 --one-threads 0 --no-cpu-baseline $args --out $OUT/b_$i.json > $OUT/b_$i.log 2>&1
  rc=$?; echo "=== [$cfg] exit $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/b_$i.json'));s=d['roofline_isolated']['stages_ms'];print(d['value'],d['ms_per_step'],s['huff_sync'],s['huff_write'],s['resize_h1'])"
done
