#!/bin/bash
# k_band_dec phase costs: isolated resize_h1 time with phases skipped (option dec_dbg bits:
# 1 IDCT, 2 fill, 4 MFMA conv, 8 stores).  Pixels are wrong in the skipped runs: timing only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/phases
mkdir -p $OUT
for v in ${DBGS:-0 1 2 4 8 3 6 15}; do
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --serial-steps 3 --no-cpu-baseline --e2e-steps 0 --one-threads 0 \
    --ctx-opt band_dec=1 --ctx-opt dec_dbg=$v $EXTRA --out $OUT/dbg$v.json > $OUT/dbg$v.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/dbg$v.json'));s=d['roofline_isolated']['stages_ms'];print('dbg=$v h1',s['resize_h1'],'value',d['value'])"
done
