#!/bin/bash
# PNG unfilter tile width (option uf_units 2 vs 1): parity, then configs[4] alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ufu
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_png.py > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
for rep in 1 2; do
for v in 2 1; do
  timeout -k 10 400 python bench.py --workload png --steps 30 --warmup 4 --e2e-steps 0 --one-threads 0 --no-cpu-baseline --ctx-opt uf_units=$v --out $OUT/png_u${v}_r$rep.json > $OUT/png_u${v}_r$rep.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/png_u${v}_r$rep.json'));s=d['stages_ms_per_step'];print('u$v r$rep',d['value'],'unfilter',s.get('png_unfilter'))"
done
done
