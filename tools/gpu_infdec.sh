#!/bin/bash
# k_inf_decode shapes (option inf_decode 0..3): parity, then configs[4] A/B alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/infdec4
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_png.py -k chunked_inflate > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -3 $OUT/test.log
for rep in 1 2; do  # variants 1..3 vs 0
for v in 0 2 3 4 5; do
  timeout -k 10 400 python bench.py --workload png --steps 30 --warmup 4 --e2e-steps 0 --one-threads 0 --no-cpu-baseline --ctx-opt inf_decode=$v --out $OUT/png_v${v}_r$rep.json > $OUT/png_v${v}_r$rep.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/png_v${v}_r$rep.json'));s=d['stages_ms_per_step'];print('v$v r$rep',d['value'],'inflate',s.get('png_inflate'))"
done
done
