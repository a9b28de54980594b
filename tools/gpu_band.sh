#!/bin/bash
# k_band_dec bring-up: its GPU tests first (stop on the first failure), then
# the whole GPU suite and an A/B bench (band_dec 1 vs 0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/band
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -x -v --timeout 120 --timeout-method thread > $OUT/band_tests.log 2>&1
rc=$?; tail -15 $OUT/band_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
for v in 1 0 1 0; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --e2e-steps 0 --one-threads 0 \
    --ctx-opt band_dec=$v --out $OUT/ab_band$v.json > $OUT/ab_band$v.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/ab_band$v.json'));print('band_dec=$v',d['value'],d['roofline_isolated']['stages_ms'])"
done
