#!/bin/bash
# Slot prewarm check: budget + parity tests, the headline (5 windows: the first
# one no longer pays for the fourth slot's buffers), the dg_decode_one leg and the
# configs[4] line.  OUT=gpurun_out/r5l
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5l}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_budget.py tests/test_gpu_parity.py tests/test_gpu_exit.py > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/tests.log | head; exit $rc; }
for r in 1 2; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --e2e-steps 0 --out $OUT/bench_$r.json > $OUT/bench_$r.log 2>&1 || { tail -20 $OUT/bench_$r.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$r.json'));o=d.get('e2e_decode_one') or {};print('headline',d['value'],d['windows']['mpix_s'],'one',o.get('mpix_s'),(o.get('native_threads') or {}).get('mpix_s'),d['allocations'])"
done
timeout -k 10 400 python bench.py --workload png --steps 10 --warmup 2 --windows 3 --e2e-steps 0 --one-threads 0 --no-cpu-baseline --out $OUT/png.json > $OUT/png.log 2>&1 || { tail -20 $OUT/png.log; exit 1; }
python -c "import json;d=json.load(open('$OUT/png.json'));print('png',d['value'],d['windows']['mpix_s'],d['allocations']['peak_device_mb'])"
