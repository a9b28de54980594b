#!/bin/bash
# k_inf_find words staged through LDS: PNG + parity tests, configs[4] bench, rocprof kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/find
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_png.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python bench.py --workload png --steps 40 --warmup 4 --e2e-steps 0 --one-threads 0 --no-cpu-baseline --out $OUT/png.json > $OUT/png.log 2>&1 || exit $?
python -c "import json;d=json.load(open('$OUT/png.json'));print('png',d['value'],d['stages_ms_per_step'].get('png_inflate'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o png -- python3 bench.py --workload png --steps 10 --warmup 2 --e2e-steps 0 --one-threads 0 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit $?
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/png_kernel_stats.csv
head -8 $OUT/png_kernel_stats.csv | cut -c1-160
