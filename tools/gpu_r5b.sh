#!/bin/bash
# Round-5 checks: the budget / table-cache / exit / parity suites, two default bench
# lines, then the dg_decode_one leg under rocprofv3 (the r4 exit-time SIGSEGV) last.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5b}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 700 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${FILES:-tests/test_gpu_budget.py tests/test_gpu_coef_cache.py tests/test_gpu_exit.py tests/test_gpu_progressive.py tests/test_gpu_samples.py tests/test_gpu_robustness.py tests/test_gpu_parity.py} > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/tests.log | head -20; exit $rc; }
fi
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e-steps 0 --one-threads 0 --no-cpu-baseline ${EXTRA:-} --out $OUT/bench_$r.json > $OUT/bench_$r.log 2>&1 || { tail -20 $OUT/bench_$r.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$r.json'));s=d['roofline_isolated']['stages_ms'];print(d['value'],d['ms_per_step'],d['windows']['mpix_s'],{k:round(v,3) for k,v in s.items() if v>0.05});print(d['allocations'])"
done
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 2 --warmup 1 --windows 1 --e2e-steps 0 --no-cpu-baseline --serial-steps 0 --one-threads 32 --one-images 2048 --out $OUT/one.json > $OUT/prof.log 2>&1
  echo "rocprof rc=$?"
  tail -5 $OUT/prof.log
fi
