#!/bin/bash
# PNG (configs[4]) session: the PNG GPU tests, then a kernel-trace profile of
# `bench.py --workload png` (per-kernel summary via tools/rocpd_stats.py).
# WORKLOAD= profiles another bench workload, NOTEST=1 skips the tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pngprof
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_png.py} -q -m gpu -x --timeout 300 --timeout-method thread \
      > gpurun_out/pngprof/pt.log 2>&1
  rc=$?; tail -3 gpurun_out/pngprof/pt.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/pngprof -o run -- python3 bench.py --workload ${WORKLOAD:-png} \
    --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --e2e-steps 0 --one-threads 0 --serial-steps 1 ${EXTRA:-} \
    --out gpurun_out/pngprof/b.json > gpurun_out/pngprof/b.log 2>&1
rc=$?; echo "bench rc $rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/rocpd_stats.py gpurun_out/pngprof/run_results.db --csv gpurun_out/pngprof/kernel_stats.csv | head -${TOP:-12}
python3 -c "import json;d=json.load(open('gpurun_out/pngprof/b.json'));print(d['value'],d['ms_per_step'],{k:round(v,2) for k,v in d['roofline_isolated']['stages_ms'].items() if v>0.05})"
