#!/bin/bash
# GPU parity tests, then the PMC passes (gpu_pmc.sh), then a bench sweep
# ($SWEEP).  Test assertion failures (exit 1) do not stop it; a crash,
# abort or timeout does.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -q -m gpu -x --timeout 240 \
    --timeout-method thread > gpurun_out/pt.log 2>&1
rc=$?; tail -3 gpurun_out/pt.log; [ $rc -le 1 ] || exit $rc
bash tools/gpu_pmc.sh || exit $?
[ -n "${SWEEP:-}" ] && STEPS=${STEPS:-8} POOL=${POOL:-4096} timeout -k 10 600 bash tools/gpu_sweep.sh
