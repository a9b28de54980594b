#!/bin/bash
# Experiment session: build check, the GPU parity tests (or $TESTS), then a
# bench sweep ($SWEEP, see gpu_sweep.sh).  Each GPU step has its own timeout;
# a crash or timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -c "import datago_amd._lib as L; L.load(); print('lib ok')" || exit 3
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -q -m gpu -x --timeout 300 --timeout-method thread \
    > gpurun_out/pt.log 2>&1
rc=$?; tail -3 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
POOL=${POOL:-4096} timeout -k 10 900 bash tools/gpu_sweep.sh
