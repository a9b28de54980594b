#!/bin/bash
# Progressive decoder check: GPU progressive tests, single-image probe, pool bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prog
timeout -k 10 300 python -u -m pytest tests/test_gpu_progressive.py -x -v --timeout 120 --timeout-method thread > gpurun_out/prog/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/prog/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/prog_probe.py > gpurun_out/prog/probe.log 2>&1
rc=$?; cat gpurun_out/prog/probe.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prog.sh
