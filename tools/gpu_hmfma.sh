#!/bin/bash
# k_resize_hm + sub_density bring-up: their tests, then the GPU suite, then A/B bench variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/hm
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_hmfma.py tests/test_gpu_entropy_density.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -8 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
VARIANTS="${VARIANTS:-h_mfma=1;h_mfma=0;h_mfma=1 sub_density=48;h_mfma=1 sub_density=80;h_mfma=1}" STEPS=20 bash tools/gpu_variants.sh
