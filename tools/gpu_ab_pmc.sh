#!/bin/bash
# Coefficient planes check: the JPEG parity suites, then the headline A/B against
# dense coefficients (sparse_coef=0, or AB), then PMC traffic per stage.  OUT=gpurun_out/ab_pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab_pmc}
OUT=$OUT AB="${AB:-sparse_coef=0}" REPS=${REPS:-2} TESTS=${TESTS:-1} TLIM=600 \
  FILES="${FILES:-tests/test_gpu_parity.py tests/test_gpu_budget.py tests/test_gpu_coef_cache.py tests/test_gpu_exit.py tests/test_gpu_semantics.py}" \
  tools/gpu_ab2.sh || exit $?
if [ "${PMC:-1}" = 1 ]; then
  OUT=$OUT/pmc tools/gpu_pmc.sh || exit $?
  python -c "import json;d=json.load(open('$OUT/pmc/pmc_traffic.json'));b=d['bytes_per_batch'];print({k:round(v/1e9,3) for k,v in b.items()}, 'total', round(sum(b.values())/1e9,3))"
fi
