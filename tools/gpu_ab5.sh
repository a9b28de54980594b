#!/bin/bash
# Round-5 A/B on the headline (defaults vs sparse_coef=0, coef_cache_mb=0, 5 slots), then
# PMC traffic per stage at the defaults (tools/gpu_pmc.sh).  OUT=gpurun_out/ab5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab5}
OUT=$OUT AB="${AB:-sparse_coef=0;coef_cache_mb=0;--inflight=5}" REPS=${REPS:-2} TESTS=0 tools/gpu_ab2.sh || exit $?
if [ "${PMC:-1}" = 1 ]; then
  OUT=$OUT/pmc tools/gpu_pmc.sh || exit $?
  python -c "import json;d=json.load(open('$OUT/pmc/pmc_traffic.json'));b=d['bytes_per_batch'];print({k:round(v/1e9,3) for k,v in b.items()}, 'total', round(sum(b.values())/1e9,3))"
fi
