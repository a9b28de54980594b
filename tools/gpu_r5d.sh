#!/bin/bash
# dg_decode_one small-batch entropy options (sub_small / lead_small under small_coded), then the
# configs[2] WebDataset line with and without the Lanczos table cache.  OUT=gpurun_out/r5d
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5d}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
OUT=$OUT/one ONE_IMAGES=2048 THREADS=32 OPTS="${ONE_OPTS:-;small_coded=33554432 sub_small=512 lead_small=4096;small_coded=33554432 sub_small=1024 lead_small=4096;small_coded=33554432 sub_small=1024 lead_small=2048}" tools/gpu_one.sh || exit $?
OUT=$OUT/wds AB="coef_cache_mb=0" EXTRA="--workload wds" TESTS=0 REPS=${WDS_REPS:-2} tools/gpu_ab2.sh || exit $?
