#!/bin/bash
# PNG workload vs hardware queues (GPU_MAX_HW_QUEUES): do the slots' long inflate kernels serialise?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pnghwq
mkdir -p $OUT
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
for q in 4 8 16 4; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python bench.py --workload png --steps 8 --warmup 2 $B --out $OUT/png_q$q.json > $OUT/png_q$q.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/png_q$q.json'));print('png hwq $q',d['value'],d['ms_per_step'])"
done
