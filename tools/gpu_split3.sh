#!/bin/bash
# Progressive aggregate size (option prog_batch): 100%-progressive pool and 10% mix.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/split3
mkdir -p $OUT
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
for pb in ${PBS:-1024 2048 4096}; do
  timeout -k 10 400 python bench.py --progressive-frac 1.0 --pool 2048 --steps ${P100_STEPS:-24} --warmup 8 $B \
      --ctx-opt prog_batch=$pb --out $OUT/p100_pb$pb.json > $OUT/p100_pb$pb.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/p100_pb$pb.json'));print('p100 pb$pb',d['value'],d['ms_per_step'])"
  timeout -k 10 400 python bench.py --progressive-frac 0.1 --pool 4096 --steps ${MIX_STEPS:-200} --warmup 8 $B \
      --ctx-opt prog_batch=$pb --out $OUT/mix10_pb$pb.json > $OUT/mix10_pb$pb.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/mix10_pb$pb.json'));print('mix10 pb$pb',d['value'],d['ms_per_step'])"
done
