#!/bin/bash
# 8 ranks sharing one GPU: hardware-queue options (each rank's slots on queues of their own oversubscribe the GPU's queues).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ranks2
mkdir -p $OUT
for v in "q0:--ctx-opt slot_queue=0" "q0s3:--ctx-opt slot_queue=0 --inflight 3" "q1s3:--inflight 3"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 700 python bench.py --gpus 8 --workload cfg4 --steps 6 --warmup 2 --e2e-steps 0 --one-threads 0 --no-cpu-baseline $args --out $OUT/g8_$name.json > $OUT/g8_$name.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/g8_$name.json'));print('gpus 8 cfg4 $name',d['value'])"
done
