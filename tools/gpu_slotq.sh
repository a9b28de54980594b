#!/bin/bash
# Baseline slots' streams on hardware queues of their own (option slot_queue): PNG and JPEG workloads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/slotq
mkdir -p $OUT
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
for q in 0 3 1 0 3; do
  timeout -k 10 400 python bench.py --workload png --steps 8 --warmup 2 $B --ctx-opt slot_queue=$q --out $OUT/png_q$q.json > $OUT/png_q$q.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/png_q$q.json'));print('png slot_queue $q',d['value'],d['ms_per_step'])"
done
for q in 0 3 1 0 3; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 2 $B --ctx-opt slot_queue=$q --out $OUT/jpeg_q$q.json > $OUT/jpeg_q$q.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/jpeg_q$q.json'));print('jpeg slot_queue $q',d['value'],d['ms_per_step'])"
done
