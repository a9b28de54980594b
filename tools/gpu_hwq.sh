#!/bin/bash
# Headline bench at 3/4 batches in flight with GPU_MAX_HW_QUEUES 4 (default) and 8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/hwq
mkdir -p $OUT
i=0
for rep in 1 2; do
  for q in 4 8; do
    for inf in 3 4; do
      i=$((i + 1))
      GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 20 --warmup 3 --inflight $inf --no-cpu-baseline --e2e-steps 0 --one-threads 0 --out $OUT/b_$i.json > $OUT/b_$i.log 2>&1
      rc=$?; echo "=== [queues $q inflight $inf] exit $rc"; [ $rc -eq 0 ] || exit $rc
      python -c "import json;d=json.load(open('$OUT/b_$i.json'));print(d['value'],d['ms_per_step'])"
    done
  done
done
