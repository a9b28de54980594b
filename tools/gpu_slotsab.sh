#!/bin/bash
# 3 vs 4 baseline slots with the driver's default bench flow (CPU baselines, e2e legs), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/slotsab
mkdir -p $OUT
for r in 1 2; do for i in 4 3; do
  timeout -k 10 500 python bench.py --inflight $i --out $OUT/d_if${i}_$r.json > $OUT/d_if${i}_$r.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/d_if${i}_$r.json'));print('default flow inflight $i run $r',d['value'],d['ms_per_step'])"
done; done
