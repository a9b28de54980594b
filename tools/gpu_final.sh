#!/bin/bash
# Round-3 final evidence (tests, smoke, bench, rocprof), then an A/B of 3 vs 4 baseline slots.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS=20 bash tools/gpu_check.sh || exit $?
OUT=gpurun_out/slots
mkdir -p $OUT
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
for r in 1 2 3; do for i in 3 4; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 2 --inflight $i $B --out $OUT/jpeg_if${i}_$r.json > $OUT/jpeg_if${i}_$r.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/jpeg_if${i}_$r.json'));print('jpeg inflight $i run $r',d['value'],d['ms_per_step'])"
done; done
