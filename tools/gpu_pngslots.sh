#!/bin/bash
# configs[4] with 4/5/6 batches in flight now that k_inf_decode holds 24 KiB of LDS per wave.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pngslots
mkdir -p $OUT
for rep in 1 2; do
for v in 4 5 6; do
  timeout -k 10 400 python bench.py --workload png --steps 30 --warmup 4 --e2e-steps 0 --one-threads 0 --no-cpu-baseline --inflight $v --out $OUT/png_i${v}_r$rep.json > $OUT/png_i${v}_r$rep.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/png_i${v}_r$rep.json'));print('i$v r$rep',d['value'])"
done
done
