#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/if6
mkdir -p $OUT
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
for i in 4 6 5; do
  timeout -k 10 400 python bench.py --workload png --steps 8 --warmup 2 --inflight $i $B --out $OUT/png_if$i.json > $OUT/png_if$i.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/png_if$i.json'));print('png inflight $i',d['value'],d['ms_per_step'])"
done
for i in 3 4 3; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 2 --inflight $i $B --out $OUT/jpeg_if$i.json > $OUT/jpeg_if$i.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/jpeg_if$i.json'));print('jpeg inflight $i',d['value'],d['ms_per_step'])"
done
