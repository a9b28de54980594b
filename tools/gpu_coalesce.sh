#!/bin/bash
# dg_decode_one leg (32 threads, 2048 images) over coalescing options.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/coalesce
mkdir -p $OUT
i=0
for cfg in "" "--ctx-opt coalesce_us=200" "--ctx-opt coalesce_us=1000" "--ctx-opt coalesce_max=128" "--ctx-opt coalesce_max=32" "" "--ctx-opt coalesce_us=1000 --ctx-opt coalesce_max=128"; do
  i=$((i + 1))
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --e2e-steps 0 --one-threads 32 --one-images 2048 --no-cpu-baseline $cfg --out $OUT/b_$i.json > $OUT/b_$i.log 2>&1
  rc=$?; echo "=== [$cfg] exit $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/b_$i.json'));o=d['e2e_decode_one'];print(o['mpix_s'],o['images_per_s'],o['gpu_batches'],o['mean_images_per_batch'])"
done
