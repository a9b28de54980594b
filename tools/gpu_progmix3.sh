#!/bin/bash
# 10%-progressive pool through dg_decode_one (32 threads): lanes / side-stream A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mix3
mkdir -p $OUT
i=0
for cfg in "--prog-lanes 1 --ctx-opt prog_side=1" "--prog-lanes 1 --ctx-opt prog_side=0" "--prog-lanes 2 --ctx-opt prog_side=0" "--prog-lanes 0 --ctx-opt prog_side=1"; do
  i=$((i + 1))
  timeout -k 10 400 python bench.py --progressive-frac 0.1 --pool 1024 --steps 2 --warmup 1 --e2e-steps 0 \
      --one-threads 32 --one-images 2048 --no-cpu-baseline $cfg --out $OUT/m_$i.json > $OUT/m_$i.log 2>&1
  rc=$?; echo "=== $cfg exit $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/m_$i.json'));o=d.get('e2e_decode_one');print(d['value'],o['mpix_s'],o['gpu_batches'],o['mean_images_per_batch'])"
done
