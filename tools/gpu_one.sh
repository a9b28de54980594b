#!/bin/bash
# dg_decode_one from many host threads: batch fill and throughput vs callers (steady state, 4096 images).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/one
mkdir -p $OUT
B="--steps 2 --warmup 1 --e2e-steps 0 --no-cpu-baseline --serial-steps 0 --one-images 4096"
for t in 32 64 128; do for opt in "" "--ctx-opt coalesce_us=2000"; do
  name=t${t}${opt:+_us2000}
  timeout -k 10 400 python bench.py $B --one-threads $t $opt --out $OUT/$name.json > $OUT/$name.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/$name.json'));o=d['e2e_decode_one'];print('$name',o['mpix_s'],o['images_per_s'],o['mean_images_per_batch'])"
done; done
