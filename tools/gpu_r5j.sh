#!/bin/bash
# configs[4] PNG with more batches in flight, configs[2] WDS with/without the
# Lanczos table cache, dg_decode_one with 4 coalesced batches.  OUT=gpurun_out/r5j
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5j}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
A="--workload png --steps 10 --warmup 6 --windows 3 --e2e-steps 0 --one-threads 0 --no-cpu-baseline"
for v in ${PNG_INFLIGHT:-4 6}; do
  timeout -k 10 400 python bench.py $A --inflight $v --out $OUT/png_i$v.json > $OUT/png_i$v.log 2>&1 || { tail -20 $OUT/png_i$v.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/png_i$v.json'));print('png inflight $v', d['value'],d['ms_per_step'],d['windows']['mpix_s'],d['allocations']['peak_device_mb'])"
done
W="--workload wds --steps 20 --warmup 4 --windows 3 --e2e-steps 0 --one-threads 0 --no-cpu-baseline"
for r in 1 2; do
  for o in "" "--ctx-opt coef_cache_mb=0"; do
    tag=wds_${r}$( [ -n "$o" ] && echo _nocache )
    timeout -k 10 400 python bench.py $W $o --out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -20 $OUT/$tag.log; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag', d['value'],d['ms_per_step'],d['windows']['mpix_s'],{k:d['stats'].get(k) for k in ('sub_bits',)})"
  done
done
OUT=$OUT/one ONE_IMAGES=2048 THREADS=32 OPTS=";coalesce_inflight=4" tools/gpu_one.sh || exit $?
