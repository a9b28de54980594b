#!/bin/bash
# dg_decode_one from host threads: batch fill and throughput vs coalescing
# options (steady state over ONE_IMAGES images).  OPTS: ';'-separated
# context-option sets; THREADS: caller thread counts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/one}
mkdir -p $OUT
B="--steps 2 --warmup 1 --e2e-steps 0 --no-cpu-baseline --serial-steps 0 --one-images ${ONE_IMAGES:-4096}"
IFS=';' read -ra OS <<< "${OPTS:-;coalesce_inflight=2;coalesce_inflight=3}"
for t in ${THREADS:-32}; do
  k=0
  for o in "${OS[@]}"; do
    k=$((k + 1))
    cfg=""; for x in $o; do cfg="$cfg --ctx-opt $x"; done
    name=t${t}_$k
    timeout -k 10 400 python bench.py $B ${ONE_EXTRA:-} --one-threads $t $cfg --out $OUT/$name.json > $OUT/$name.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('$OUT/$name.json'));o=d['e2e_decode_one'];print('$name [$o]',o['mpix_s'],o['images_per_s'],o['mean_images_per_batch'],'native',o.get('native_threads'))"
  done
done
