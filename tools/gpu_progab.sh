#!/bin/bash
# Progressive aggregate knobs: prog_batch 2048 / 4096 and 3 progressive slots (DG_LIB_PATH experiment build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/progab
mkdir -p $OUT
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
run() {  # name lib opts...
  local name=$1 lib=$2; shift 2
  DG_LIB_PATH=$lib timeout -k 10 400 python bench.py --progressive-frac 0.1 --pool 4096 --steps 200 --warmup 8 $B "$@" --out $OUT/mix_$name.json > $OUT/mix_$name.log 2>&1 || return $?
  DG_LIB_PATH=$lib timeout -k 10 400 python bench.py --progressive-frac 1.0 --pool 2048 --steps 24 --warmup 8 $B "$@" --out $OUT/p100_$name.json > $OUT/p100_$name.log 2>&1 || return $?
  python -c "import json;a=json.load(open('$OUT/mix_$name.json'));b=json.load(open('$OUT/p100_$name.json'));print('$name mix10',a['value'],'p100',b['value'])"
}
run base "" || exit $?
run pb4096 "" --ctx-opt prog_batch=4096 || exit $?
run ps3 datago_amd/_exp/ps3.so || exit $?
