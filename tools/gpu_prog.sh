#!/bin/bash
# Progressive-mix lines in round 3's configurations (profiles/r03/mixlong,
# profiles/r03/prog): 10% progressive over 200 / 600 steps, 100% progressive
# at 1,024 images per batch.  OUT=gpurun_out/prog
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/prog}
mkdir -p $OUT
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
run() {  # name args...
  local name=$1; shift
  timeout -k 10 500 python bench.py $B "$@" --out $OUT/$name.json > $OUT/$name.log 2>&1
  local rc=$?; echo "=== $name [$*] exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/$name.log; return $rc; }
  python -c "import json;d=json.load(open('$OUT/$name.json'));print(d['value'],d['ms_per_step'])"
}
run mix_s200 --progressive-frac 0.1 --steps 200 --warmup 8 &&
run mix_s600 --progressive-frac 0.1 --steps 600 --warmup 8 &&
run p100_b1024 --progressive-frac 1.0 --batch 1024 --steps 3 --warmup 1
