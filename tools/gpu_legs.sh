#!/bin/bash
# The secondary workloads at HEAD, one bench line each (reported, not the
# headline): progressive mixes, JPEG and PNG re-encode.  OUT=gpurun_out/legs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/legs}
mkdir -p $OUT
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline"
run() {  # name args...
  local name=$1; shift
  timeout -k 10 500 python bench.py $B "$@" --out $OUT/$name.json > $OUT/$name.log 2>&1
  local rc=$?; echo "=== $name [$*] exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/$name.log; return $rc; }
  python -c "import json;d=json.load(open('$OUT/$name.json'));print(d['value'],d['ms_per_step'])"
}
run prog10 --progressive-frac 0.1 --steps 100 --warmup 5 &&
run prog100 --progressive-frac 1.0 --steps 20 --warmup 3 &&
run jpeg_enc --encode --steps 10 --warmup 2 &&
run png_enc --workload png --encode --steps 10 --warmup 2
