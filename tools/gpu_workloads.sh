#!/bin/bash
# The non-headline bench lines: configs[2] (WDS), configs[4] (PNG pairs, with
# and without re-encode), configs[3] (cfg4: 1M samples over a 16,384 pool,
# sharded, here 2 ranks on one GPU) and the default workload at --gpus 2.
# Each under its own timeout; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/wl
mkdir -p $OUT
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$to" python bench.py "$@" --out $OUT/$name.json > $OUT/$name.log 2>&1
  local rc=$?
  echo "exit $rc"; tail -c 400 $OUT/$name.json 2>/dev/null; echo
  return $rc
}
run wds 300 --workload wds --steps 8 --warmup 2 &&
run png 400 --workload png --steps 10 --warmup 2 &&
run png_encode 400 --workload png --encode --steps 10 --warmup 2 &&
run cfg4_gpus2 500 --workload cfg4 --gpus 2 --steps 5 --warmup 1 --e2e-steps 0 --one-threads 0 &&
run jpeg_gpus2 400 --gpus 2 --steps 10 --warmup 2 --e2e-steps 0 --one-threads 0
