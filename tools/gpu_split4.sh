#!/bin/bash
# Kernel trace of a 100%-progressive run through the aggregate (dispatch sizes, durations, overlap).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/split4
mkdir -p $OUT
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
timeout -k 10 400 python bench.py --progressive-frac 1.0 --pool 2048 --steps 2 --warmup 1 $B --out $OUT/gen.json > $OUT/gen.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 bench.py --progressive-frac 1.0 --pool 2048 --steps 24 --warmup 8 $B --ctx-opt prog_batch=${PB:-2048} --out $OUT/p100.json > $OUT/p100.log 2>&1 || exit $?
python -c "import json;d=json.load(open('$OUT/p100.json'));print('p100',d['value'],d['ms_per_step'])"
