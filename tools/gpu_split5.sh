#!/bin/bash
# Do the two progressive slots overlap? Kernel trace of a 100%-progressive run per prog_queue mode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/split5
mkdir -p $OUT
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
timeout -k 10 400 python bench.py --progressive-frac 1.0 --pool 2048 --steps 2 --warmup 1 $B --out $OUT/gen.json > $OUT/gen.log 2>&1 || exit $?
for q in 3 1; do
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_q$q -o run -- python3 bench.py --progressive-frac 1.0 --pool 2048 --steps 16 --warmup 4 $B --ctx-opt prog_queue=$q --out $OUT/p100_q$q.json > $OUT/p100_q$q.log 2>&1 || exit $?
python -c "import json;d=json.load(open('$OUT/p100_q$q.json'));print('p100 q$q',d['value'],d['ms_per_step'])"
done
