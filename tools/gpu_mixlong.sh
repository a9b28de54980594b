#!/bin/bash
# 10%-progressive mix at steady state: longer runs amortise the last aggregate's tail.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mixlong
mkdir -p $OUT
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
for st in 200 600; do
  timeout -k 10 500 python bench.py --progressive-frac 0.1 --pool 4096 --steps $st --warmup 8 $B --out $OUT/mix_s$st.json > $OUT/mix_s$st.log 2>&1 || exit $?
  python -c "import json;a=json.load(open('$OUT/mix_s$st.json'));print('mix10 steps $st',a['value'],a['ms_per_step'])"
done
timeout -k 10 500 python bench.py --progressive-frac 0.1 --pool 4096 --steps 600 --warmup 8 $B --ctx-opt prog_batch=4096 --out $OUT/mix_s600_pb4096.json > $OUT/mix_s600_pb4096.log 2>&1 || exit $?
python -c "import json;a=json.load(open('$OUT/mix_s600_pb4096.json'));print('mix10 steps 600 pb4096',a['value'],a['ms_per_step'])"
