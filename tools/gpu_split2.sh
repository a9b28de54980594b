#!/bin/bash
# Progressive split: which hardware-queue arrangement keeps the baseline slots clear (option prog_queue).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/split2
mkdir -p $OUT
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
for q in ${QS:-3 1 2 0}; do
  timeout -k 10 400 python bench.py --progressive-frac 0.1 --pool 4096 --steps ${MIX_STEPS:-80} --warmup 8 $B \
      --ctx-opt prog_queue=$q $EXTRA --out $OUT/mix10_q$q.json > $OUT/mix10_q$q.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/mix10_q$q.json'));print('mix10 q$q',d['value'],d['ms_per_step'],d['stages_ms_per_step']['resize_h1'],d['stages_ms_per_step']['prog_scans'])"
done
