#!/bin/bash
# 100%-progressive pool: batch size x prog_chain (dg_submit, default slots).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prog4
mkdir -p $OUT
for cfg in ${CFGS:-"1024 100" "1024 0" "512 100" "2048 100"}; do
  set -- $cfg
  timeout -k 10 500 python bench.py --progressive-frac 1.0 --pool ${POOL:-2048} --batch $1 --steps 3 --warmup 1 --e2e-steps 0 \
      --one-threads 0 --no-cpu-baseline --serial-steps 1 --ctx-opt prog_chain=$2 --out $OUT/p100_b$1_c$2.json > $OUT/p100_b$1_c$2.log 2>&1
  rc=$?; echo "=== batch $1 chain $2 exit $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/p100_b$1_c$2.json'));print(d['value'],d['ms_per_step'],d['stages_ms_per_step'].get('prog_scans'))"
done
