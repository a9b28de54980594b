#!/bin/bash
# Parameter sweep for bench.py (each run under its own timeout; stop on crash).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sweep
mkdir -p $OUT
for cfg in ${SWEEP:-1024:64 2048:64 4096:64 2048:256}; do
  sb=${cfg%%:*}; bt=${cfg##*:}
  echo "=== sub_bits=$sb batch=$bt"
  timeout -k 10 300 python bench.py --steps ${STEPS:-8} --warmup 2 --batch $bt --pool ${POOL:-256} --sub-bits $sb \
      --no-cpu-baseline --e2e-steps 0 --out $OUT/b_${sb}_${bt}.json > $OUT/b_${sb}_${bt}.log 2>&1
  rc=$?
  echo "exit $rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/b_${sb}_${bt}.json'));print(d['value'],d['ms_per_step'],d['stages_ms_per_step'],d['stats'])"
done
