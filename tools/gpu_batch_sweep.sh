#!/bin/bash
# headline vs images per step / batches in flight (SWEEP: ';'-separated bench argument sets)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/bsweep
mkdir -p $OUT
i=0
IFS=';' read -ra VS <<< "$SWEEP"
for v in "${VS[@]}"; do
  timeout -k 10 400 python bench.py --steps ${STEPS:-20} --warmup 2 --serial-steps 0 --no-cpu-baseline --e2e-steps 0 \
    --one-threads 0 $v --out $OUT/s$i.json > $OUT/s$i.log 2>&1 || { tail -5 $OUT/s$i.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/s$i.json'));print('[$v]','value',d['value'],'ms/step',d['ms_per_step'])"
  i=$((i+1))
done
