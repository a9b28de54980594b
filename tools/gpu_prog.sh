#!/bin/bash
# Progressive-JPEG throughput: 100%-progressive pool at 2 and 4 batches in flight
# (and $EXTRA), CPU oracle baseline in the first run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prog
i=0
for cfg in "--inflight 2" "--inflight 4 --no-cpu-baseline" ${EXTRA_CFG:-}; do
  i=$((i + 1))
  echo "=== $cfg"
  timeout -k 10 400 python bench.py --progressive-frac 1.0 --pool ${POOL:-256} --steps ${STEPS:-3} --warmup 1 \
      --e2e-steps 0 --one-threads 0 --cpu-seconds 6 $cfg --out gpurun_out/prog/b_$i.json > gpurun_out/prog/b_$i.log 2>&1
  rc=$?; echo "exit $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/prog/b_$i.json'));print(d['value'],d['ms_per_step'],(d.get('cpu_baseline') or {}).get('value'),{k:round(v,1) for k,v in d['roofline_isolated']['stages_ms'].items() if v>0.5})"
done
