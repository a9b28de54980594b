#!/bin/bash
# configs[3] rehearsal: 8 ranks sharing one GPU at the default 4 slots under a
# per-rank device budget (max_device_mb): no OOM, peak
# footprint per rank in the line.  OUT=gpurun_out/ranks5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/ranks5}
mkdir -p $OUT
for v in ${RUNS:-"b30:--max-device-mb 30000" "b30sq:--max-device-mb 30000 --ctx-opt side_queue=-1"}; do
  name=${v%%:*}; args=$(echo ${v#*:} | tr "," " ")
  timeout -k 10 700 python bench.py --gpus 8 --workload cfg4 --steps ${STEPS:-6} --warmup ${WARMUP:-2} --windows 1 --e2e-steps 0 --one-threads 0 --no-cpu-baseline $args --out $OUT/g8_$name.json > $OUT/g8_$name.log 2>&1 || { tail -20 $OUT/g8_$name.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/g8_$name.json'));a=d.get('allocations',{});print('gpus 8 cfg4 $name',d['value'],{k:a.get(k) for k in ('peak_device_mb','max_device_mb','budget_slots','budget_splits','budget_frees','budget_oom')})"
done
