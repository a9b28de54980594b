#!/bin/bash
# The N>1 launcher: 2 and 8 ranks sharing the one GPU (configs[1] / configs[3]),
# with each rank's host submit phases (wall and thread CPU ms per step).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/ranks}
mkdir -p $OUT
show() {
  python -c "
import json;d=json.load(open('$1'))
print('$2', d['value'], d['n_gpus'], d['ms_per_step_per_rank'], d.get('rank_cpus'))
for r, ph in enumerate(d.get('host_submit_phases_per_rank') or []):
    print('  rank', r, 'wall', ph['wall'], 'cpu', ph['cpu'])"
}
timeout -k 10 500 python bench.py --gpus 2 --steps 10 --warmup 2 --e2e-steps 0 --one-threads 0 --no-cpu-baseline \
  ${EXTRA:-} --out $OUT/g2.json > $OUT/g2.log 2>&1 || exit $?
show $OUT/g2.json "gpus 2"
# 8 ranks share this one device: 2 batches in flight each (8 x 4 slots of
# configs[3] buffers with growth headroom exceed its 288 GB; on the 8-GPU node
# each rank owns a device)
timeout -k 10 700 python bench.py --gpus 8 --workload cfg4 --steps 6 --warmup 2 --e2e-steps 0 --one-threads 0 \
  --inflight ${G8_INFLIGHT:-2} --no-cpu-baseline ${EXTRA:-} --out $OUT/g8.json > $OUT/g8.log 2>&1 || exit $?
show $OUT/g8.json "gpus 8 cfg4"
