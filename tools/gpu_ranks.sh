#!/bin/bash
# The N>1 launcher with the round-3 defaults: 2 and 8 ranks sharing the one GPU (configs[1] / configs[3]).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ranks
mkdir -p $OUT
timeout -k 10 500 python bench.py --gpus 2 --steps 10 --warmup 2 --e2e-steps 0 --one-threads 0 --no-cpu-baseline --out $OUT/g2.json > $OUT/g2.log 2>&1 || exit $?
python -c "import json;d=json.load(open('$OUT/g2.json'));print('gpus 2',d['value'],d['n_gpus'],d['ms_per_step_per_rank'])"
timeout -k 10 700 python bench.py --gpus 8 --workload cfg4 --steps 6 --warmup 2 --e2e-steps 0 --one-threads 0 --no-cpu-baseline --out $OUT/g8.json > $OUT/g8.log 2>&1 || exit $?
python -c "import json;d=json.load(open('$OUT/g8.json'));print('gpus 8 cfg4',d['value'],d['n_gpus'],d['ms_per_step_per_rank'])"
