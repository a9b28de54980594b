#!/bin/bash
# Headline bench at 2/3/4 batches in flight, with and without the side stream.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/inflight
mkdir -p $OUT
i=0
for cfg in ${CFGS:-"--inflight 2" "--inflight 3" "--inflight 4" "--inflight 3 --ctx-opt side_stream=0" "--inflight 4 --ctx-opt side_stream=0" "--inflight 2 --ctx-opt side_stream=0" "--inflight 2"}; do
  i=$((i + 1))
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e-steps 0 --one-threads 0 --no-cpu-baseline $cfg --out $OUT/b_$i.json > $OUT/b_$i.log 2>&1
  rc=$?; echo "=== [$cfg] exit $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/b_$i.json'));print(d['value'],d['ms_per_step'])"
done
