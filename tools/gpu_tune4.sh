#!/bin/bash
# Re-tune under 4 slots on their own queues: band H rows per workgroup and entropy subsequence size.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/tune4
mkdir -p $OUT
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
for r in 1 2; do
for v in "hb16:--hb-bands 16" "hb24:--hb-bands 24" "hb12:--hb-bands 12" "sb4096:--sub-bits 4096" "wp2:--ctx-opt write_pair=2"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 400 python bench.py --steps 20 --warmup 2 $B $args --out $OUT/${name}_$r.json > $OUT/${name}_$r.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/${name}_$r.json'));print('$name run $r',d['value'],d['ms_per_step'])"
done; done
