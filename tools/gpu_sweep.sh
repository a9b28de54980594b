#!/bin/bash
# Parameter sweep for bench.py.  SWEEP is a comma-separated list of bench
# argument strings, e.g. SWEEP="--hb-bands 2,--hb-bands 8 --inflight 3".
# Each run under its own timeout; stop on crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sweep
mkdir -p $OUT
IFS=, read -r -a CFGS <<< "${SWEEP:---sub-bits 2048,--sub-bits 4096}"
i=0
for cfg in "${CFGS[@]}"; do
  i=$((i + 1))
  echo "=== [$i] $cfg"
  # shellcheck disable=SC2086
  timeout -k 10 300 python bench.py --steps ${STEPS:-8} --warmup 2 --pool ${POOL:-256} $cfg ${EXTRA:-} \
      --no-cpu-baseline --e2e-steps 0 --serial-steps 1 --out $OUT/b_$i.json > $OUT/b_$i.log 2>&1
  rc=$?
  echo "exit $rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/b_$i.json'));s=d['stages_ms_per_step'];iso=(d.get('roofline_isolated') or {}).get('stages_ms') or {};print(d['value'],d['ms_per_step'],{k:round(v,3) for k,v in iso.items() if v>0.05})"
done
