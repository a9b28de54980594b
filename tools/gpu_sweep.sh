#!/bin/bash
# Parameter sweep for bench.py: SWEEP="sub_bits:batch:lead ..." (lead -1 =
# library default).  Each run under its own timeout; stop on crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sweep
mkdir -p $OUT
for cfg in ${SWEEP:-2048:256:-1 4096:256:-1}; do
  IFS=: read -r sb bt ld <<< "$cfg"
  ld=${ld:--1}
  tag=${sb}_${bt}_${ld}
  echo "=== sub_bits=$sb batch=$bt lead=$ld"
  timeout -k 10 300 python bench.py --steps ${STEPS:-8} --warmup 2 --batch $bt --pool ${POOL:-256} --sub-bits $sb \
      --lead-bits $ld ${EXTRA:-} --no-cpu-baseline --e2e-steps 0 --out $OUT/b_$tag.json > $OUT/b_$tag.log 2>&1
  rc=$?
  echo "exit $rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/b_$tag.json'));s=d['stages_ms_per_step'];print(d['value'],d['ms_per_step'],{k:s[k] for k in ('huff_sync','huff_fix','huff_write')},d['stats'],d.get('wg_timing_us'))"
done
