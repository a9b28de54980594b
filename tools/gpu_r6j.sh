#!/bin/bash
# round 6: PNG suite (dword run fills), configs[4] kernel trace (mask inflate max), entry capacity under 32 GB
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6j}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_png.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/tests.log | head; exit $rc; }
OUT=$OUT/wl WL=png ARGS="--steps 10 --warmup 2 --windows 3" tools/gpu_wl.sh || exit $?
OUT=$OUT TESTS=0 REPS=1 STEPS=10 EXTRA="--workload png --windows 3" \
  AB="inf_cap=10;--max-device-mb=32000 inf_cap=10;--max-device-mb=32000 inf_cap=20" tools/gpu_ab2.sh
for f in $OUT/*.json; do python -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['stats'].get('png_serial_fallbacks'),d['allocations']['peak_device_mb'],d['allocations'].get('budget_slots'))"; done
