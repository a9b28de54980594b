#!/bin/bash
# round 6: PNG suite with the entries aliased (png_alias), then configs[4] under a 32 GB budget
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6i}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_png.py \
  tests/test_gpu_samples.py tests/test_gpu_budget.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/tests.log | head; exit $rc; }
OUT=$OUT TESTS=0 REPS=1 STEPS=10 EXTRA="--workload png --windows 3" \
  AB="png_alias=0;--max-device-mb=32000;--max-device-mb=32000 inf_cap=15 inf_pad=16384;inf_cap=15 inf_pad=16384" tools/gpu_ab2.sh
for f in $OUT/*.json; do python -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['stats'].get('png_serial_fallbacks'),d['stats'].get('png_chunks'),d['allocations']['peak_device_mb'],d['allocations'].get('budget_slots'))"; done
