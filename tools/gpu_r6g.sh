#!/bin/bash
# round 6: budget suite + inf_cap parity, then configs[4] under device budgets x chunk entry capacities
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6g}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_budget.py \
  "tests/test_gpu_png.py::test_chunk_entry_capacity_bit_exact" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc $rc"; grep -E "PASS|FAIL" $OUT/tests.log | tail -12; [ $rc -le 1 ] || exit $rc
OUT=$OUT TESTS=0 REPS=1 STEPS=10 EXTRA="--workload png --windows 3" \
  AB="inf_cap=20;inf_cap=15;--max-device-mb=32000 inf_cap=15;--max-device-mb=32000 inf_cap=12;--max-device-mb=40000 inf_cap=15" tools/gpu_ab2.sh
