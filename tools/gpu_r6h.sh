#!/bin/bash
# round 6: PNG chunk entry capacity + padding under a 32 GB budget (configs[4])
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6h}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread \
  "tests/test_gpu_png.py::test_chunk_entry_capacity_bit_exact" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc $rc"; grep -E "PASS|FAIL" $OUT/tests.log | tail -8; [ $rc -le 1 ] || exit $rc
OUT=$OUT TESTS=0 REPS=1 STEPS=10 EXTRA="--workload png --windows 3" \
  AB="inf_cap=15 inf_pad=16384;--max-device-mb=32000 inf_cap=15 inf_pad=16384;--max-device-mb=32000 inf_cap=15 inf_pad=8192;--max-device-mb=32000 inf_cap=12 inf_pad=8192" tools/gpu_ab2.sh
for f in $OUT/*.json; do python -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['stats'].get('png_serial_fallbacks'),d['stats'].get('png_chunks'),d['allocations']['peak_device_mb'],d['allocations'].get('budget_slots'))"; done
