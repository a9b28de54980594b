#!/bin/bash
# Per-dispatch k_prog_scan durations (one launch per level) for tools/prog_probe.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/progprof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/progprof -o run -- python3 tools/prog_probe.py > gpurun_out/progprof/probe.log 2>&1
rc=$?; cat gpurun_out/progprof/probe.log; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/progprof -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'prog_scan' in r['Kernel_Name']]
for r in rows:
    print(r['Grid_Size'] if 'Grid_Size' in r else r.get('Grid_Size_X'), (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6, 'ms')
PY
