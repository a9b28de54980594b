#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/split7
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT CHAINS=100 timeout -k 10 300 python -u tools/probe/prog_scan_probe.py > $OUT/probe.log 2>&1 || exit $?
awk '{print $1, $5, $6, $7, $9, ($13-$12)/100000 " ms"}' $OUT/dump_largest_c100.txt
PBS="${PBS:-2048}" bash tools/gpu_split3.sh || exit $?
PB=2048 bash tools/gpu_split4.sh || exit $?
python - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/split4/trace/run_kernel_trace.csv')))
t0=min(int(r['Start_Timestamp']) for r in rows)
for r in rows:
    if 'prog_scan<1>' in r['Kernel_Name']:
        print(' q',r['Queue_Id'],'grid',int(r['Grid_Size_X'])//64, 'start %.0f'%((int(r['Start_Timestamp'])-t0)/1e6), 'dur %.0f ms'%((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6))
PY
