#!/bin/bash
# One workload's bench line plus a rocprof kernel trace of the same command
# (stats summarised per batch by tools/rocpd_stats.py).
#   OUT=gpurun_out/wds WL=wds ARGS="--steps 20" tools/gpu_wl.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/wl}
WL=${WL:-wds}
ARGS=${ARGS:-"--steps 20 --warmup 3"}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
timeout -k 10 500 python bench.py --workload $WL $ARGS --out $OUT/bench.json > $OUT/bench.log 2>&1
rc=$?; echo "=== bench $WL exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench.log; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['host_submit_ms_per_step'],d.get('host_submit_phases_per_rank'));s=d['roofline_isolated']['stages_ms'];print({k:round(v,3) for k,v in s.items() if v>0.02})"
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --workload $WL $ARGS \
    --no-cpu-baseline --e2e-steps 0 --one-threads 0 --out $OUT/prof_bench.json > $OUT/prof.log 2>&1
  rc=$?; echo "=== rocprof exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/prof.log; exit $rc; }
  db=$(find $OUT/prof -name '*.db' | head -1)
  [ -n "$db" ] && python tools/rocpd_stats.py "$db" > $OUT/kernel_stats.csv && head -30 $OUT/kernel_stats.csv
fi
exit 0
