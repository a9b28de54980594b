#!/bin/bash
# configs[4] PNG investigation: the PNG tests, the bench line over inflate-decode
# variants (VARIANTS: inf_decode values), a rocprof kernel trace (per-kernel spans,
# timeline) and SQ counter passes per kernel (one batch in flight).  OUT=gpurun_out/png
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/png}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_png.py > $OUT/tests.log 2>&1
  rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/tests.log | head -20; exit $rc; }
fi
A="--workload png --steps 10 --warmup 2 --windows ${WINDOWS:-3} --e2e-steps 0 --one-threads 0 --no-cpu-baseline"
for v in ${VARIANTS:-2 8 9}; do
  timeout -k 10 400 python bench.py $A --ctx-opt inf_decode=$v ${EXTRA:-} --out $OUT/bench_$v.json > $OUT/bench_$v.log 2>&1 || { tail -20 $OUT/bench_$v.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('inf_decode $v', d['value'],d['ms_per_step'],d['windows']['mpix_s']);s=d['roofline_isolated']['stages_ms'];print({k:round(v,3) for k,v in s.items() if v>0.02})"
done
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py $A --windows 1 ${PROF_EXTRA:-} --serial-steps 0 --out $OUT/prof_bench.json > $OUT/prof.log 2>&1
  rc=$?; echo "=== rocprof exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/prof.log; exit $rc; }
  db=$(find $OUT/prof -name '*.db' | head -1)
  [ -n "$db" ] && python tools/rocpd_stats.py "$db" > $OUT/kernel_stats.csv && head -16 $OUT/kernel_stats.csv
  [ -n "$db" ] && python tools/trace_window.py "$db" --last-s 0 > $OUT/timeline.txt 2>&1; head -30 $OUT/timeline.txt
fi
if [ "${PMC:-1}" = 1 ]; then
  P="--workload png --steps 2 --warmup 1 --windows 1 --inflight 1 --serial-steps 0 --e2e-steps 0 --one-threads 0 --no-cpu-baseline ${PROF_EXTRA:-}"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/pmc/sq -o run -- python3 bench.py $P > $OUT/pmc_sq.log 2>&1
  rc=$?; echo "=== pmc sq exit $rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $OUT/pmc/sq2 -o run -- python3 bench.py $P > $OUT/pmc_sq2.log 2>&1
  rc=$?; echo "=== pmc sq2 exit $rc"; [ $rc -eq 0 ] || exit $rc
  python tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.txt; head -60 $OUT/pmc_summary.txt
fi
