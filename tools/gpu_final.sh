#!/bin/bash
# Round-end evidence at HEAD, in parts (one gpurun call each):
#   PART=tests  the -m gpu suite + smoke, then the default bench line and a
#               rocprof kernel trace of the headline
#   PART=pmc    hardware-counter passes (tools/gpu_pmc.sh) + both decode semantics
#   PART=wl     configs[2] / configs[4] lines with kernel traces, the rank rehearsal
# OUT=gpurun_out/final/<part>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
PART=${PART:-tests}
OUT=${OUT:-gpurun_out/final}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
case $PART in
tests)
  OUT=$OUT/tests tools/gpu_tests.sh || exit $?
  timeout -k 10 500 python bench.py --out $OUT/bench.json > $OUT/bench.log 2>&1
  rc=$?; echo "=== bench exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench.log; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['cpu_baseline']['value'],(d.get('e2e_decode_one') or {}).get('mpix_s'),d.get('e2e_host_mpix_s'))"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 3 \
    --e2e-steps 0 --one-threads 0 --no-cpu-baseline --out $OUT/prof_bench.json > $OUT/prof.log 2>&1
  rc=$?; echo "=== rocprof exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/prof.log; exit $rc; }
  db=$(find $OUT/prof -name '*.db' | head -1)
  [ -n "$db" ] && python tools/rocpd_stats.py "$db" > $OUT/kernel_stats.csv && head -16 $OUT/kernel_stats.csv
  find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/rocprof_kernel_stats.csv \;
  ;;
pmc)
  OUT=$OUT/pmc tools/gpu_pmc.sh || exit $?
  OUT=$OUT/modes PROF=0 tools/gpu_modes.sh || exit $?
  ;;
wl)
  OUT=$OUT/wds WL=wds tools/gpu_wl.sh || exit $?
  OUT=$OUT/png WL=png ARGS="--steps 10 --warmup 2" tools/gpu_wl.sh || exit $?
  OUT=$OUT/ranks tools/gpu_ranks.sh || exit $?
  ;;
esac
exit 0
