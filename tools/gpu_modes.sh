#!/bin/bash
# Headline bench in both decode semantics, alternating (A B A B), then a
# rocprof kernel trace of the zune-mode headline.
#   OUT=gpurun_out/modes EXTRA="--ctx-opt x=1" tools/gpu_modes.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/modes}
EXTRA=${EXTRA:-}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
i=0
for sem in 0 1 0 1; do
  i=$((i + 1))
  timeout -k 10 400 python bench.py --steps 20 --warmup 3 --e2e-steps 0 --one-threads 0 --no-cpu-baseline \
    --decode-semantics $sem $EXTRA --out $OUT/b_${i}_sem$sem.json > $OUT/b_${i}_sem$sem.log 2>&1
  rc=$?; echo "=== sem $sem exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/b_${i}_sem$sem.log; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/b_${i}_sem$sem.json'));s=d['roofline_isolated']['stages_ms'];print(d['value'],d['ms_per_step'],{k:round(v,3) for k,v in s.items() if v>0.05})"
done
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 3 \
    --e2e-steps 0 --one-threads 0 --no-cpu-baseline --decode-semantics 1 $EXTRA --out $OUT/prof_bench.json > $OUT/prof.log 2>&1
  rc=$?; echo "=== rocprof exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/prof.log; exit $rc; }
  find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
  head -25 $OUT/kernel_stats.csv | cut -c1-200
fi
