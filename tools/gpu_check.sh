#!/bin/bash
# One GPU-box session: build check, GPU parity tests, short bench, rocprof.
# Each GPU step runs under its own timeout; a crash/timeout stops the script
# (test assertion failures, exit 1, do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-10}
BARGS=${BARGS:-}
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name exit $rc" | tee -a $OUT/steps.log
  tail -5 $OUT/$name.log
  return $rc
}
ok_or_fail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
python -c "import datago_amd._lib as L; L.load(); print('lib ok')" > $OUT/libload.log 2>&1 || { cat $OUT/libload.log; exit 3; }
step pytest_gpu 900 python -u -m pytest tests -q -m gpu -rf --maxfail=40 --timeout 300 --timeout-method thread
rc=$?; ok_or_fail $rc || exit $rc
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
rc=$?; ok_or_fail $rc || exit $rc
step bench 900 python bench.py --steps $STEPS --warmup 2 $BARGS --out $OUT/bench.json
rc=$?; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 1 $BARGS --no-cpu-baseline --e2e-steps 0 --one-threads 0
exit $?
