#!/bin/bash
# GPU test suite (optionally a subset: K='expr' or FILES='tests/x.py ...'),
# then smoke.  OUT=gpurun_out/<name>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/tests}
mkdir -p $OUT
FILES=${FILES:-tests}
KARG=()
[ -n "${K:-}" ] && KARG=(-k "$K")
timeout -k 10 ${TLIM:-900} python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "${KARG[@]}" $FILES \
  > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
if [ "${SMOKE:-1}" = 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
