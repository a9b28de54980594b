#!/bin/bash
# Round-3 end: full GPU suite and smoke at HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final3
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
