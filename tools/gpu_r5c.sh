set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r5c
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
DG_SEGV_TRACE=1 timeout -k 10 600 python -u -m pytest -x -v -s -p no:faulthandler --timeout 120 --timeout-method thread -m gpu ${FILES:-tests/test_gpu_coef_cache.py tests/test_gpu_budget.py tests/test_gpu_exit.py tests/test_gpu_parity.py} > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -B2 -A30 "native stack" $OUT/tests.log | head -60; grep -E "FAIL|Error" $OUT/tests.log | head -20; exit $rc; }
