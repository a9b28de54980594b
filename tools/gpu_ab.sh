#!/bin/bash
# Full GPU suite, then the headline bench with and without $AB (a context option=value).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab
mkdir -p $OUT
AB=${AB:-multi_lead=0}
python -c "import datago_amd._lib as L; L.load()" || exit 3
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for cfg in "" "--ctx-opt $AB" "" "--ctx-opt $AB"; do
  i=$((i + 1))
  timeout -k 10 400 python bench.py --steps 10 --warmup 2 --e2e-steps 0 --one-threads 0 --no-cpu-baseline $cfg --out $OUT/b_$i.json > $OUT/b_$i.log 2>&1
  rc=$?; echo "=== [$cfg] exit $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/b_$i.json'));s=d['roofline_isolated']['stages_ms'];print(d['value'],d['ms_per_step'],{k:round(v,3) for k,v in s.items() if v>0.05})"
done
