#!/bin/bash
# round 6: budget probe, sync2 parity, budget suite, headline A/B (sync2, sparse_coef), dg_decode_one legs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6d}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
timeout -k 10 120 python tools/probe/budget_dbg.py > $OUT/budget_dbg.txt 2>&1; rc=$?; cat $OUT/budget_dbg.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread "tests/test_gpu_parity.py::test_sync2_bit_exact" tests/test_gpu_budget.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc $rc"; grep -E "PASS|FAIL" $OUT/tests.log | tail -20; [ $rc -le 1 ] || exit $rc
OUT=$OUT/ab TESTS=0 REPS=2 AB="sync2=1;sparse_coef=0;sync2=1 sparse_coef=0" tools/gpu_ab2.sh || exit $?
for r in 1 2; do
  for v in base:"" s2:"--ctx-opt sync2=1"; do
    tag=${v%%:*}; args=${v#*:}
    timeout -k 10 400 python bench.py --steps 5 --windows 1 --warmup 2 --e2e-steps 0 --no-cpu-baseline --serial-steps 0 \
      --one-threads 32 $args --out $OUT/one_${tag}_$r.json > $OUT/one_${tag}_$r.log 2>&1
    rc=$?; echo "=== one $tag $r exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/one_${tag}_$r.log; exit $rc; }
    python -c "import json;d=json.load(open('$OUT/one_${tag}_$r.json'));o=d['e2e_decode_one'];print(o['mpix_s'],o.get('mean_images_per_batch'),(o.get('native_threads') or {}).get('mpix_s'))"
  done
done
