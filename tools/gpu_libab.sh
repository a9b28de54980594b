#!/bin/bash
# Library A/B: optional GPU test subset on the in-tree library, then the
# headline bench alternating library builds (LIBS="ab_libs/lib_base.so;"
# -- ';'-separated DG_LIB_PATH values, empty = the in-tree build), REPS rounds.
#   OUT=gpurun_out/x LIBS="ab_libs/lib_base.so;" FILES="tests/test_gpu_parity.py" tools/gpu_libab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/libab}
LIBS=${LIBS:-ab_libs/lib_base.so;}
REPS=${REPS:-2}
STEPS=${STEPS:-20}
EXTRA=${EXTRA:-}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
if [ "${TESTS:-1}" = 1 ]; then
  KARG=()
  [ -n "${K:-}" ] && KARG=(-k "$K")
  timeout -k 10 ${TLIM:-900} python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "${KARG[@]}" \
    ${FILES:-tests} > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
IFS=';' read -ra LS <<< "$LIBS"
[ "${LIBS: -1}" = ";" ] && LS+=("")
for r in $(seq 1 $REPS); do
  for k in "${!LS[@]}"; do
    lib=${LS[$k]}; tag=lib${k}_$r
    DG_LIB_PATH=$lib timeout -k 10 400 python bench.py --steps $STEPS --warmup 3 --e2e-steps 0 --one-threads 0 \
      --no-cpu-baseline $EXTRA --out $OUT/$tag.json > $OUT/$tag.log 2>&1
    rc=$?; echo "=== $tag [${lib:-in-tree}] exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/$tag.log; exit $rc; }
    python -c "import json;d=json.load(open('$OUT/$tag.json'));s=d['roofline_isolated']['stages_ms'];print(d['value'],d['ms_per_step'],{k:round(v,3) for k,v in s.items() if v>0.05})"
  done
done
