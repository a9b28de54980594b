#!/bin/bash
# PNG chunk-decode variants: the PNG tests, then the images-only probe under a
# kernel trace for each inf_decode variant (isolated launch times), then the
# configs[4] bench line for the best candidates (VARIANTS).  OUT=gpurun_out/r5g
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5g}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_png.py > $OUT/tests.log 2>&1
  rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/tests.log | head -20; exit $rc; }
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/probe -o run -- python3 tools/png_probe.py 128 2 --variants=${PVARS:-2,6,7,8,11,12,14,15} > $OUT/probe.log 2>&1
rc=$?; grep -E "^(masks|images|pairs|img_)" $OUT/probe.log; [ $rc -eq 0 ] || { tail -20 $OUT/probe.log; exit $rc; }
db=$(find $OUT/probe -name '*.db' | head -1)
[ -n "$db" ] && python tools/rocpd_stats.py "$db" > $OUT/probe_stats.csv && grep -E "inf_decode|png_inflate|inf_find" $OUT/probe_stats.csv
A="--workload png --steps 10 --warmup 2 --windows 3 --e2e-steps 0 --one-threads 0 --no-cpu-baseline"
for v in ${VARIANTS:-}; do
  timeout -k 10 400 python bench.py $A --ctx-opt inf_decode=$v --out $OUT/png_v$v.json > $OUT/png_v$v.log 2>&1 || { tail -20 $OUT/png_v$v.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/png_v$v.json'));print('png inf_decode $v', d['value'],d['ms_per_step'],d['windows']['mpix_s'])"
done
