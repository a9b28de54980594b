#!/bin/bash
# Round-5 check: JPEG + PNG parity (sparse coefficient masks, serial inflate copy
# specialisation), a mask/image split probe under a kernel trace, then the PNG and
# JPEG bench lines over side-stream queue modes (SIDEQ).  OUT=gpurun_out/r5e
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5e}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    ${TESTFILES:-tests/test_gpu_parity.py tests/test_gpu_png.py tests/test_gpu_budget.py tests/test_gpu_coef_cache.py} > $OUT/tests.log 2>&1
  rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/tests.log | head -20; exit $rc; }
fi
if [ "${PROBE:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/probe -o run -- python3 tools/png_probe.py 128 3 > $OUT/probe.log 2>&1
  rc=$?; cat $OUT/probe.log | grep -E "^(masks|images|pairs)"; [ $rc -eq 0 ] || { tail -20 $OUT/probe.log; exit $rc; }
  db=$(find $OUT/probe -name '*.db' | head -1)
  [ -n "$db" ] && python tools/rocpd_stats.py "$db" > $OUT/probe_stats.csv && head -12 $OUT/probe_stats.csv
fi
A="--workload png --steps 10 --warmup 2 --windows 3 --e2e-steps 0 --one-threads 0 --no-cpu-baseline"
for q in ${SIDEQ:--1 3 0}; do
  timeout -k 10 400 python bench.py $A --ctx-opt side_queue=$q --out $OUT/png_sq$q.json > $OUT/png_sq$q.log 2>&1 || { tail -20 $OUT/png_sq$q.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/png_sq$q.json'));print('png side_queue $q', d['value'],d['ms_per_step'],d['windows']['mpix_s'],{k:d['stats'][k] for k in ('png_chunks','png_serial_fallbacks','png_small_streams')})"
done
k=0
for o in ${PNGOPTS:-}; do  # extra PNG lines: comma-separated ctx options each
  k=$((k+1))
  timeout -k 10 400 python bench.py $A $(echo $o | tr ',' '\n' | sed 's/^/--ctx-opt /') --out $OUT/png_o$k.json > $OUT/png_o$k.log 2>&1 || { tail -20 $OUT/png_o$k.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/png_o$k.json'));print('png $o', d['value'],d['ms_per_step'],d['windows']['mpix_s'])"
done
J="--steps 20 --warmup 3 --windows 3 --e2e-steps 0 --one-threads 0 --no-cpu-baseline"
for q in ${JSIDEQ:--1 3}; do
  timeout -k 10 400 python bench.py $J --ctx-opt side_queue=$q --out $OUT/jpeg_sq$q.json > $OUT/jpeg_sq$q.log 2>&1 || { tail -20 $OUT/jpeg_sq$q.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/jpeg_sq$q.json'));print('jpeg side_queue $q', d['value'],d['ms_per_step'],d['windows']['mpix_s'])"
done
