#!/bin/bash
# configs[4] unfilter worker caps (uf_per_cu / uf_units: the unfilter's LDS no
# longer fills every CU while other batches wait) and configs[1] entropy wave
# priority (entropy_prio).  OUT=gpurun_out/r5m
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5m}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
A="--workload png --steps 10 --warmup 2 --windows 3 --e2e-steps 0 --one-threads 0 --no-cpu-baseline"
k=0
for o in "" "uf_per_cu=1" "uf_units=1" "uf_units=1,uf_per_cu=2"; do
  k=$((k+1))
  timeout -k 10 400 python bench.py $A $(echo $o | tr ',' '\n' | sed '/^$/d; s/^/--ctx-opt /') --out $OUT/png_$k.json > $OUT/png_$k.log 2>&1 || { tail -20 $OUT/png_$k.log; exit 1; }
  python -c "import json;d=json.load(open('$OUT/png_$k.json'));print('png [$o]', d['value'],d['windows']['mpix_s'],d['roofline_isolated']['stages_ms']['png_unfilter'])"
done
OUT=$OUT/jpeg AB="entropy_prio=1;entropy_prio=2" REPS=2 TESTS=0 tools/gpu_ab2.sh || exit $?
