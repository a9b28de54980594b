#!/bin/bash
# PNG write-combining (tests + A/B vs the HEAD kernel) and progressive aggregate knobs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/combo
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_fuzz.py tests/test_gpu_samples.py -q -x --timeout 200 --timeout-method thread > $OUT/pytest_png.log 2>&1
rc=$?; tail -2 $OUT/pytest_png.log; [ $rc -eq 0 ] || exit $rc
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 1"
for i in 1 2; do for v in head new; do
  lib=""; [ $v = head ] && lib=datago_amd/_exp/png_head.so
  DG_LIB_PATH=$lib timeout -k 10 400 python bench.py --workload png --steps 6 --warmup 2 $B --out $OUT/png_${v}_$i.json > $OUT/png_${v}_$i.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/png_${v}_$i.json'));print('png $v',d['value'],d['ms_per_step'],d.get('roofline_isolated',{}).get('stages_ms'))"
done; done
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
run() {  # name lib opts...
  local name=$1 lib=$2; shift 2
  DG_LIB_PATH=$lib timeout -k 10 400 python bench.py --progressive-frac 0.1 --pool 4096 --steps 200 --warmup 8 $B "$@" --out $OUT/mix_$name.json > $OUT/mix_$name.log 2>&1 || return $?
  DG_LIB_PATH=$lib timeout -k 10 400 python bench.py --progressive-frac 1.0 --pool 2048 --steps 24 --warmup 8 $B "$@" --out $OUT/p100_$name.json > $OUT/p100_$name.log 2>&1 || return $?
  python -c "import json;a=json.load(open('$OUT/mix_$name.json'));b=json.load(open('$OUT/p100_$name.json'));print('$name mix10',a['value'],'p100',b['value'])"
}
run base "" || exit $?
run pb4096 "" --ctx-opt prog_batch=4096 || exit $?
run cus128 "" --ctx-opt prog_cus=128 --ctx-opt prog_queue=3 || exit $?
run ps3 datago_amd/_exp/ps3.so || exit $?
