#!/bin/bash
# slot_queue 1 by default: GPU tests, JPEG headline, PNG pairs, progressive pools.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
timeout -k 10 400 python bench.py --steps 20 --warmup 2 $B --out $OUT/jpeg.json > $OUT/jpeg.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload png --steps 8 --warmup 2 $B --out $OUT/png.json > $OUT/png.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload png --encode --steps 8 --warmup 2 $B --out $OUT/png_enc.json > $OUT/png_enc.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --progressive-frac 0.1 --pool 4096 --steps 600 --warmup 8 $B --out $OUT/mix.json > $OUT/mix.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --progressive-frac 1.0 --pool 2048 --steps 24 --warmup 8 $B --out $OUT/p100.json > $OUT/p100.log 2>&1 || exit $?
for f in jpeg png png_enc mix p100; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',d['value'],d['ms_per_step'])"; done
