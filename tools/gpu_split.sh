#!/bin/bash
# Progressive split: GPU tests, headline bench, 100% / 10% progressive pools through dg_submit_device.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/split
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 1"
timeout -k 10 500 python bench.py --steps 20 --warmup 2 $B --out $OUT/head.json > $OUT/head.log 2>&1 || exit $?
python -c "import json;d=json.load(open('$OUT/head.json'));print('headline',d['value'],d['ms_per_step'])"
timeout -k 10 600 python bench.py --progressive-frac 1.0 --pool 1024 --steps ${P100_STEPS:-16} --warmup 4 $B --out $OUT/p100.json > $OUT/p100.log 2>&1 || exit $?
python -c "import json;d=json.load(open('$OUT/p100.json'));print('p100',d['value'],d['ms_per_step'],d['stages_ms_per_step'].get('prog_scans'))"
timeout -k 10 600 python bench.py --progressive-frac 0.1 --pool 4096 --steps ${MIX_STEPS:-120} --warmup 8 $B --out $OUT/mix10.json > $OUT/mix10.log 2>&1 || exit $?
python -c "import json;d=json.load(open('$OUT/mix10.json'));print('mix10',d['value'],d['ms_per_step'])"
