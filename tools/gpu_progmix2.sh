#!/bin/bash
# Progressive tests, then: 100%-progressive pool (dg_submit, 2 in flight) and
# 10%-progressive pool (dg_submit + dg_decode_one from 32 threads, prog_lanes 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mix2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_progressive.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --progressive-frac 1.0 --pool 256 --steps 3 --warmup 1 --e2e-steps 0 --one-threads 0 \
    --cpu-seconds 6 --out $OUT/p100.json > $OUT/p100.log 2>&1
rc=$?; echo "=== p100 exit $rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('$OUT/p100.json'));print(d['value'],d['ms_per_step'],d['cpu_baseline'])"
timeout -k 10 400 python bench.py --progressive-frac 0.1 --pool 1024 --steps 4 --warmup 1 --e2e-steps 0 \
    --one-threads 32 --one-images 2048 --no-cpu-baseline --prog-lanes 2 --out $OUT/mix_l2.json > $OUT/mix_l2.log 2>&1
rc=$?; echo "=== mix lanes 2 exit $rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('$OUT/mix_l2.json'));print(d['value'],d['ms_per_step'],d.get('e2e_decode_one'))"
