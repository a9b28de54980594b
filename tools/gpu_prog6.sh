#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prog6
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_progressive.py tests/test_gpu_semantics.py tests/test_gpu_fuzz.py -q -x --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/probe/prog_one.py > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/sq -o run -- python3 tools/probe/prog_one.py > $OUT/sq.log 2>&1 || exit $?
OUT=$OUT CHAINS=100 timeout -k 10 300 python -u tools/probe/prog_scan_probe.py > $OUT/probe.log 2>&1
rc=$?; tail -4 $OUT/probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --progressive-frac 1.0 --pool 1024 --batch 1024 --steps 3 --warmup 1 --e2e-steps 0 \
      --one-threads 0 --no-cpu-baseline --serial-steps 1 --out $OUT/p100_b1024.json > $OUT/p100_b1024.log 2>&1 || exit $?
python -c "import json;d=json.load(open('$OUT/p100_b1024.json'));print(d['value'],d['ms_per_step'],d['stages_ms_per_step'].get('prog_scans'))"
