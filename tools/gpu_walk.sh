#!/bin/bash
# Refinement walk A/B: progressive tests, per-scan probe, PMC on the final refinement, p100 and mix.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/walk
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_progressive.py tests/test_gpu_semantics.py tests/test_gpu_fuzz.py -q -x --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT CHAINS=100 timeout -k 10 300 python -u tools/probe/prog_scan_probe.py > $OUT/probe.log 2>&1 || exit $?
awk '{print $1, $5, $6, $7, $9, ($13-$12)/100000 " ms"}' $OUT/dump_largest_c100.txt
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH --output-format csv -d $OUT/sq -o run -- python3 tools/probe/prog_one.py > $OUT/sq.log 2>&1 || exit $?
B="--e2e-steps 0 --one-threads 0 --no-cpu-baseline --serial-steps 0"
timeout -k 10 400 python bench.py --progressive-frac 1.0 --pool 2048 --steps 24 --warmup 8 $B --out $OUT/p100.json > $OUT/p100.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --progressive-frac 0.1 --pool 4096 --steps 200 --warmup 8 $B --out $OUT/mix.json > $OUT/mix.log 2>&1 || exit $?
python -c "import json;a=json.load(open('$OUT/mix.json'));b=json.load(open('$OUT/p100.json'));print('mix10',a['value'],'p100',b['value'])"
