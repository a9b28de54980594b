#!/bin/bash
# Refinement walk: progressive GPU tests, per-scan probe, 100%-progressive pool at batch 256 and 1024.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prog5
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_progressive.py tests/test_gpu_semantics.py tests/test_gpu_fuzz.py -q -x --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT CHAINS=100 timeout -k 10 300 python -u tools/probe/prog_scan_probe.py > $OUT/probe.log 2>&1
rc=$?; tail -5 $OUT/probe.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT CFGS="256 100|1024 100|1024 0" bash -c 'IFS="|"; for cfg in $CFGS; do IFS=" "; set -- $cfg;
  timeout -k 10 500 python bench.py --progressive-frac 1.0 --pool 1024 --batch $1 --steps 3 --warmup 1 --e2e-steps 0 \
      --one-threads 0 --no-cpu-baseline --serial-steps 1 --ctx-opt prog_chain=$2 --out $OUT/p100_b$1_c$2.json > $OUT/p100_b$1_c$2.log 2>&1
  rc=$?; echo "=== batch $1 chain $2 exit $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open(\"$OUT/p100_b$1_c$2.json\"));print(d[\"value\"],d[\"ms_per_step\"],d[\"stages_ms_per_step\"].get(\"prog_scans\"))"
done'
