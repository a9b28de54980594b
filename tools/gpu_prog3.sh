#!/bin/bash
# Progressive chains: GPU tests, per-scan probe, 100%-progressive pool A/B over prog_chain.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prog3
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_progressive.py tests/test_gpu_semantics.py -q -x --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/prog_scan_probe.py > $OUT/probe.log 2>&1
rc=$?; tail -12 $OUT/probe.log; [ $rc -eq 0 ] || exit $rc
for c in ${CHAINS:-0 100}; do
  timeout -k 10 400 python bench.py --progressive-frac 1.0 --pool 256 --steps 3 --warmup 1 --e2e-steps 0 --one-threads 0 \
      --no-cpu-baseline --ctx-opt prog_chain=$c --out $OUT/p100_c$c.json > $OUT/p100_c$c.log 2>&1
  rc=$?; echo "=== p100 chain $c exit $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/p100_c$c.json'));print(d['value'],d['ms_per_step'],d['stages_ms_per_step'].get('prog_scans'))"
done
