#!/bin/bash
# Full GPU suite, progressive probe, then mixed (10% progressive) benches:
# dg_submit batches + dg_decode_one from 32 threads, prog_lanes 1 vs 0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mix
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/prog_probe.py > $OUT/probe.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/probe.log; [ $rc -eq 0 ] || exit $rc
i=0
for cfg in "--prog-lanes 1" "--prog-lanes 0"; do
  i=$((i + 1))
  timeout -k 10 400 python bench.py --progressive-frac 0.1 --pool 1024 --steps 4 --warmup 1 --e2e-steps 0 \
      --one-threads 32 --one-images 2048 --no-cpu-baseline $cfg --out $OUT/mix_$i.json > $OUT/mix_$i.log 2>&1
  rc=$?; echo "=== $cfg exit $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/mix_$i.json'));print(d['value'],d['ms_per_step'],d.get('e2e_decode_one'))"
done
