#!/bin/bash
# Second-pass round-end evidence at the final defaults: PMC traffic (one
# batch in flight), the default bench line (with the native decode_one leg)
# and the configs[2] line with its kernel trace.  OUT=gpurun_out/final2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/final2}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
OUT=$OUT/pmc tools/gpu_pmc.sh || exit $?
timeout -k 10 500 python bench.py --out $OUT/bench.json > $OUT/bench.log 2>&1
rc=$?; echo "=== bench exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench.log; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench.json'));o=d.get('e2e_decode_one') or {};print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['cpu_baseline']['value'],o.get('mpix_s'),o.get('native_threads'),d.get('e2e_host_mpix_s'))"
OUT=$OUT/wds WL=wds tools/gpu_wl.sh || exit $?
