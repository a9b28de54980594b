#!/bin/bash
# Headline bench with experiment library builds (DG_LIB_PATH) against the in-tree one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/libab
mkdir -p $OUT
i=0
for lib in "" exp/lib_m11.so exp/lib_m12.so "" exp/lib_m11.so exp/lib_m12.so; do
  i=$((i + 1))
  DG_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --e2e-steps 0 --one-threads 0 --no-cpu-baseline --out $OUT/b_$i.json > $OUT/b_$i.log 2>&1
  rc=$?; echo "=== [$lib] exit $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$OUT/b_$i.json'));s=d['roofline_isolated']['stages_ms'];print(d['value'],d['ms_per_step'],s['huff_sync'],s['huff_write'])"
done
