#!/bin/bash
# A/B of library builds (DG_LIB_PATH): $LIBS (space-separated, "-" = in-tree) x $ARGS, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/libab2/${TAG:-x}
mkdir -p $OUT
i=0
for rep in 1 2; do
  for lib in $LIBS; do
    i=$((i + 1))
    l=$lib; [ "$l" = "-" ] && l=""
    DG_LIB_PATH=$l timeout -k 10 300 python bench.py ${ARGS:-} --no-cpu-baseline --e2e-steps 0 --one-threads 0 --out $OUT/b_$i.json > $OUT/b_$i.log 2>&1
    rc=$?; echo "=== [$lib] exit $rc"; [ $rc -eq 0 ] || exit $rc
    python -c "import json;d=json.load(open('$OUT/b_$i.json'));s=(d.get('roofline_isolated') or {}).get('stages_ms',{});print(d['value'],d['ms_per_step'],{k:round(v,3) for k,v in s.items() if v>0.3})"
  done
done
