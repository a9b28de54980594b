#!/bin/bash
# HEAD evidence after the PNG inflate/unfilter options: smoke, default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/head3
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log > $OUT/bench.json
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['roofline']['frac'],d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
