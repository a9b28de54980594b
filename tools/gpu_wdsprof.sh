#!/bin/bash
# configs[2] (WebDataset, small images) kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/wdsprof
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/wdsprof -o run -- python3 bench.py --workload wds \
    --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --e2e-steps 0 --one-threads 0 --serial-steps 1 ${EXTRA:-} \
    --out gpurun_out/wdsprof/b.json > gpurun_out/wdsprof/b.log 2>&1
rc=$?; echo "bench rc $rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/rocpd_stats.py gpurun_out/wdsprof/run_results.db --csv gpurun_out/wdsprof/kernel_stats.csv | head -16
python3 -c "import json;d=json.load(open('gpurun_out/wdsprof/b.json'));print(d['value'],d['ms_per_step'],{k:round(v,3) for k,v in d['roofline_isolated']['stages_ms'].items() if v>0.02})"
