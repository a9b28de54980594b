#!/bin/bash
# Integration-path check: GPU tests that use host buffers, then a bench run
# with the host-in/host-out legs (e2e_host_mpix_s, dg_decode_one).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/e2e
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_samples.py tests/test_gpu_parity.py} -q -m gpu -x \
    --timeout 300 --timeout-method thread > gpurun_out/e2e/pt.log 2>&1
rc=$?; tail -2 gpurun_out/e2e/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${EXTRA:-} \
    --out gpurun_out/e2e/b.json > gpurun_out/e2e/b.log 2>&1
rc=$?; echo "bench rc $rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.load(open('gpurun_out/e2e/b.json'));print(d['value'],d['e2e_host_mpix_s'],d['e2e_host_in_hbm_out_mpix_s'],d['e2e_decode_one'])"
