#!/bin/bash
# dg_decode_one latency: small-batch entropy options (OPTS via tools/gpu_one.sh),
# then the default under a kernel trace with the per-batch chain and a timeline
# of every stream around one batch (tools/one_chain.py).  OUT=gpurun_out/one_trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/one_trace}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
OUT=$OUT/one ONE_IMAGES=2048 THREADS=32 OPTS="${ONE_OPTS:-;small_coded=33554432 sub_small=512 lead_small=1024;small_coded=33554432 sub_small=1024 lead_small=2048}" tools/gpu_one.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 2 --warmup 1 --windows 1 --e2e-steps 0 --no-cpu-baseline --serial-steps 0 --one-threads 32 --one-images 2048 ${TRACE_OPTS:-} --out $OUT/one_trace.json > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
db=$(find $OUT/prof -name '*.db' | head -1)
python tools/one_chain.py "$db" --timeline 6000 > $OUT/chain.txt 2>&1; head -20 $OUT/chain.txt
