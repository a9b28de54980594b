#!/bin/bash
# k_band_dec diagnosis: kernel trace + two SQ counter passes of a short bench run with EXTRA bench args.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcb
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 --one-threads 0 --serial-steps 0 ${EXTRA:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $OUT/sq2 -o run -- python3 bench.py $ARGS > $OUT/sq2.log 2>&1 || exit $?
python tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt 2>&1
grep -E "band_dec|resize_hb|k_idct" $OUT/trace/*kernel_stats.csv | cut -c1-160
