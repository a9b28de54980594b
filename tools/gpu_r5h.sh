#!/bin/bash
# SQ counters per k_inf_decode variant (tools/png_probe.py --variants, one batch
# in flight): what the chunk decode waits on.  OUT=gpurun_out/r5h
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5h}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
V=${PVARS:-2,6,8,12}
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/pmc/sq -o run -- python3 tools/png_probe.py 128 1 --variants=$V > $OUT/pmc_sq.log 2>&1
rc=$?; echo "=== pmc sq exit $rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc_sq.log; exit $rc; }
timeout -s KILL 240 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $OUT/pmc/sq2 -o run -- python3 tools/png_probe.py 128 1 --variants=$V > $OUT/pmc_sq2.log 2>&1
rc=$?; echo "=== pmc sq2 exit $rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc_sq2.log; exit $rc; }
python tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.txt; grep -A23 "inf_decode" $OUT/pmc_summary.txt
