#!/bin/bash
# PMC passes over the largest progressive file's per-level scan launches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/progpmc
mkdir -p $OUT
run() {
  local name=$1; shift
  echo "=== $name"
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d $OUT/$name -o run -- python3 tools/probe/prog_one.py > $OUT/$name.log 2>&1
  local rc=$?; echo "exit $rc"; return $rc
}
run trace --kernel-trace --stats &&
run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS &&
run sq2 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS &&
run sq3 --pmc SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_IFETCH SQ_ACTIVE_INST_FLAT SQ_INSTS_SENDMSG SQ_BUSY_CYCLES
