#!/bin/bash
# Hardware-counter passes over a short bench run, one batch in flight so that
# dispatch order maps kernels to stages exactly (one rocprofv3 --pmc pass per
# counter group; never combined with runtime/sys traces).  Output under
# gpurun_out/pmc/<pass>/; summarise with tools/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
ARGS="--steps ${STEPS:-2} --warmup 1 --batch ${BATCH:-256} --pool ${POOL:-4096} --inflight ${INFLIGHT:-1} ${PMC_EXTRA:-} --no-cpu-baseline --e2e-steps 0 --one-threads 0 --serial-steps 0"
run() {  # name counters...
  local name=$1; shift
  echo "=== pmc $name: $*"
  timeout -k 10 400 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 bench.py $ARGS \
      > $OUT/$name.log 2>&1
  local rc=$?
  echo "exit $rc"
  return $rc
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS &&
run sq2 SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run req TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum &&
run wreq TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
rc=$?
[ $rc -eq 0 ] || exit $rc
python tools/pmc_traffic.py $OUT "batch=${BATCH:-256} pool=${POOL:-4096} size=1024/32 short=256-2048" ${BATCH:-256} \
    > $OUT/pmc_traffic.json && python tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt
