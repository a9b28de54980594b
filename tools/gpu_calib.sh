#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on known byte counts (tools/fetch_calib),
# then the isolated-pass kernel trace of the headline bench (batches one at a
# time: roofline_isolated) summarised per stage by tools/rocpd_stages.py.
# OUT=gpurun_out/calib
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/calib}
mkdir -p $OUT
if [ "${CALIB:-1}" = 1 ]; then
  timeout -k 10 60 rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || echo "counter list rc $?"
  for pass in fetch:FETCH_SIZE write:WRITE_SIZE \
      req:TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_128B_sum \
      wreq:TCC_EA0_WRREQ_sum,TCC_EA0_WRREQ_64B_sum; do
    sub=${pass%%:*}; ctr=${pass#*:}
    echo "=== pmc $ctr"
    timeout -s KILL 120 rocprofv3 --pmc ${ctr//,/ } --output-format csv -d $OUT/$sub -o run -- tools/fetch_calib \
      > $OUT/$sub.jsonl 2> $OUT/$sub.err
    rc=$?; echo "exit $rc"; [ $rc -eq 0 ] || { tail -5 $OUT/$sub.err; exit $rc; }
  done
  python tools/fetch_calib.py $OUT > $OUT/fetch_calib.json && cat $OUT/fetch_calib.json
fi
if [ "${ISO:-1}" = 1 ]; then
  echo "=== isolated-pass kernel trace"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/iso -o run -- python3 bench.py --steps 5 --windows 1 \
    --warmup 3 --serial-steps ${SERIAL:-5} --e2e-steps 0 --one-threads 0 --no-cpu-baseline ${BENCH_ARGS:-} \
    --out $OUT/iso_bench.json > $OUT/iso.log 2>&1
  rc=$?; echo "exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/iso.log; exit $rc; }
  db=$(find $OUT/iso -name '*.db' | head -1)
  python tools/rocpd_stages.py "$db" --batches ${SERIAL:-5} > $OUT/stage_spans_isolated.txt
  cat $OUT/stage_spans_isolated.txt
  python -c "import json;d=json.load(open('$OUT/iso_bench.json'));print(json.dumps(d['roofline_isolated']))"
fi
exit 0
