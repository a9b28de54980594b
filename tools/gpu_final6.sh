#!/bin/bash
# Round-6 end-of-round evidence at HEAD, in parts (one gpurun call each):
#   PART=pmc    hardware-counter passes incl. request sizes (tools/gpu_pmc.sh) -> pmc_traffic.json
#   PART=tests  the -m gpu suite + smoke
#   PART=bench  the default bench line, then the isolated-pass kernel trace (tools/gpu_calib.sh ISO)
#   PART=wl     configs[2] / configs[4] lines, configs[3] 8 ranks under budgets
# OUT=gpurun_out/final6/<part>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
PART=${PART:-tests}
OUT=${OUT:-gpurun_out/final6}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
case $PART in
pmc)
  OUT=$OUT/pmc tools/gpu_pmc.sh || exit $?
  ;;
tests)
  OUT=$OUT/tests TLIM=1500 tools/gpu_tests.sh || exit $?
  ;;
bench)
  mkdir -p $OUT/bench
  timeout -k 10 600 python bench.py --out $OUT/bench/bench.json > $OUT/bench/bench.log 2>&1
  rc=$?; echo "=== bench exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench/bench.log; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/bench/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline'].get('traffic'),d['cpu_baseline']['value'],(d.get('e2e_decode_one') or {}).get('mpix_s'),d.get('e2e_host_mpix_s'))"
  OUT=$OUT/iso CALIB=0 ISO=1 SERIAL=5 tools/gpu_calib.sh || exit $?
  db=$(find $OUT/iso -name '*.db' | head -1)
  [ -n "$db" ] && python tools/rocpd_stats.py "$db" > $OUT/iso/kernel_stats.csv
  ;;
wl)
  OUT=$OUT/wds WL=wds PROF=0 tools/gpu_wl.sh || exit $?
  OUT=$OUT/png WL=png PROF=0 ARGS="--steps 10 --warmup 2" tools/gpu_wl.sh || exit $?
  OUT=$OUT/png32 WL=png PROF=0 ARGS="--steps 10 --warmup 2 --max-device-mb 32000" tools/gpu_wl.sh || exit $?
  OUT=$OUT/ranks WARMUP=2 STEPS=6 RUNS="b20:--max-device-mb,20000 b30:--max-device-mb,30000" tools/gpu_ranks5.sh || exit $?
  ;;
esac
exit 0
