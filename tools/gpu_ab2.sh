#!/bin/bash
# GPU tests (FILES / K subset, TESTS=0 to skip), then the headline bench
# alternating the default and variants (AB="k=v k2=v2;k3=v3": ';'-separated
# variants of space-separated context options, or bench arguments written
# --flag=value), REPS rounds.
#   OUT=gpurun_out/x AB="chroma_rec=0;destuff_one=0" FILES="tests/test_gpu_parity.py" tools/gpu_ab2.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/ab2}
AB=${AB:-chroma_rec=0}
REPS=${REPS:-2}
STEPS=${STEPS:-20}
EXTRA=${EXTRA:-}
mkdir -p $OUT
python -c "import datago_amd._lib as L; L.load()" || exit 3
if [ "${TESTS:-1}" = 1 ]; then
  KARG=()
  [ -n "${K:-}" ] && KARG=(-k "$K")
  timeout -k 10 ${TLIM:-900} python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "${KARG[@]}" \
    ${FILES:-tests} > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
IFS=';' read -ra ABS <<< "$AB"
for r in $(seq 1 $REPS); do
  for k in $(seq 0 ${#ABS[@]}); do
    if [ $k -eq 0 ]; then cfg=""; tag=base_$r; else
      cfg=""; for o in ${ABS[$((k-1))]}; do case $o in --*) cfg="$cfg ${o/=/ }";; *) cfg="$cfg --ctx-opt $o";; esac; done
      tag=ab${k}_$r; fi
    timeout -k 10 400 python bench.py --steps $STEPS --warmup 3 --e2e-steps 0 --one-threads 0 --no-cpu-baseline \
      $EXTRA $cfg --out $OUT/$tag.json > $OUT/$tag.log 2>&1
    rc=$?; echo "=== $tag [$cfg] exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/$tag.log; exit $rc; }
    python -c "import json;d=json.load(open('$OUT/$tag.json'));s=d['roofline_isolated']['stages_ms'];print(d['value'],d['ms_per_step'],{k:round(v,3) for k,v in s.items() if v>0.05});print('  host',d['host_submit_ms_per_step'],d['host_submit_phases_per_rank'][0]['cpu'],d.get('allocations'))"
  done
done
