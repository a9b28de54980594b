python -c "import datago_amd._lib as L; L.load()" && timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -le 1 ] || exit $rc
SWEEP="--batch 256,--batch 256" timeout -k 10 600 bash tools/gpu_sweep.sh
