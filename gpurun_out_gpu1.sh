set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/pytest1.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench1.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench1.log
exit $rc
