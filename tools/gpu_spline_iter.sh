# spline path: parity tests then the configs[4] bench line (no profiler)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_spline.py -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_spline.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_spline.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config 5 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1; rc=$?; echo "bench rc=$rc"; cut -c1-2500 gpurun_out/bench_c5.log
exit $rc
