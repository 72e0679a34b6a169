# GPU check: parity tests, bench line, per-config GN rates (configs 2-4 at full size on one GPU)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/bench_configs.py 100 > gpurun_out/configs.log 2>&1; rc=$?; echo "configs rc=$rc"; cat gpurun_out/configs.log
exit $rc
