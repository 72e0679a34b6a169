# quick GPU iteration: parity tests, stamp diagnostics, bench (no profiler)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/diag_stamps.py 2 200 > gpurun_out/diag.log 2>&1; rc=$?; echo "diag rc=$rc"; tail -5 gpurun_out/diag.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/bench.log
exit $rc
