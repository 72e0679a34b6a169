# GPU check of the configs[4] spline path: parity tests, then a short timing probe
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_spline.py -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_spline.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_spline.log
exit $rc
