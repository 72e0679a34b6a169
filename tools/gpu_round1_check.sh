# GPU check used during round 1: parity tests, smoke, bench, rocprofv3 kernel-trace summary
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests/ -q -m gpu > gpurun_out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$?; echo "rocprof rc=$rc"
find gpurun_out/prof -name "*stats*"
exit $rc
