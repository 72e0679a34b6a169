# Round-1 full GPU check: all -m gpu tests, smoke, the contract bench line (configs[1]) and configs[4],
# rocprofv3 kernel stats of both
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_all.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err; rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/bench_c2.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config 5 --steps 200 --warmup 20 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err; rc=$?; echo "bench5 rc=$rc"; cut -c1-300 gpurun_out/bench_c5.json
if [ $rc -ne 0 ]; then exit $rc; fi
rm -rf gpurun_out/prof_c2 gpurun_out/prof_c5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c2 -o c2 -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1; rc=$?; echo "rocprof c2 rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5 -o c5 -- python3 bench.py --config 5 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1; rc=$?; echo "rocprof c5 rc=$rc"
exit $rc
