# configs[4] bench line + rocprofv3 kernel stats of the spline GN pass
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config 5 --steps 50 --warmup 5 > gpurun_out/bench_c5.log 2>&1; rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_c5.log | cut -c1-3000
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5 -o c5 -- python3 bench.py --config 5 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1; rc=$?; echo "rocprof rc=$rc"
find gpurun_out/prof_c5 -name "*stats*"
exit $rc
