# rocprofv3 kernel stats of the configs[4] spline GN pass
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/prof_c5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5 -o c5 -- python3 bench.py --config 5 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1; rc=$?; echo "rocprof rc=$rc"
f=$(find gpurun_out/prof_c5 -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | head -30
exit $rc
