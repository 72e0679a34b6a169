set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/prof3 gpurun_out/prof4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof3 -o bench -- python3 tools/bench_configs.py 50 3 > gpurun_out/prof3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof4 -o bench -- python3 tools/bench_configs.py 30 4 > gpurun_out/prof4.log 2>&1 || exit $?
python3 tools/prof_summary.py gpurun_out/prof3
python3 tools/prof_summary.py gpurun_out/prof4
