# config 4 at the 8-GPU per-rank shard size (250 frames) and full size on one GPU: rate + kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/prof4s
timeout -k 10 200 python3 tools/bench_configs.py 100 4 250 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof4s -o bench -- python3 tools/bench_configs.py 50 4 250 > gpurun_out/prof4s.log 2>&1 || exit $?
python3 tools/prof_summary.py gpurun_out/prof4s
