# Round-1 profile refresh: PMC traffic passes for the bench kernels, per-config rates, config 3/4 kernel traces
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
true
true
timeout -k 10 300 python3 tools/bench_configs.py 100 > gpurun_out/configs.log 2>&1 || exit $?
cat gpurun_out/configs.log
timeout -k 10 700 bash tools/gpu_prof34.sh > gpurun_out/prof34.log 2>&1 || exit $?
cat gpurun_out/prof34.log
