set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t/gputests.log 2>&1 || { tail -40 gpurun_out/t/gputests.log; exit 1; }
tail -2 gpurun_out/t/gputests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/t/prof5 -o bench -- python3 bench.py --config 5 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/t/c5.json 2> gpurun_out/t/c5.err || { tail -5 gpurun_out/t/c5.err; exit 1; }
python3 tools/prof_summary.py gpurun_out/t/prof5 > gpurun_out/t/sum5.txt; head -30 gpurun_out/t/sum5.txt
