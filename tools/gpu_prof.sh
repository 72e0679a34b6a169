# rocprofv3 kernel trace + stats of a short bench run (no counters), for the per-kernel timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$?; echo "rocprof rc=$rc"
tail -1 gpurun_out/prof.log | cut -c1-300
python3 tools/prof_summary.py gpurun_out/prof
exit $rc
