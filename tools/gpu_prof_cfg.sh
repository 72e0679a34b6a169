# rocprofv3 kernel trace + stats of a bench run of one configuration (no counters):
#   bash tools/gpu_prof_cfg.sh <config index> <out dir under gpurun_out> [extra bench.py args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
cfg=$1; O=gpurun_out/$2; shift 2
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O -o bench -- python3 bench.py --config $cfg --steps 200 --warmup 20 --no-cpu-baseline "$@" > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
python3 tools/prof_summary.py $O > $O/summary.txt && head -30 $O/summary.txt
