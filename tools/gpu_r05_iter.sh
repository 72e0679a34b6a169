#!/bin/bash
# round-5 iteration: the -m gpu tests matching $1 (all when empty, none when "none"), the default bench line at 200
# and at 20 passes (no CPU baseline), the --shard-of 8 line, and rocprofv3 kernel stats of the default line when
# PROF=1.  Everything under gpurun_out/it5/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/it5; rm -rf $O; mkdir -p $O
if [ "$1" != "none" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${1:+-k "$1"} > $O/gputests.log 2>&1 || { tail -60 $O/gputests.log; exit 1; }
  tail -1 $O/gputests.log
fi
for S in 200 20; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps $S --warmup 5 > $O/bench$S.json 2> $O/bench$S.err || { cat $O/bench$S.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench$S.json')); print('bench$S', round(d['value'],1), d['ms_per_step'], d['per_pass_median_ms'], d['roofline']['avg_ms'], d['roofline']['frac'])"
done
timeout -k 10 200 python3 bench.py --shard-of 8 --no-cpu-baseline --steps 200 --warmup 5 > $O/shard8.json 2> $O/shard8.err || { tail -20 $O/shard8.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/shard8.json')); print('shard8', round(d['value'],1), d['per_pass_median_ms'], d['roofline']['avg_ms'])"
if [ "${PROF:-0}" = 1 ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
  python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -8 $O/sum.txt
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_shard8 -o bench -- python3 bench.py --shard-of 8 --steps 200 --warmup 20 --no-cpu-baseline > $O/prof_shard8.log 2>&1 || exit $?
  python3 tools/prof_summary.py $O/prof_shard8 > $O/sum_shard8.txt; head -8 $O/sum_shard8.txt
fi
