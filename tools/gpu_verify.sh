#!/bin/bash
# round-end rehearsal: the -m gpu suite, smoke(), the default bench line and the configs[4] kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/v; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -3 $O/gputests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --config 5 --steps 50 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -20 $O/sum.txt
