#!/bin/bash
# iteration check: GPU tests, bench (pipelined build vs k_build), kernel stats of the pipelined bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/it; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -3 $O/gputests.log
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
cat $O/bench.json
KB_BUILD_PIPE=0 timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench_old.json 2> $O/bench_old.err || { cat $O/bench_old.err; exit 1; }
cat $O/bench_old.json
timeout -k 10 200 python3 bench.py --no-cpu-baseline --config 3 > $O/bench3.json 2> $O/bench3.err || { cat $O/bench3.err; exit 1; }
cat $O/bench3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof
