#!/bin/bash
# iteration check: GPU tests, bench, camera-solve timeline, kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/it5; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('value', d['value'], 'build_ms', d['roofline']['avg_ms'])"
timeout -k 10 200 python3 tools/diag_tstamps.py 4 > $O/ts.log 2>&1 || { cat $O/ts.log; exit 1; }
tail -42 $O/ts.log | head -44
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -4 $O/sum.txt
