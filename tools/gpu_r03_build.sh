#!/bin/bash
# round-3 build-kernel iteration: parity subset, bench line, k_buildp block timeline, kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/b3; rm -rf $O; mkdir -p $O
K=${1:-"fullsize or parity or edge or sharded"}
CFG=${2:-4}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "$K" > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 200 python3 bench.py --config $CFG --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('value', d['value'], 'kernel_ms', d['roofline'].get('avg_ms'))"
timeout -k 10 200 python3 tools/diag_bstamps.py $CFG > $O/bs.log 2>&1 || { cat $O/bs.log; exit 1; }
tail -60 $O/bs.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --config $CFG --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -6 $O/sum.txt
