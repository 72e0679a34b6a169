#!/bin/bash
# configs[4] iteration: spline parity tests, bench line, kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/sp5; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_spline.py -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 200 python3 bench.py --config 5 --no-cpu-baseline > $O/bench5.json 2> $O/bench5.err || { cat $O/bench5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench5.json')); print('c5', d['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof5 -o bench -- python3 bench.py --config 5 --steps 200 --warmup 20 --no-cpu-baseline > $O/prof5.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof5 > $O/sum5.txt; head -8 $O/sum5.txt
