#!/bin/bash
# round-5 spline close-out: -m gpu suite, smoke(), the configs[4] bench line (with its CPU baseline) and rocprofv3
# kernel stats of it, and the default configs[3] line as a regression check.  gpurun_out/spf/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/spf; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { tail -60 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --config 5 > $O/bench_c5.json 2> $O/bench_c5.err || { cat $O/bench_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c5.json')); print('c5', d['value'], d['pass_breakdown_ms'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c5 -o bench -- python3 bench.py --config 5 --steps 100 --warmup 10 --no-cpu-baseline > $O/prof_c5.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof_c5 > $O/sum_c5.txt; head -14 $O/sum_c5.txt
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { cat $O/bench_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c4.json')); print('c4', d['value'], d['per_pass_median_ms'])"
