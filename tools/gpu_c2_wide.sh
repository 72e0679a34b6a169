#!/bin/bash
# configs[2] (4-cam omni-radtan + EUCM): the -m gpu suite, then the bench line with the 12-wave (spilling) and the
# 8-wave (spill-free, default) k_buildp, and kernel stats of the default
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/c2; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
KB_BUILDP_WIDE=0 timeout -k 10 200 python3 bench.py --config 3 --no-cpu-baseline > $O/bench_w0.json 2> $O/bench_w0.err || { cat $O/bench_w0.err; exit 1; }
timeout -k 10 200 python3 bench.py --config 3 --no-cpu-baseline > $O/bench_w1.json 2> $O/bench_w1.err || { cat $O/bench_w1.err; exit 1; }
python3 -c "
import json
for t in ('w0','w1'):
    d=json.load(open('$O/bench_'+t+'.json')); print(t, round(d['value'],1), 'it/s', round(d['roofline']['avg_ms']*1e3,2), 'us build')"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --config 3 --steps 100 --warmup 10 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -8 $O/sum.txt
