#!/bin/bash
# partitioned spline solve: spline parity (partitioned), timeline stamps, configs[4] bench both ways
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/spts; rm -rf $O; mkdir -p $O
KSP_PARTITION=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_spline.py -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
KSP_PARTITION=1 timeout -k 10 120 python3 tools/diag_sp_ts.py > $O/sp_ts.log 2>&1 || { tail -30 $O/sp_ts.log; exit 1; }
tail -45 $O/sp_ts.log
KSP_PARTITION=1 timeout -k 10 200 python3 bench.py --config 5 --no-cpu-baseline > $O/bench5.json 2> $O/bench5.err || { cat $O/bench5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench5.json')); print('partitioned', d['value'], d['pass_breakdown_ms'])"
KSP_PARTITION=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --config 5 --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -6 $O/sum.txt
