#!/bin/bash
# round-4 iteration: the -m gpu suite (optional filter $1), the default bench line (200 and 20 steps), rocprofv3 kernel
# stats of the bench (gpurun_out/it/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/it; rm -rf $O; mkdir -p $O
F=${1:-tests}
timeout -k 10 600 python -u -m pytest $F -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputests.log 2>&1 || { tail -60 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('value', d['value'], 'build_ms', d['roofline'].get('avg_ms'), d.get('per_pass_median_ms'))"
timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { cat $O/bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench20.json')); print('value20', d['value'], d.get('per_pass_median_ms'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -10 $O/sum.txt
