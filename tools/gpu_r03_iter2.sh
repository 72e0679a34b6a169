#!/bin/bash
# round-3 iteration: -m gpu suite, configs[3] bench + kernel stats, the k_solve timeline, PCG timing, configs[4] bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/it2; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('c4 value', d['value'], 'build_ms', d['roofline'].get('avg_ms'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -5 $O/sum.txt
timeout -k 10 120 python3 tools/diag_tstamps.py 4 > $O/solve_timeline.log 2>&1 || { tail -20 $O/solve_timeline.log; exit 1; }
grep -A3 "panel 6" $O/solve_timeline.log | head -8
timeout -k 10 300 python3 tools/pcg_bench.py 10 > $O/pcg_bench.jsonl 2> $O/pcg_bench.err || { tail -20 $O/pcg_bench.err; exit 1; }
cat $O/pcg_bench.jsonl
timeout -k 10 200 python3 bench.py --config 5 --no-cpu-baseline > $O/bench5.json 2> $O/bench5.err || { cat $O/bench5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench5.json')); print('c5 value', d['value'])"
