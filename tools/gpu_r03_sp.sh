#!/bin/bash
# round 3: the partitioned spline band solve -- spline parity tests, configs[4] bench (partitioned vs KSP_CYCLIC=1
# cyclic reduction), kernel stats of the partitioned pass
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/sp; rm -rf $O; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_spline.py -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 200 python3 bench.py --config 5 --no-cpu-baseline > $O/bench5.json 2> $O/bench5.err || { cat $O/bench5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench5.json')); print('partitioned', d['value'], d['pass_breakdown_ms'])"
KSP_CYCLIC=1 timeout -k 10 200 python3 bench.py --config 5 --no-cpu-baseline > $O/bench5_cr.json 2> $O/bench5_cr.err || { cat $O/bench5_cr.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench5_cr.json')); print('cyclic', d['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --config 5 --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -24 $O/sum.txt
# PCG: parity tests and per-iteration timing
timeout -k 10 300 python -u -m pytest tests/test_gpu_pcg.py -x -q --timeout 200 --timeout-method thread > $O/pcgtests.log 2>&1 || { tail -40 $O/pcgtests.log; exit 1; }
tail -1 $O/pcgtests.log
timeout -k 10 300 python3 tools/pcg_bench.py 10 > $O/pcg_bench.jsonl 2> $O/pcg_bench.err || { tail -20 $O/pcg_bench.err; exit 1; }
cat $O/pcg_bench.jsonl
