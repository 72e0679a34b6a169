#!/bin/bash
# Schur-complement PCG: PCG tests (full-system and Schur), timing, then the solve-path suite and the configs[3] bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/pcgs; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pcg.py -x -q --timeout 200 --timeout-method thread > $O/pcgtests.log 2>&1 || { tail -40 $O/pcgtests.log; exit 1; }
tail -1 $O/pcgtests.log
timeout -k 10 300 python3 tools/pcg_bench.py 10 > $O/pcg_bench.jsonl 2> $O/pcg_bench.err || { tail -20 $O/pcg_bench.err; exit 1; }
cat $O/pcg_bench.jsonl
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('c4 value', d['value'], 'build_ms', d['roofline'].get('avg_ms'))"
