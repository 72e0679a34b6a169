#!/bin/bash
# round-3 camera-solve iteration: parity tests over the C > 64 path, bench line, solve timeline, kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/s3; rm -rf $O; mkdir -p $O
K=${1:-"fullsize or parity or edge or sharded"}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "$K" > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('value', d['value'], 'build_ms', d['roofline'].get('avg_ms'))"
timeout -k 10 200 python3 tools/diag_tstamps.py 4 > $O/ts.log 2>&1 || { cat $O/ts.log; exit 1; }
tail -30 $O/ts.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -6 $O/sum.txt
# the multi-process launch path at N=1: torch.distributed.run + stdlib rendezvous + one-rank RCCL communicator
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --comm --no-cpu-baseline > $O/bench_comm.json 2> $O/bench_comm.err || { tail -30 $O/bench_comm.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_comm.json')); print('comm value', d['value'], d['comm'])"
