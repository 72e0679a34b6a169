#!/bin/bash
# round 3 status: full -m gpu suite, smoke, the default bench line (with CPU baselines), its rocprof kernel stats,
# the configs[4] bench line and the N=1 launcher + RCCL path
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/st; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('value', d['value'], 'build_ms', d['roofline'].get('avg_ms'), 'cpu', d['cpu_baseline']['value'], d.get('cpu_baseline_all_cores',{}).get('value'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -8 $O/sum.txt
timeout -k 10 200 python3 bench.py --config 5 --no-cpu-baseline > $O/bench5.json 2> $O/bench5.err || { cat $O/bench5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench5.json')); print('c5 value', d['value'])"
timeout -k 10 200 python3 bench.py --config 3 --no-cpu-baseline > $O/bench3.json 2> $O/bench3.err || { cat $O/bench3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench3.json')); print('c3 value', d['value'], d['roofline']['avg_ms'])"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --comm --no-cpu-baseline > $O/bench_comm.json 2> $O/bench_comm.err || { tail -30 $O/bench_comm.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_comm.json')); print('comm value', d['value'], d['comm'])"
