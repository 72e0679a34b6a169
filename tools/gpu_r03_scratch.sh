#!/bin/bash
# scratch-free k_sp_frames / k_solve: spline + PCG + solve-path tests, configs[4] and configs[3] bench lines, configs[4]
# kernel stats and WRITE_SIZE of the frames kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/scr; rm -rf $O; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 200 python3 bench.py --config 5 --no-cpu-baseline > $O/bench5.json 2> $O/bench5.err || { cat $O/bench5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench5.json')); print('c5', d['value'], d['roofline']['frames_kernel'], d['roofline']['avg_ms'])"
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('c4', d['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof5 -o bench -- python3 bench.py --config 5 --steps 200 --warmup 20 --no-cpu-baseline > $O/prof5.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof5 > $O/sum5.txt; head -8 $O/sum5.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof4 -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/prof4.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof4 > $O/sum4.txt; head -4 $O/sum4.txt
D=$O/c5; mkdir -p $D
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$D/pmc_fetch -o pmc -- python3 bench.py --config 5 --steps 20 --warmup 2 --no-cpu-baseline > $D/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$D/pmc_write -o pmc -- python3 bench.py --config 5 --steps 20 --warmup 2 --no-cpu-baseline > $D/write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $D $D/pmc_traffic_c5.json 5 > /dev/null || exit 1
python3 -c "
import json; d=json.load(open('$D/pmc_traffic_c5.json'))
for k,v in d['kernels'].items():
  if 'frames' in k or 'assemble' in k: print(k[:40], v)"
