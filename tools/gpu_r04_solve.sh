#!/bin/bash
# round-4 camera-solve iteration: the C > 64 solve tests (or $1), the default bench line, the k_solve timeline
# (stamps library), rocprofv3 kernel stats of the bench.  gpurun_out/sv/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/sv; rm -rf $O; mkdir -p $O
T=${1:-"tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_edge_cases.py tests/test_gpu_conditioner.py tests/test_gpu_sharded_local.py tests/test_gpu_pcg.py"}
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputests.log 2>&1 || { tail -60 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('c4', d['value'], d['per_pass_median_ms'], d['roofline']['avg_ms'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -6 $O/sum.txt
if [ -f kalibr_amd/libkalibr_hip_stamps.so ]; then
  timeout -k 10 200 python3 tools/diag_tstamps.py 4 > $O/ts.log 2>&1 || { cat $O/ts.log; exit 1; }
  tail -36 $O/ts.log
fi
