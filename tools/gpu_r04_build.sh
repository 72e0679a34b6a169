#!/bin/bash
# round-4 build-kernel iteration: the build-path tests (or $1), the default bench line, rocprofv3 kernel stats, the
# k_buildp block-0 timeline at 2000 and 250 frames (stamps library).  gpurun_out/bd/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/bd; rm -rf $O; mkdir -p $O
T=${1:-"tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_edge_cases.py tests/test_gpu_sharded_local.py tests/test_gpu_conditioner.py"}
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputests.log 2>&1 || { tail -60 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('c4', d['value'], d['per_pass_median_ms'], d['roofline']['avg_ms'])"
timeout -k 10 200 python3 bench.py --no-cpu-baseline --shard-of 8 > $O/sh8.json 2> $O/sh8.err || { cat $O/sh8.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/sh8.json')); print('shard8', d['value'], d['per_pass_median_ms'], d['roofline']['avg_ms'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -4 $O/sum.txt
if [ -f kalibr_amd/libkalibr_hip_stamps.so ]; then
  timeout -k 10 200 python3 tools/diag_bstamps.py 4 > $O/bs.log 2>&1 || { cat $O/bs.log; exit 1; }
  sed -n '/rep 1/,$p' $O/bs.log | head -60
  timeout -k 10 200 python3 tools/diag_bstamps.py 4 250 > $O/bs250.log 2>&1 || { cat $O/bs250.log; exit 1; }
  sed -n '/rep 1/,$p' $O/bs250.log
fi
