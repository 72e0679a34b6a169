#!/bin/bash
# round-5 diagnosis: the -m gpu tests matching $1, then the k_buildp block-0 timelines at 2000 and 250 frames and the
# camera-solve timeline (stamps library).  gpurun_out/dg/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/dg; rm -rf $O; mkdir -p $O
if [ -n "$1" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$1" > $O/gputests.log 2>&1 || { tail -60 $O/gputests.log; exit 1; }
  tail -1 $O/gputests.log
fi
timeout -k 10 200 python3 tools/diag_bstamps.py 4 250 > $O/bs250.log 2>&1 || { cat $O/bs250.log; exit 1; }
sed -n '/rep 1/,$p' $O/bs250.log
timeout -k 10 200 python3 tools/diag_bstamps.py 4 > $O/bs.log 2>&1 || { cat $O/bs.log; exit 1; }
timeout -k 10 200 python3 tools/diag_tstamps.py > $O/ts.log 2>&1 || { cat $O/ts.log; exit 1; }
tail -40 $O/ts.log
if [ "${INCR:-0}" = 1 ]; then
  bash tools/incr_bench.sh 100 16 || exit 1
fi
