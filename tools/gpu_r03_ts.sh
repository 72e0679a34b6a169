#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/ts; rm -rf $O; mkdir -p $O
timeout -k 10 200 python3 tools/diag_tstamps.py 4 > $O/ts.log 2>&1 || { cat $O/ts.log; exit 1; }
tail -36 $O/ts.log
timeout -k 10 200 python3 tools/diag_bstamps.py 4 > $O/bs.log 2>&1 || { cat $O/bs.log; exit 1; }
tail -50 $O/bs.log
