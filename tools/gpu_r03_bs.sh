#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/bs; rm -rf $O; mkdir -p $O
timeout -k 10 200 python3 tools/diag_bstamps.py ${1:-4} > $O/bs.log 2>&1 || { cat $O/bs.log; exit 1; }
cat $O/bs.log
