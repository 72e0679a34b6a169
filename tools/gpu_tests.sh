#!/bin/bash
# the -m gpu suite (optionally a -k filter as $1)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/t; rm -rf $O; mkdir -p $O
if [ -n "$1" ]; then K="-k $1"; else K=""; fi
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread $K > $O/gputests.log 2>&1
rc=$?
tail -30 $O/gputests.log
exit $rc
