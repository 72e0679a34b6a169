#!/bin/bash
# round 3 microbenchmarks: the panel LDL^T broadcast variants and dependent-chain latencies, instruction-cache cost
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/m2; rm -rf $O; mkdir -p $O
[ -n "$ALL" ] && timeout -k 10 60 ./tools/micro/panel_factor > $O/panel.txt 2>&1; cat $O/panel.txt
timeout -k 10 60 ./tools/micro/camera_solve > $O/camsolve.txt 2>&1; cat $O/camsolve.txt
timeout -k 10 60 ./tools/micro/simd_share > $O/share.txt 2>&1; cat $O/share.txt
