#!/bin/bash
# SIMD-sharing micro + MFMA rate micro (round 3 build-kernel design)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/share; rm -rf $O; mkdir -p $O
[ -n "$SHARE" ] && timeout -k 10 60 ./tools/micro/simd_share > $O/share.txt 2>&1; cat $O/share.txt
timeout -k 10 60 ./tools/micro/mfma_f64_rate > $O/rate.txt 2>&1; cat $O/rate.txt
