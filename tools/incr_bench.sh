#!/bin/bash
# IncrementalEstimator::addBatch sequence timing (configs[1]: 2-cam rig, 500 batches, one per frame) on the GPU
# (in-place appends, kb_append_frames) beside the same estimator over the oracle's marginal solver for the first
# $1 batches (default 100) at $2 host threads (default 16).  Output: gpurun_out/incr/incr_c1.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/incr; mkdir -p $O
g++ -O2 -std=c++17 -o $O/test_host tests/cpp/test_host.cpp -I include -I kalibr_amd/host -I oracle \
  -L kalibr_amd -lkalibr_backend -lkalibr_hip -L oracle/_build -lkb_oracle -lpthread \
  -Wl,-rpath,$R/kalibr_amd:$R/oracle/_build || exit 1
python3 -c "
import sys; sys.path.insert(0, '.')
from kalibr_amd import synth
from tests.host_problem import write_problem
write_problem('$O/c1.bin', synth.make_config(2))
" || exit 1
timeout -k 10 900 $O/test_host incr-time $O/c1.bin 0.2 20 ${1:-100} ${2:-16} > $O/incr_c1.json 2> $O/incr_c1.err || { cat $O/incr_c1.err; exit 1; }
cat $O/incr_c1.json
