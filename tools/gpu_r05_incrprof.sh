#!/bin/bash
# round 5: rocprofv3 kernel statistics of the incremental estimator run (configs[1], 500 batches) -> gpurun_out/ip5/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/ip5; rm -rf $O; mkdir -p $O
g++ -O2 -std=c++17 -o $O/test_host tests/cpp/test_host.cpp -I include -I kalibr_amd/host -I oracle \
  -L kalibr_amd -lkalibr_backend -lkalibr_hip -L oracle/_build -lkb_oracle -lpthread \
  -Wl,-rpath,$R/kalibr_amd:$R/oracle/_build || exit 1
python3 -c "
import sys; sys.path.insert(0, '.')
from kalibr_amd import synth
from tests.host_problem import write_problem
write_problem('$O/c1.bin', synth.make_config(2))
" || exit 1
KB_INCR_EAGER_ONLY=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o incr -- $O/test_host incr-time $O/c1.bin 0.2 20 2 4 > $O/incr.json 2> $O/incr.err || { tail -20 $O/incr.err; exit 1; }
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -24 $O/sum.txt
