#!/bin/bash
# round 3 iteration: microbenchmark + launch-path diagnostics, then the solve iteration (tests, bench, timeline, stats)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_r03_micro.sh
bash tools/gpu_r03_solve.sh "$@"
