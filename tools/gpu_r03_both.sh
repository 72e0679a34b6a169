#!/bin/bash
# round 3: camera-solve microbenchmark, then the solve iteration (tests, bench, timeline, kernel stats, launch path)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_r03_micro.sh && bash tools/gpu_r03_solve.sh "$@"
