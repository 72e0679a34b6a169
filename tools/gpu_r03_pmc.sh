#!/bin/bash
# round-3 PMC traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the configs[3] and configs[4] bench workloads,
# and the k_solve timeline of the diagnostic library
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/pmc3; rm -rf $O; mkdir -p $O
for CFG in 4 5; do
  D=$O/c$CFG; mkdir -p $D
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$D/pmc_fetch -o pmc -- python3 bench.py --config $CFG --steps 20 --warmup 2 --no-cpu-baseline > $D/fetch.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$D/pmc_write -o pmc -- python3 bench.py --config $CFG --steps 20 --warmup 2 --no-cpu-baseline > $D/write.log 2>&1 || exit $?
  python3 tools/pmc_traffic.py $D $D/pmc_traffic_c$CFG.json $CFG || exit 1
done
timeout -k 10 120 python3 tools/diag_tstamps.py 4 > $O/solve_timeline.log 2>&1 || { tail -20 $O/solve_timeline.log; exit 1; }
tail -30 $O/solve_timeline.log
