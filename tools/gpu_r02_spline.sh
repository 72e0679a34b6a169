#!/bin/bash
# configs[4] (spline + IMU) measurement: spline GPU tests, bench line (with the CPU baseline), rocprofv3 kernel
# stats, FETCH / WRITE PMC passes (-> tools/pmc_traffic.py ... 5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/s5; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_spline.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 bench.py --config 5 --steps 200 --warmup 10 > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --config 5 --steps 100 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -24 $O/sum.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_fetch -o pmc -- python3 bench.py --config 5 --steps 8 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit $?
echo "fetch ok"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_write -o pmc -- python3 bench.py --config 5 --steps 8 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1 || exit $?
echo "write ok"
python3 tools/pmc_traffic.py $O $O/pmc_traffic_c5.json 5 > /dev/null && echo "traffic ok"
