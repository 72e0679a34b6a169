#!/bin/bash
# round 5: k_marg (marginal Jacobi SVD) rework -- the marginal / incremental -m gpu tests, the incremental estimator
# timing (incr_bench.sh), the eager device loop with cold starts (KB_MARG_COLD) beside it, and the rocprofv3 kernel
# statistics of the eager run.  gpurun_out/incr/, gpurun_out/ip5/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "${1:-marginal or incremental or host_cpp}" > gpurun_out/marg_tests.log 2>&1 || { tail -60 gpurun_out/marg_tests.log; exit 1; }
tail -1 gpurun_out/marg_tests.log
bash tools/incr_bench.sh 100 16 || exit 1
O=gpurun_out/incr
KB_MARG_COLD=1 KB_INCR_EAGER_ONLY=1 timeout -k 10 300 $O/test_host incr-time $O/c1.bin 0.2 20 2 4 > $O/cold.json 2>&1 || { cat $O/cold.json; exit 1; }
echo cold: $(cat $O/cold.json)
KB_INCR_EAGER_ONLY=1 timeout -k 10 300 $O/test_host incr-time $O/c1.bin 0.2 20 2 4 > $O/warm.json 2>&1 || { cat $O/warm.json; exit 1; }
echo warm: $(cat $O/warm.json)
if [ "${PROF:-1}" = 1 ]; then
  P=gpurun_out/ip5; rm -rf $P; mkdir -p $P
  KB_INCR_EAGER_ONLY=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$P/prof -o incr -- $O/test_host incr-time $O/c1.bin 0.2 20 2 4 > $P/incr.json 2> $P/incr.err || { tail -20 $P/incr.err; exit 1; }
  python3 tools/prof_summary.py $P/prof > $P/sum.txt; head -16 $P/sum.txt
fi
