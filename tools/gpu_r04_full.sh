#!/bin/bash
# round-4 measurement call: the -m gpu suite, the default bench line (200 / 20 steps), rocprofv3 kernel stats of it,
# FETCH_SIZE / WRITE_SIZE passes (configs[3], configs[4]), an SQ stall pass of configs[3], the --shard-of 8 profile,
# the configs[4] bench line and the incremental-estimator timing.  Everything under gpurun_out/r4/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/r4; rm -rf $O; mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputests.log 2>&1 || { tail -60 $O/gputests.log; exit 1; }
  tail -1 $O/gputests.log
fi
timeout -k 10 200 python3 bench.py > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { cat $O/bench20.err; exit 1; }
echo bench20; cat $O/bench20.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -12 $O/sum.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_shard8 -o bench -- python3 bench.py --shard-of 8 --steps 200 --warmup 20 --no-cpu-baseline > $O/shard8.json 2> $O/shard8.err || { tail -20 $O/shard8.err; exit 1; }
python3 tools/prof_summary.py $O/prof_shard8 > $O/sum_shard8.txt; cat $O/shard8.json; head -12 $O/sum_shard8.txt
for CFG in 4 5; do
  D=$O/pmc_c$CFG; mkdir -p $D
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$D/pmc_fetch -o pmc -- python3 bench.py --config $CFG --steps 20 --warmup 2 --no-cpu-baseline > $D/fetch.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$D/pmc_write -o pmc -- python3 bench.py --config $CFG --steps 20 --warmup 2 --no-cpu-baseline > $D/write.log 2>&1 || exit $?
  python3 tools/pmc_traffic.py $D $D/pmc_traffic_c$CFG.json $CFG || exit 1
done
echo pmc done
S=$O/sq; mkdir -p $S
timeout -s KILL 60 rocprofv3 -L > $S/avail.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" $S/avail.txt | sort -u > $S/sq_names.txt || true
P3=""
for c in SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY; do
  if grep -qx $c $S/sq_names.txt; then P3="$P3 $c"; else echo "counter $c not available"; fi
done
timeout -s KILL 120 rocprofv3 --pmc $P3 --output-format csv -d $R/$S/pmc_sq3 -o pmc -- python3 bench.py --config 4 --steps 16 --warmup 2 --no-cpu-baseline > $S/p3.log 2>&1 || exit $?
python3 tools/sq_summary.py $S $S/sq.json "bench.py --config 4" || exit 1
timeout -k 10 200 python3 bench.py --config 5 --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { cat $O/bench_c5.err; exit 1; }
echo c5; cat $O/bench_c5.json
timeout -k 10 400 bash tools/incr_bench.sh ${INCR_BATCHES:-100} 16 || exit 1
