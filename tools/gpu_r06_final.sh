#!/bin/bash
# round-6 final measurement, two parts (each within one gpurun call), everything under gpurun_out/r6f/:
#   PART=A: -m gpu suite, smoke(), the default bench line (with the CPU baselines), configs[2] / configs[4] lines,
#           the --shard-of 8 line
#   PART=B: rocprofv3 kernel stats of configs[3] / configs[2] / configs[4] / the shard-of-8 pass, FETCH_SIZE /
#           WRITE_SIZE passes (configs[3], configs[2], configs[4]), one SQ stall pass and one SQ instruction-mix pass of
#           configs[3]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/r6f; mkdir -p $O
if [ "${PART:-A}" = A ]; then
  if [ "${SKIP_TESTS:-0}" != 1 ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1 || { tail -60 $O/gputests.log; exit 1; }
    tail -1 $O/gputests.log
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
    tail -1 $O/smoke.log
  fi
  timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['per_pass_median_ms'], d['roofline']['avg_ms'], d.get('cpu_baseline',{}).get('value'))"
  timeout -k 10 300 python3 bench.py --config 5 > $O/bench_c5.json 2> $O/bench_c5.err || { cat $O/bench_c5.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_c5.json')); print('c5', d['value'], d['pass_breakdown_ms'])"
  timeout -k 10 300 python3 bench.py --config 3 > $O/bench_c3.json 2> $O/bench_c3.err || { cat $O/bench_c3.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_c3.json')); print('c3', d['value'], d['roofline']['frac'])"
  timeout -k 10 200 python3 bench.py --shard-of 8 --no-cpu-baseline > $O/shard8.json 2> $O/shard8.err || { tail -20 $O/shard8.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/shard8.json')); print('shard8', d['value'], d['per_pass_median_ms'], d['roofline']['avg_ms'])"
  exit 0
fi
for C in 4 3 5; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c$C -o bench -- python3 bench.py --config $C --steps 200 --warmup 20 --no-cpu-baseline > $O/prof_c$C.log 2>&1 || exit $?
  python3 tools/prof_summary.py $O/prof_c$C > $O/sum_c$C.txt; head -6 $O/sum_c$C.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_shard8 -o bench -- python3 bench.py --shard-of 8 --steps 200 --warmup 20 --no-cpu-baseline > $O/prof_shard8.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof_shard8 > $O/sum_shard8.txt; head -6 $O/sum_shard8.txt
for CFG in 4 3 5; do
  D=$O/pmc_c$CFG; mkdir -p $D
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$D/pmc_fetch -o pmc -- python3 bench.py --config $CFG --steps 20 --warmup 2 --no-cpu-baseline > $D/fetch.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$D/pmc_write -o pmc -- python3 bench.py --config $CFG --steps 20 --warmup 2 --no-cpu-baseline > $D/write.log 2>&1 || exit $?
  python3 tools/pmc_traffic.py $D $D/pmc_traffic_c$CFG.json $CFG || exit 1
done
echo pmc done
S=$O/sq; mkdir -p $S
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d $R/$S/pmc_sq3 -o pmc -- python3 bench.py --config 4 --steps 16 --warmup 2 --no-cpu-baseline > $S/p3.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $R/$S/pmc_sq1 -o pmc -- python3 bench.py --config 4 --steps 16 --warmup 2 --no-cpu-baseline > $S/p1.log 2>&1 || echo "instruction-mix pass failed (see $S/p1.log)"
python3 tools/sq_summary.py $S $S/sq.json "bench.py --config 4" || exit 1
echo sq done
