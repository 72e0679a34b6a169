# Round-2 measurement of the headline workload (bench.py default = configs[3], 8-cam x 2000 frames):
# GPU tests, the bench line, rocprofv3 kernel stats, FETCH/WRITE PMC passes, SQ counter passes, phase stamps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/m; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -3 $O/gputests.log
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
echo "trace ok"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_fetch -o pmc -- python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit $?
echo "fetch ok"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_write -o pmc -- python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline > $O/pmc_write.log 2>&1 || exit $?
echo "write ok"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $R/$O/pmc_sq1 -o pmc -- python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline > $O/pmc_sq1.log 2>&1 || exit $?
echo "sq1 ok"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS --output-format csv -d $R/$O/pmc_sq2 -o pmc -- python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline > $O/pmc_sq2.log 2>&1 || echo "sq2 failed (counter names?)"
timeout -k 10 200 python3 tools/diag_stamps.py 4 50 0 k_build_gn,k_solve > $O/stamps.log 2>&1 || { cat $O/stamps.log; exit 1; }
cat $O/stamps.log
python3 tools/prof_summary.py $O/prof
