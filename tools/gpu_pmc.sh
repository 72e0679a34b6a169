# Committed profile of the bench workload: rocprofv3 kernel trace + stats, then two separate PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), summarised by tools/pmc_traffic.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit $?
echo "trace ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o pmc -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 || exit $?
echo "fetch ok"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o pmc -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1 || exit $?
echo "write ok"
find gpurun_out/pmc_fetch gpurun_out/pmc_write -name "*.csv"
python3 tools/prof_summary.py gpurun_out/prof
