# rocprofv3 kernel trace + stats of short bench runs with the GN fused pass on and off
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
for fz in 1 0; do
  rm -rf gpurun_out/prof_$fz
  KB_GN_FUSED=$fz timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$fz -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof_$fz.log 2>&1; rc=$?; echo "fused=$fz rocprof rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof_$fz.log; exit $rc; fi
  tail -1 gpurun_out/prof_$fz.log | cut -c1-200
  python3 tools/prof_summary.py gpurun_out/prof_$fz
done
