# rocprofv3 of bench.py for the committed tree (_head/, built locally) next to the working tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
for t in head work; do
  D=$R; [ $t = head ] && D=$R/_head
  rm -rf gpurun_out/prof_$t
  (cd $D && KB_GN_FUSED=${FZ:-0} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$t -o bench -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $R/gpurun_out/prof_$t.log 2>&1); rc=$?; echo "$t rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof_$t.log; exit $rc; fi
  tail -1 gpurun_out/prof_$t.log | cut -c1-120
  python3 tools/prof_summary.py gpurun_out/prof_$t | head -8
done
