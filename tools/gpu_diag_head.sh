# stop-point diagnostics of k_solve for the committed tree (_head/) and the working tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for t in head work; do
  D=$R; [ $t = head ] && D=$R/_head
  (cd $D && timeout -k 10 300 python tools/diag_stamps.py 2 200 0 ${KERN:-k_solve} > $R/gpurun_out/diag_$t.log 2>&1); rc=$?; echo "$t rc=$rc"
  cat gpurun_out/diag_$t.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
