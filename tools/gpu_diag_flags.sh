# end-to-end duration of one diagnostic kernel (KB_STAMPS build) under several dbg_flags values
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for f in ${FLAGS:-0 2 4 6}; do
  timeout -k 10 300 python tools/diag_stamps.py ${CFG:-2} 300 $f ${KERN:-k_build_gn} > gpurun_out/diagf_$f.log 2>&1; rc=$?
  echo "flags=$f rc=$rc"; tail -1 gpurun_out/diagf_$f.log | grep -o "end [0-9.]*"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/diagf_$f.log; exit $rc; fi
done
