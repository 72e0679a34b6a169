#!/bin/bash
# configs[4] stop-point timing: the spline kernels return after phase KSP_DBG_STOP (results invalid, timing only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/stops; rm -rf $O; mkdir -p $O
for st in 0 1 2 3 4; do
  KB_DIAG_LIB=1 KSP_DBG_STOP=$st timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p$st -o bench -- python3 bench.py --config 5 --steps 30 --warmup 2 --no-cpu-baseline > $O/p$st.log 2>&1 || exit $?
  python3 tools/prof_summary.py $O/p$st > $O/sum$st.txt
  echo "== stop $st"; grep -E 'k_sp_level|k_sp_back|k_sp_assemble' $O/sum$st.txt | head -3
done
