set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
O=gpurun_out/stops6; rm -rf $O; mkdir -p $O
for st in 0 1 2 3; do
  KB_DIAG_LIB=1 KSP_DBG_STOP=$st timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p$st -o bench -- python3 bench.py --config 5 --steps 30 --warmup 2 --no-cpu-baseline > $O/p$st.log 2>&1 || exit $?
  python3 tools/prof_summary.py $O/p$st > $O/sum$st.txt
  echo "== stop $st"; grep -E 'k_sp_assemble' $O/sum$st.txt | head -3
done
