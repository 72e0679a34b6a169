#!/bin/bash
# k_solve timeline (stamps library) and the instruction-cache counters of the default bench (one --pmc pass).
# gpurun_out/ic/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/ic; rm -rf $O; mkdir -p $O
timeout -k 10 200 python3 tools/diag_tstamps.py 4 > $O/ts.log 2>&1 || { cat $O/ts.log; exit 1; }
tail -44 $O/ts.log
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQC_[A-Z0-9_]*" $O/avail.txt | sort -u > $O/sqc_names.txt || true
cat $O/sqc_names.txt | tr '\n' ' '; echo
P=""
for c in SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE; do
  if grep -qx $c $O/sqc_names.txt; then P="$P $c"; fi
done
echo "counters: $P"
if [ -n "$P" ]; then
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/$O/pmc_sq1 -o pmc -- python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline > $O/pmc.log 2>&1 || exit $?
  python3 tools/sq_summary.py $O $O/sqc.json "bench.py --config 4 (SQC)" || exit 1
  python3 -c "import json; d=json.load(open('$O/sqc.json'))['kernels']; [print(k[:40], v) for k,v in d.items()]"
fi
