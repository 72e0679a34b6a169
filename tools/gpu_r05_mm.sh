#!/bin/bash
# k_marg micro-run, warm and cold (KB_MARG_COLD), with rocprofv3 kernel statistics.  gpurun_out/mm/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/mm; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "marginal or incremental" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in warm cold; do
  if [ $v = cold ]; then export KB_MARG_COLD=1; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/$v -o mm -- python3 tools/marg_micro.py > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  cat $O/$v.log | grep -v "^W\|rocprof" | tail -3
  python3 - $O/$v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_marg" in r["Name"]:
            print(r["Name"][:40], r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 2), "min", round(float(r["MinNs"]) / 1e3, 2), "max", round(float(r["MaxNs"]) / 1e3, 2))
PY
done
