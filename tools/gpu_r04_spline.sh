#!/bin/bash
# round-4 spline iteration: the spline tests, the configs[4] bench line with the deep-level kernel and without it
# (KSP_DEEP=0), kernel stats of the default.  gpurun_out/sp/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/sp; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_spline.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in 1 0 1 0; do
  KSP_DEEP=$v timeout -k 10 200 python3 bench.py --config 5 --no-cpu-baseline > $O/b$v.json 2> $O/b$v.err || { tail -5 $O/b$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b$v.json')); print('deep=$v c5', round(d['value']), {k: round(v*1e3,1) for k,v in d['pass_breakdown_ms'].items()})"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 bench.py --config 5 --steps 50 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof > $O/sum.txt; head -18 $O/sum.txt
