#!/bin/bash
# round-5 spline reduction iteration: the spline GPU tests, the cyclic-reduction timeline (stamps library), and
# configs[4] bench lines A/B over KSP_BACK2 (and $1 extra env for the B side).  gpurun_out/sp/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/sp; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_spline.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
for v in 0 1; do
  KSP_BACK2=$v timeout -k 10 200 python3 tools/diag_sp_levels.py > $O/levels_b$v.log 2>&1 || { cat $O/levels_b$v.log; exit 1; }
  echo "== KSP_BACK2=$v"; grep -A30 "^rep 2" $O/levels_b$v.log | grep "elim\|level\|back\|total\|tile"
done
for v in 0 1; do
  KSP_BACK2=$v timeout -k 10 200 python3 bench.py --config 5 --no-cpu-baseline > $O/bench_b$v.json 2> $O/bench_b$v.err || { cat $O/bench_b$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_b$v.json')); print('back2=$v', round(d['value'],1), d['pass_breakdown_ms'])"
done
