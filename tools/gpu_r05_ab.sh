#!/bin/bash
# round 5: A/B of variants (VARIANTS, default "main") on the default and --shard-of 8 lines, then the incremental
# estimator timing with per-phase host profiles when INCR=1 (gpurun_out/ab5/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/ab5; rm -rf $O; mkdir -p $O
for v in ${VARIANTS:-main}; do
  if [ $v = main ]; then unset KB_VARIANT_LIB; else export KB_VARIANT_LIB=$v; fi
  for rep in 1 2; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/b_$v.json 2> $O/b_$v.err || { tail -5 $O/b_$v.err; exit 1; }
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --shard-of 8 > $O/s_$v.json 2> $O/s_$v.err || { tail -5 $O/s_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_$v.json')); s=json.load(open('$O/s_$v.json')); print('$v  c4 %.0f med %.5f build %.5f | shard8 %.0f med %.5f build %.5f' % (d['value'], d['per_pass_median_ms'], d['roofline']['avg_ms'], s['value'], s['per_pass_median_ms'], s['roofline']['avg_ms']))"
  done
done
unset KB_VARIANT_LIB
if [ "${INCR:-0}" = 1 ]; then
  bash tools/incr_bench.sh 20 16 || exit 1
fi
