#!/bin/bash
# round 6: A/B of measurement variants (KB_VARIANT_LIB, kalibr_amd/build.py build_variant): the build-path parity tests
# (TESTS, "none" to skip) and the default bench line + the --shard-of 8 line, twice each; VARIANTS="main v1 v2 ..."
# (gpurun_out/var6/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/var6; rm -rf $O; mkdir -p $O
T=${TESTS:-"tests/test_gpu_fullsize.py tests/test_gpu_parity.py"}
for v in ${VARIANTS:-main}; do
  if [ $v = main ]; then unset KB_VARIANT_LIB; else export KB_VARIANT_LIB=$v; fi
  if [ "$T" != none ]; then
    timeout -k 10 300 python -u -m pytest $T -m gpu -q -x --timeout 150 --timeout-method thread > $O/t_$v.log 2>&1 || { tail -30 $O/t_$v.log; exit 1; }
    echo "== $v: $(tail -1 $O/t_$v.log)"
  fi
  for rep in 1 2; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/b_$v.json 2> $O/b_$v.err || { tail -5 $O/b_$v.err; exit 1; }
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --shard-of 8 > $O/s_$v.json 2> $O/s_$v.err || { tail -5 $O/s_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_$v.json')); s=json.load(open('$O/s_$v.json')); print('  $v c4 %.0f med %.5f build %.5f | shard8 %.0f med %.5f build %.5f' % (d['value'], d['per_pass_median_ms'], d['roofline']['avg_ms'], s['value'], s['per_pass_median_ms'], s['roofline']['avg_ms']))"
  done
done
