#!/bin/bash
# A/B of measurement variants (KB_VARIANT_LIB, kalibr_amd/build.py build_variant) against the default library:
# the C > 64 camera-solve tests (variants bs1: readlane-era backsolve, pf1: readlane panel factor) and the spline
# tests + configs[4] bench (variant ch1: the readlane 18 x 18 Cholesky).  gpurun_out/ab/
cd ${GRAFT_REPO_ROOT:-$(pwd)}; export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
T="tests/test_gpu_conditioner.py tests/test_gpu_fullsize.py tests/test_gpu_edge_cases.py tests/test_gpu_parity.py"
for v in ${VARIANTS:-main bs1 pf1}; do
  if [ $v = main ]; then unset KB_VARIANT_LIB; else export KB_VARIANT_LIB=$v; fi
  echo "== $v"; timeout -k 10 300 python -u -m pytest $T -m gpu -q -x --timeout 150 --timeout-method thread > $O/t_$v.log 2>&1; tail -3 $O/t_$v.log
done
for v in ${SPVARIANTS:-main ch1}; do
  if [ $v = main ]; then unset KB_VARIANT_LIB; else export KB_VARIANT_LIB=$v; fi
  echo "== spline $v"; timeout -k 10 300 python -u -m pytest tests/test_gpu_spline.py -m gpu -q -x --timeout 150 --timeout-method thread > $O/s_$v.log 2>&1; tail -2 $O/s_$v.log
  timeout -k 10 200 python3 bench.py --config 5 --no-cpu-baseline > $O/b5_$v.json 2> $O/b5_$v.err || { tail -5 $O/b5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b5_$v.json')); print('c5', d['value'], d['pass_breakdown_ms'])"
done
unset KB_VARIANT_LIB
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/b4.json 2> $O/b4.err || { tail -5 $O/b4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b4.json')); print('c4', d['value'], d['per_pass_median_ms'], d['roofline']['avg_ms'])"
