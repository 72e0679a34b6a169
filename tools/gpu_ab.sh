# parity tests, then GN it/s on every config with the GN fused pass on and off (KB_GN_FUSED)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for fz in 1 0; do
  KB_GN_FUSED=$fz timeout -k 10 300 python tools/bench_configs.py ${STEPS:-300} ${CFGS:-1,2,3,4} > gpurun_out/ab_$fz.log 2>&1; rc=$?
  echo "fused=$fz rc=$rc"; cut -c1-300 gpurun_out/ab_$fz.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
