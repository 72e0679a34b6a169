# phase stamps of the GN pass kernels at the bench workload (diagnostic library) -> gpurun_out/s/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/s; export TMPDIR=/tmp
timeout -k 10 300 python3 tools/diag_stamps.py ${1:-4} 50 0 ${2:-k_build_gn,k_solve} > gpurun_out/s/stamps.log 2>&1 || { cat gpurun_out/s/stamps.log; exit 1; }
cat gpurun_out/s/stamps.log
