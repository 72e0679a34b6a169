set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t/gputests.log 2>&1 || { tail -40 gpurun_out/t/gputests.log; exit 1; }
tail -2 gpurun_out/t/gputests.log
