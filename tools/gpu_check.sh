# GPU tests (incl. full-size parity) + the default bench line; logs under gpurun_out/c/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/c; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -3 $O/gputests.log
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
cat $O/bench.json
