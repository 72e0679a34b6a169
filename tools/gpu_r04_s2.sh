#!/bin/bash
# round-4 (second session) baseline call: -m gpu suite, the default bench line, the --shard-of 8 line with the
# pipelined build and with k_build (KB_BUILD_PIPE=0) + kernel stats of both, the k_solve and k_buildp timelines
# (stamps library).  gpurun_out/s2/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/s2; rm -rf $O; mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputests.log 2>&1 || { tail -60 $O/gputests.log; exit 1; }
  tail -1 $O/gputests.log
fi
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('c4', d['value'], d['per_pass_median_ms'], d['roofline']['avg_ms'])"
for PIPE in 1 0; do
  KB_BUILD_PIPE=$PIPE timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_sh8_p$PIPE -o bench -- python3 bench.py --shard-of 8 --no-cpu-baseline > $O/sh8_p$PIPE.json 2> $O/sh8_p$PIPE.err || { tail -20 $O/sh8_p$PIPE.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/sh8_p$PIPE.json')); print('shard8 pipe=$PIPE', d['value'], d['per_pass_median_ms'], d['roofline']['avg_ms'])"
  python3 tools/prof_summary.py $O/prof_sh8_p$PIPE > $O/sum_sh8_p$PIPE.txt; head -8 $O/sum_sh8_p$PIPE.txt
done
if [ -f kalibr_amd/libkalibr_hip_stamps.so ]; then
  timeout -k 10 200 python3 tools/diag_tstamps.py 4 > $O/ts.log 2>&1 || { cat $O/ts.log; exit 1; }
  tail -34 $O/ts.log
  timeout -k 10 200 python3 tools/diag_bstamps.py 4 > $O/bs.log 2>&1 || { cat $O/bs.log; exit 1; }
  tail -40 $O/bs.log
fi
if [ -f kalibr_amd/libkalibr_hip_stamps.so ]; then
  timeout -k 10 200 python3 tools/diag_bstamps.py 4 250 > $O/bs250.log 2>&1 || { cat $O/bs250.log; exit 1; }
  tail -30 $O/bs250.log
fi
