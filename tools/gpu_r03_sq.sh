#!/bin/bash
# SQ instruction-mix counters of the bench workload (two passes, 8 SQ counters each), summarised per kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
O=gpurun_out/sq; rm -rf $O; mkdir -p $O
CFG=${1:-4}
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" $O/avail.txt | sort -u > $O/sq_names.txt || true
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_MFMA"
P2="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
for c in $P1 $P2; do grep -qx $c $O/sq_names.txt || { echo "counter $c not available"; exit 3; }; done
timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $R/$O/pmc_sq1 -o pmc -- python3 bench.py --config $CFG --steps 16 --warmup 2 --no-cpu-baseline > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d $R/$O/pmc_sq2 -o pmc -- python3 bench.py --config $CFG --steps 16 --warmup 2 --no-cpu-baseline > $O/p2.log 2>&1 || exit $?
python3 tools/sq_summary.py $O $O/sq.json "bench.py --config $CFG" && python3 - <<'PY'
import json
d = json.load(open("gpurun_out/sq/sq.json"))
for k, v in d["kernels"].items():
    if "buildp" in k or "k_solve" in k or "colimg" in k:
        w = max(v.get("SQ_WAVES", 1), 1)
        print(k[:60], {a: round(b / w, 1) for a, b in v.items() if a != "SQ_WAVES"})
PY
