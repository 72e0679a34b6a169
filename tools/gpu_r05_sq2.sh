#!/bin/bash
# round 5: a second SQ instruction-mix pass of configs[3] (FP64 add / mul, conversions, INT64, branches, flat and
# vector-memory reads, LDS loads) beside the first one in gpu_r05_final.sh (gpurun_out/sq2/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; export TMPDIR=/tmp
S=gpurun_out/sq2; rm -rf $S; mkdir -p $S
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_INSTS_BRANCH SQ_INSTS_FLAT SQ_INSTS_VMEM_RD SQ_INSTS_LDS_LOAD --output-format csv -d $R/$S/pmc_sq2 -o pmc -- python3 bench.py --config 4 --steps 16 --warmup 2 --no-cpu-baseline > $S/p2.log 2>&1 || { tail -5 $S/p2.log; exit 1; }
python3 tools/sq_summary.py $S $S/sq2.json "bench.py --config 4" || exit 1
python3 -c "
import json; d=json.load(open('$S/sq2.json'))
for k,v in d['kernels'].items():
    if 'buildp' in k or 'k_solve' in k: print(k[:50], {a: round(b) for a,b in v.items()})
"
