#!/bin/bash
# sharded path, several ranks on one GPU (kb_comm_init_local)
set -o pipefail
mkdir -p gpurun_out/sl
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded_local.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/sl/tests.log 2>&1
rc=$?
tail -30 gpurun_out/sl/tests.log
exit $rc
