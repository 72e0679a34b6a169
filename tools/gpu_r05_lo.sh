#!/bin/bash
# launch-overhead measurement (tools/launch_overhead.py), then the 20- and 200-pass bench lines twice each
cd ${GRAFT_REPO_ROOT:-$(pwd)}; export TMPDIR=/tmp; mkdir -p gpurun_out/lo
KB_LAUNCH_DIAG=1 timeout -k 10 200 python3 tools/launch_overhead.py 3 > gpurun_out/lo/auto.json 2> gpurun_out/lo/auto.err || { tail gpurun_out/lo/auto.err; exit 1; }
cat gpurun_out/lo/auto.json
for i in 1 2; do
  for S in 20 200; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps $S --warmup 5 > gpurun_out/lo/b${S}_$i.json 2> gpurun_out/lo/b${S}_$i.err || { tail gpurun_out/lo/b${S}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/lo/b${S}_$i.json')); print('bench$S', round(d['value'],1), d['ms_per_step'], d['per_pass_median_ms'], d['python_wall_seconds'], d['device_warmup'])"
  done
done
