set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
D=gpurun_out/pmc5x; rm -rf $D; mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_spline.py > $D/t.log 2>&1 || { tail -20 $D/t.log; exit 1; }
tail -1 $D/t.log
for i in 1 2; do timeout -k 10 120 python bench.py --config 5 --steps 200 --warmup 20 --no-cpu-baseline > $D/b$i.json || exit 1; python3 -c "import json; d=json.load(open('$D/b$i.json')); print(d['value'], d['roofline']['avg_ms'])"; done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$D/pmc_fetch -o pmc -- python3 bench.py --config 5 --steps 20 --warmup 2 --no-cpu-baseline > $D/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$D/pmc_write -o pmc -- python3 bench.py --config 5 --steps 20 --warmup 2 --no-cpu-baseline > $D/write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $D $D/pmc_traffic_c5.json 5 > /dev/null && grep -A6 "k_sp_assemble" $D/pmc_traffic_c5.json | grep hbm
