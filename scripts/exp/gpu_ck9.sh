set -u
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "band_walk or ck_walk or digest" > gpurun_out/ck_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ck_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/ck_bench.json 2> gpurun_out/ck_bench.err || exit 1
grep '^{' gpurun_out/ck_bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], 'fill', d.get('fill_ms'), 'tb', d.get('traceback_ms'), d.get('parity'))"
BL_N=8,16,4096 bash scripts/exp/gpu_bl.sh
