# DevicePipeline A/B on config 2 (and config 3 / affine when PIPE_ALL=1)
set -o pipefail
mkdir -p gpurun_out
show() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:40], d['value'], 'h2h', (d.get('host_to_host') or {}).get('value'), (d.get('host_to_host') or {}).get('parity',{}).get('bit_exact'), d['ms_per_step'], 'fill', d.get('fill_ms'), 'tb', d.get('traceback_ms'), 'pipe', d.get('pipeline'), 'parity', (d.get('parity') or {}).get('bit_exact'))"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "pipeline" > gpurun_out/pipe_tests.log 2>&1
rc=$?; tail -8 gpurun_out/pipe_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu ${HOSTFLAG---no-host} --no-score-only > gpurun_out/pipe_cfg2.json 2> gpurun_out/pipe_cfg2.err
rc=$?; tail -3 gpurun_out/pipe_cfg2.err; show gpurun_out/pipe_cfg2.json; [ $rc -eq 0 ] || exit $rc
if [ "${PIPE_ALL:-0}" = 1 ]; then
  for w in "--workload cfg3" "--workload cfg3 --mode local" "--gap-open 2 --scoring 1,-1,-1"; do
    timeout -k 10 300 python -u bench.py $w --steps 10 --warmup 2 --no-cpu --no-host --no-score-only > gpurun_out/pipe_x.json 2> gpurun_out/pipe_x.err
    rc=$?; tail -2 gpurun_out/pipe_x.err; show gpurun_out/pipe_x.json; [ $rc -eq 0 ] || exit $rc
  done
fi
exit 0
