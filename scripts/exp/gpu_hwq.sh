# config 2 pipelined bench at several hardware-queue counts and step counts
set -o pipefail
mkdir -p gpurun_out
for q in 4 8 16; do
  for st in 10 30; do
    TA_BENCH_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --steps $st --warmup 3 --no-cpu --no-host --no-score-only --no-parity > gpurun_out/hwq.json 2> gpurun_out/hwq.err
    rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/hwq.err; exit $rc; }
    grep '^{' gpurun_out/hwq.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['pipeline']; print('q=$q steps=$st', d['ms_per_step'], 'serial', p['serial_ms_per_step'], p['slots_bit_identical'])"
  done
done
