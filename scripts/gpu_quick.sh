#!/usr/bin/env bash
# Quick GPU loop: the parity tests of the path, then bench variants (BENCH_SPECS="args|args|...").
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_affine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-gpu or not gpu}" > gpurun_out/pytest_q.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_q.log
[ $rc -eq 0 ] || exit 1
IFS='|' read -ra SPECS <<< "${BENCH_SPECS:---steps 10 --warmup 2 --no-cpu --no-host}"
for spec in "${SPECS[@]}"; do
  timeout -k 10 300 python -u bench.py $spec > gpurun_out/w.json 2> gpurun_out/w.err
  rc=$?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/w.json').read().strip().splitlines()[-1]); print('[$spec]', d['value'], 'fill', d['fill_ms'], 'tb', d['traceback_ms'], 'parity', (d.get('parity') or {}).get('bit_exact'))" || { echo "[$spec] rc=$rc"; tail -5 gpurun_out/w.err; }
  [ $rc -le 1 ] || exit $rc
done
