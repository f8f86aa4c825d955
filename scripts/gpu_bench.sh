#!/usr/bin/env bash
# Bench variants only (BENCH_SPECS="args|args|..."), one line each.
set -u
mkdir -p gpurun_out
IFS='|' read -ra SPECS <<< "${BENCH_SPECS:---steps 10 --warmup 2 --no-cpu --no-host}"
for spec in "${SPECS[@]}"; do
  timeout -k 10 400 python -u bench.py $spec > gpurun_out/w.json 2> gpurun_out/w.err
  rc=$?
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/w.json') if l.startswith('{')][-1]); print('[$spec]', d['value'], 'fill', d.get('fill_ms'), 'tb', d.get('traceback_ms'), 'parity', (d.get('parity') or {}).get('bit_exact'))" || { echo "[$spec] rc=$rc"; tail -5 gpurun_out/w.err; }
  [ $rc -le 1 ] || exit $rc
done
