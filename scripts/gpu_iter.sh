#!/usr/bin/env bash
# One GPU iteration (run on the box): GPU tests selected by PYTEST_K, bench lines
# (BENCH_SPECS="args|args"), then, when PMC_TAG is set, the PMC passes of the
# default workload (scripts/pmc_walk.sh) and, when TRACE_TAG is set, a kernel trace
# of the pipelined steps (scripts/exp/overlap_summary.py).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$PYTEST_K" \
    > gpurun_out/pt_iter.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 gpurun_out/pt_iter.log)"; [ $rc -eq 0 ] || exit 1
fi
IFS='|' read -ra SPECS <<< "${BENCH_SPECS:-}"
i=0
for spec in "${SPECS[@]}"; do
  i=$((i + 1))
  timeout -k 10 400 python -u bench.py $spec > gpurun_out/b$i.json 2> gpurun_out/b$i.err
  rc=$?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/b$i.json').read().strip().splitlines()[-1]); p=d.get('pipeline') or {}; print('[$spec]', d['value'], 'ms', d['ms_per_step'], 'fill', d['fill_ms'], 'tb', d['traceback_ms'], 'serial', p.get('serial_value'), 'parity', (d.get('parity') or {}).get('bit_exact'), 'slots', p.get('slots_bit_exact'))" \
    || { echo "[$spec] rc=$rc"; tail -5 gpurun_out/b$i.err; }
  [ $rc -eq 0 ] || exit 1
done
if [ -n "${PMC_TAG:-}" ]; then bash scripts/pmc_walk.sh "$PMC_TAG" ${PMC_ARGS:-} || exit 1; fi
if [ -n "${TRACE_TAG:-}" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/$TRACE_TAG" -o run \
    -- python3 "$PWD/bench.py" --steps 20 --warmup 2 --no-cpu --no-host --no-score-only --no-parity \
    > "gpurun_out/$TRACE_TAG.log" 2>&1 || exit 1
  python3 scripts/exp/overlap_summary.py "$(find gpurun_out/$TRACE_TAG -name '*kernel_trace.csv' | head -1)" \
    "gpurun_out/$TRACE_TAG/overlap.json"
fi
