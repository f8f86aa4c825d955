#!/usr/bin/env bash
# One GPU-box session of round evidence: the GPU test suite, then named bench
# runs (gpurun_out/<name>.json).  Every GPU step has its own time limit; a
# crash / abort / time-out ends the session.
# Usage: scripts/gpu_evidence.sh [name ...]   (default: all)
set -u
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
declare -A RUN=(
  [cfg2]=""  # (bench.py defaults: the driver's own run)
  [cfg3]="--workload cfg3 --steps 3 --warmup 1"
  [cfg3_local]="--workload cfg3 --mode local --steps 3 --warmup 1"
  [cfg3map]="--workload cfg3map --steps 2 --warmup 1"
  [cfg4]="--workload cfg4 --steps 5 --warmup 1"
  [cfg5_100k]="--workload cfg5 --pairs 100000 --steps 2 --warmup 1 --check-all"
  [cfg5_100k_affine]="--workload cfg5 --pairs 100000 --gap-open -2 --steps 2 --warmup 1 --check-all"
  [dropin]="--workload dropin"
)
ORDER=(cfg2 cfg3 cfg3_local cfg3map cfg4 cfg5_100k cfg5_100k_affine dropin)
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  ok $rc || exit $rc
fi
[ $# -gt 0 ] && ORDER=("$@")
for n in "${ORDER[@]}"; do
  timeout -k 10 500 python -u bench.py ${RUN[$n]} > gpurun_out/$n.json 2> gpurun_out/$n.err
  rc=$?
  python3 -c "import json; d=json.loads(open('gpurun_out/$n.json').read().strip().splitlines()[-1]); print('$n', d.get('value'), d.get('unit'), 'fill', d.get('fill_ms'), 'parity', (d.get('parity') or {}).get('bit_exact'))" || { echo "$n rc=$rc"; tail -5 gpurun_out/$n.err; }
  ok $rc || exit $rc
done
