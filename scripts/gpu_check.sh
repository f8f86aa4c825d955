#!/usr/bin/env bash
# One GPU-box session: GPU tests, then (only if they ended normally, pass or
# fail) a default bench line and the drop-in measurement.  Every GPU step has
# its own time limit; a crash / abort / time-out ends the session.
set -u
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
ok $rc || exit $rc
if [ -n "${DROPIN:-}" ]; then
  timeout -k 10 300 python -u bench.py --workload dropin > gpurun_out/dropin.json 2> gpurun_out/dropin.err
  rc=$?; echo "dropin rc=$rc"; cat gpurun_out/dropin.json; tail -3 gpurun_out/dropin.err
fi
