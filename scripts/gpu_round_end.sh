#!/usr/bin/env bash
# Round evidence in one GPU session: smoke(), then scripts/gpu_evidence.sh
# (GPU test suite + every named bench run).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_evidence.sh "$@"
