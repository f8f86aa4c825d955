#!/usr/bin/env bash
# s16: first GPU run of the mapper stages (minimizers, chaining, CLI vs reference PAF)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s16; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_mapper_gpu.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_mapper.log 2>&1
rc=$?
tail -40 $O/pytest_mapper.log
exit $rc
