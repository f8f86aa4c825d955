#!/usr/bin/env bash
# Affine check + bench on the GPU box: the affine GPU tests, then config 5
# affine at the stated size (every CIGAR checked) and config 5 linear.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_affine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_aff.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_aff.log
[ $rc -eq 0 ] || exit 1
NO_TESTS=1 bash scripts/gpu_evidence.sh "$@"
