#!/usr/bin/env bash
# s27: affine-gap extension parity (new kernels), then the linear-gap suite (host-batch refactor)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s27; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_affine_gpu.py -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest_affine.log 2>&1 || { tail -60 $O/pytest_affine.log; exit 1; }
tail -1 $O/pytest_affine.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_abi.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
echo s27 done
