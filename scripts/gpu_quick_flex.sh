set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "local or flex or digest or fuzz" > gpurun_out/pq.log 2>&1; rc=$?
tail -3 gpurun_out/pq.log; [ $rc -eq 0 ] || exit 1
NO_TESTS=1 bash scripts/gpu_evidence.sh cfg3_local cfg3 cfg2
