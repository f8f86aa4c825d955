set -u
for k in 1 2; do
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "band_walk or ck_walk" > gpurun_out/ck_rep$k.log 2>&1
echo "run $k rc=$?"; grep -E "passed|failed|^FAILED" gpurun_out/ck_rep$k.log | tail -5
done
timeout -k 10 200 python -u scripts/exp/ck_diff.py > gpurun_out/ck_diff.log 2>&1; grep -v amdgpu gpurun_out/ck_diff.log | tail -8
