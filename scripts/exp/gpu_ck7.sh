set -u
timeout -k 10 200 python -u scripts/exp/ck_diff.py > gpurun_out/ck_diff.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/ck_diff.log | tail -40
exit $rc
