set -u
BL_SHAPES=1000 BL_N=${BL_N:-8,16,64} BL_FLAGS=0,256 timeout -k 10 300 python -u scripts/exp/batch_latency.py > gpurun_out/bl_ck.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/bl_ck.log; exit $rc
