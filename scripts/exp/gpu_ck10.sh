set -u
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "band_walk or ck_walk or digest" > gpurun_out/ck_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ck_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_profiles.sh r05f cfg2
