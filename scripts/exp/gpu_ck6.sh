set -u
cp bioinfo1_amd/libteam_alignment.so /tmp/main_lib.so
cp build/exp/cknopf.so bioinfo1_amd/libteam_alignment.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "band_walk or ck_walk" > gpurun_out/ck_nopf.log 2>&1
rc=$?
cp /tmp/main_lib.so bioinfo1_amd/libteam_alignment.so
tail -3 gpurun_out/ck_nopf.log
exit $rc
