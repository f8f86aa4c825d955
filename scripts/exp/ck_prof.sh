set -u
cp bioinfo1_amd/libteam_alignment.so /tmp/main_lib.so
cp build/exp/ckprof.so bioinfo1_amd/libteam_alignment.so
CK_LANES=${CK_LANES:-8} timeout -k 10 120 python -u scripts/exp/ck_prof.py > gpurun_out/ck_prof.log 2>&1
rc=$?
CK_LANES=${CK_LANES:-8} timeout -k 10 120 python -u scripts/exp/ck_prof.py --related >> gpurun_out/ck_prof.log 2>&1 || rc=1
cp /tmp/main_lib.so bioinfo1_amd/libteam_alignment.so
grep -v amdgpu.ids gpurun_out/ck_prof.log
exit $rc
