set -u
cp bioinfo1_amd/libteam_alignment.so build/exp/_orig.so
cp build/exp/lwprof.so bioinfo1_amd/libteam_alignment.so
timeout -k 10 200 python -u scripts/exp/lw_prof.py > gpurun_out/lwp.log 2>&1; rc=$?
timeout -k 10 200 python -u scripts/exp/lw_prof.py --related >> gpurun_out/lwp.log 2>&1
cp build/exp/_orig.so bioinfo1_amd/libteam_alignment.so
cat gpurun_out/lwp.log | grep iter
exit $rc
