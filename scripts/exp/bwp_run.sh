# band-walk phase profiles (scripts/exp/bw_prof.py) of each TA_BW_PROF variant in BWP_VARIANTS;
# stops at the first failing run.
set -u
cp bioinfo1_amd/libteam_alignment.so build/exp/_orig.so
rc=0
for v in ${BWP_VARIANTS:-bwprof}; do
  cp build/exp/$v.so bioinfo1_amd/libteam_alignment.so
  echo "== $v" >> gpurun_out/bwp.log
  timeout -k 10 100 python -u scripts/exp/bw_prof.py >> gpurun_out/bwp.log 2>&1 || { rc=1; break; }
  timeout -k 10 100 python -u scripts/exp/bw_prof.py --related >> gpurun_out/bwp.log 2>&1 || { rc=1; break; }
done
cp build/exp/_orig.so bioinfo1_amd/libteam_alignment.so
grep "iter 2\|==" gpurun_out/bwp.log
exit $rc
