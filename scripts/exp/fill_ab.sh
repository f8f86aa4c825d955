set -u
cp bioinfo1_amd/libteam_alignment.so build/exp/main.so
rc=0
for v in main ck main ck; do
  cp build/exp/$v.so bioinfo1_amd/libteam_alignment.so
  echo "== $v" >> gpurun_out/fill_ab.log
  timeout -k 10 120 python -u scripts/exp/fill_ab.py >> gpurun_out/fill_ab.log 2>&1 || { rc=1; break; }
done
cp build/exp/main.so bioinfo1_amd/libteam_alignment.so
grep -v "amdgpu.ids" gpurun_out/fill_ab.log | tail -20
exit $rc
