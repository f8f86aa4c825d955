# run scripts/exp/walk_ab.py with each library variant in AB_VARIANTS (build/exp/<v>.so; "main" = the build)
# Stops at the first failing run (a fault or time limit ends the GPU work of the call).
set -u
cp bioinfo1_amd/libteam_alignment.so build/exp/main.so
rc=0
for v in ${AB_VARIANTS:-main}; do
  cp build/exp/$v.so bioinfo1_amd/libteam_alignment.so
  echo "== $v" >> gpurun_out/walk_ab.log
  timeout -k 10 150 python -u scripts/exp/walk_ab.py >> gpurun_out/walk_ab.log 2>&1 || { rc=1; break; }
done
cp build/exp/main.so bioinfo1_amd/libteam_alignment.so
grep -v "amdgpu.ids" gpurun_out/walk_ab.log | tail -40
exit $rc
