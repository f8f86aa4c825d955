set -u
bash scripts/exp/gpu_ck.sh || exit 1
bash scripts/exp/ck_prof.sh
