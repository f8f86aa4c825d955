set -u
bash scripts/profile.sh r02b_cfg2 && bash scripts/profile.sh r02b_cfg3local --workload cfg3 --mode local
