set -u
bash scripts/exp/gpu_ck.sh || exit 1
bash scripts/exp/bench_variants.sh "--steps 10 --warmup 3" ckint
