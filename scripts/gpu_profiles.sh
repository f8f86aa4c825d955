#!/usr/bin/env bash
# rocprofv3 evidence (kernel trace + PMC passes, scripts/profile.sh) for the
# named workloads, one after another: gpurun_out/<tag>_<name>/.
#   scripts/gpu_profiles.sh <tag> name...   (names: cfg2 cfg3 cfg3_local cfg5 cfg5_affine cfg5_100k cfg5_100k_affine)
set -u
TAG=$1; shift
declare -A ARGS=(
  [cfg2]=""
  [cfg3]="--workload cfg3 --steps 3 --warmup 1"
  [cfg3_local]="--workload cfg3 --mode local --steps 3 --warmup 1"
  [cfg5]="--workload cfg5 --pairs 8192"
  [cfg5_affine]="--workload cfg5 --pairs 4096 --gap-open -2"
  [cfg5_100k]="--workload cfg5 --pairs 100000 --steps 2 --warmup 1"
  [cfg5_100k_affine]="--workload cfg5 --pairs 100000 --gap-open -2 --steps 2 --warmup 1"
)
for n in "$@"; do
  bash scripts/profile.sh "${TAG}_$n" ${ARGS[$n]} || exit $?
  python3 scripts/prof_compact.py "gpurun_out/${TAG}_$n" || exit $?
done
