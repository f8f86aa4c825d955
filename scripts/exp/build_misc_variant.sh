#!/usr/bin/env bash
# Experiment build: recompile only the traceback TU (ta_kernels.hip, TA_TU_MISC)
# with extra flags and relink against the objects of the last build.sh run.
#   scripts/exp/build_misc_variant.sh <name> <flags...>  -> build/exp/<name>.so
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
CS="$ROOT/bioinfo1_amd/csrc"; B="$ROOT/build"
NAME=$1; shift
mkdir -p "$B/exp"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-function "$@" \
  -DTA_TU_MISC -c "$CS/ta_kernels.hip" -o "$B/exp/misc_$NAME.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "$B"/ta_fill_{0,1,2}{0,1}.o "$B"/ta_dual_{0,1,2}{0,1}.o "$B/ta_dual_blk.o" \
  "$B"/ta_flex_{0,1,2}{0,1}.o "$B/exp/misc_$NAME.o" "$B/ta_affine.o" "$B/ta_api.o" "$B/ta_server.o" "$B/ta_planner.o" "$B/shim.o" \
  -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib -o "$B/exp/$NAME.so"
echo "built $B/exp/$NAME.so"
