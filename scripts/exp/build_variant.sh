#!/usr/bin/env bash
# Experiment build: recompile some translation units with extra flags and link
# them with the other objects of the last build.sh run (same sources):
#   scripts/exp/build_variant.sh <name> "<units>" <flags...>  -> build/exp/<name>.so
# units: dual_blk dual_ck_M flex_ck_M walk_ck dual_MC flex_MC fill_MC (M mode 0-2, C cigar 0/1) misc affine
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
CS="$ROOT/bioinfo1_amd/csrc"; B="$ROOT/build"
NAME=$1; UNITS=$2; shift 2
mkdir -p "$B/exp/$NAME"
FLAGS=(-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-function "$@")
objs=()
for o in "$B"/ta_fill_{0,1,2}{0,1}.o "$B"/ta_dual_{0,1,2}{0,1}.o "$B/ta_dual_blk.o" "$B"/ta_dual_ck_{0,1,2}.o "$B/ta_walk_ck.o" \
         "$B"/ta_flex_{0,1,2}{0,1}.o "$B"/ta_flex_ck_{0,1,2}.o \
         "$B/ta_misc.o" "$B/ta_affine.o" "$B/ta_api.o" "$B/ta_server.o" "$B/ta_planner.o" "$B/shim.o"; do
  objs+=("$o")
done
pids=()
for u in $UNITS; do
  out="$B/exp/$NAME/ta_$u.o"
  case "$u" in
    dual_blk) args=(-DTA_DUAL_MODE=1 -DTA_DUAL_CIGAR=1 -DTA_DUAL_BLK -c "$CS/ta_dual.hip") ;;
    dual_ck_?) args=(-DTA_DUAL_MODE=${u:8:1} -DTA_DUAL_CIGAR=1 -DTA_DUAL_BLK -DTA_DUAL_CK=1 -c "$CS/ta_dual.hip") ;;
    flex_ck_?) args=(-DTA_FLEX_MODE=${u:8:1} -DTA_FLEX_CIGAR=1 -DTA_FLEX_CK=1 -c "$CS/ta_flex.hip") ;;
    walk_ck) args=(-c "$CS/ta_walk_ck.hip") ;;
    dual_??) args=(-DTA_DUAL_MODE=${u:5:1} -DTA_DUAL_CIGAR=${u:6:1} -c "$CS/ta_dual.hip") ;;
    flex_??) args=(-DTA_FLEX_MODE=${u:5:1} -DTA_FLEX_CIGAR=${u:6:1} -c "$CS/ta_flex.hip") ;;
    fill_??) args=(-DTA_FILL_MODE=${u:5:1} -DTA_FILL_CIGAR=${u:6:1} -c "$CS/ta_kernels.hip") ;;
    misc) args=(-DTA_TU_MISC -c "$CS/ta_kernels.hip") ;;
    affine) args=(-c "$CS/ta_affine.hip") ;;
    *) echo "unknown unit $u"; exit 2 ;;
  esac
  /opt/rocm/bin/hipcc "${FLAGS[@]}" "${args[@]}" -o "$out" & pids+=($!)
  for k in "${!objs[@]}"; do [ "${objs[$k]}" = "$B/ta_$u.o" ] && objs[$k]="$out"; done
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "${objs[@]}" -L/opt/rocm/lib -lrocprofiler-sdk-roctx \
  -Wl,-rpath,/opt/rocm/lib -o "$B/exp/$NAME.so"
echo "built $B/exp/$NAME.so"
