#!/usr/bin/env bash
# Builds libteam_alignment.so (gfx950 HIP kernels + C-ABI + team::Align shim)
# in-tree, and the test-only oracle libraries.  Used by __graft_entry__.build().
# ta_kernels.hip is compiled once per (fill mode, cigar) pair (TA_FILL_MODE,
# TA_FILL_CIGAR) and once for the traceback/compact kernels (TA_TU_MISC), in
# parallel; ta_dual.hip (packed two-pair fill) likewise per (mode, cigar).
set -euo pipefail
ROOT="$(cd "$(dirname "$0")" && pwd)"
CS="$ROOT/bioinfo1_amd/csrc"
OUT="${TA_OUT:-$ROOT/bioinfo1_amd/libteam_alignment.so}"  # (experiment variants: TA_OUT, TA_BUILD_DIR, TA_LIB_ONLY=1)
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
B="${TA_BUILD_DIR:-$ROOT/build}"
mkdir -p "$B"
FLAGS=(-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-function ${TA_EXTRA_FLAGS:-})
pids=()
# incremental: an object is rebuilt when its source or any csrc header is newer (TA_FORCE=1: always)
if [ "$(cat "$B/.flags" 2>/dev/null)" != "${FLAGS[*]}" ]; then TA_FORCE=1; fi  # other flags: rebuild all
echo "${FLAGS[*]}" > "$B/.flags"
stale() {  # stale <obj> <src>: missing, or older than its source / a header it includes (<obj>.d)
  [ "${TA_FORCE:-0}" = 1 ] || [ ! -f "$1" ] || [ ! -f "$1.d" ] || [ "$2" -nt "$1" ] || [ "$0" -nt "$1" ] && return 0
  local dep
  for dep in $(sed -e 's/^[^:]*://' -e 's/\\$//' "$1.d"); do
    case "$dep" in /opt/*|/usr/*) continue ;; esac
    [ "$dep" -nt "$1" ] && return 0
  done
  return 1
}
cc() {  # cc <obj> <src> <compiler args...>: background compile when stale (dependencies into <obj>.d)
  local o="$1" src="$2"; shift 2
  if stale "$o" "$src"; then "$@" -MD -MF "$o.d" -o "$o" & pids+=($!); fi
}
for m in 0 1 2; do
  for c in 0 1; do
    cc "$B/ta_fill_$m$c.o" "$CS/ta_kernels.hip" "$HIPCC" "${FLAGS[@]}" -DTA_FILL_MODE=$m -DTA_FILL_CIGAR=$c -c "$CS/ta_kernels.hip"
    cc "$B/ta_dual_$m$c.o" "$CS/ta_dual.hip" "$HIPCC" "${FLAGS[@]}" -DTA_DUAL_MODE=$m -DTA_DUAL_CIGAR=$c -c "$CS/ta_dual.hip"
  done
done
# the blocked-layout local fill (band walks) in a translation unit of its own
cc "$B/ta_dual_blk.o" "$CS/ta_dual.hip" "$HIPCC" "${FLAGS[@]}" -DTA_DUAL_MODE=1 -DTA_DUAL_CIGAR=1 -DTA_DUAL_BLK -c "$CS/ta_dual.hip"
# ... in the checkpoint layout (every mode), and the recomputing walks over it
for m in 0 1 2; do
  cc "$B/ta_dual_ck_$m.o" "$CS/ta_dual.hip" "$HIPCC" "${FLAGS[@]}" -DTA_DUAL_MODE=$m -DTA_DUAL_CIGAR=1 -DTA_DUAL_BLK -DTA_DUAL_CK=1 -c "$CS/ta_dual.hip"
done
cc "$B/ta_walk_ck.o" "$CS/ta_walk_ck.hip" "$HIPCC" "${FLAGS[@]}" -c "$CS/ta_walk_ck.hip"
for m in 0 1 2; do
  for c in 0 1; do
    cc "$B/ta_flex_$m$c.o" "$CS/ta_flex.hip" "$HIPCC" "${FLAGS[@]}" -DTA_FLEX_MODE=$m -DTA_FLEX_CIGAR=$c -c "$CS/ta_flex.hip"
  done
  # ... with checkpoints instead of codes (checkpoint plans)
  cc "$B/ta_flex_ck_$m.o" "$CS/ta_flex.hip" "$HIPCC" "${FLAGS[@]}" -DTA_FLEX_MODE=$m -DTA_FLEX_CIGAR=1 -DTA_FLEX_CK=1 -c "$CS/ta_flex.hip"
done
cc "$B/ta_misc.o" "$CS/ta_kernels.hip" "$HIPCC" "${FLAGS[@]}" -DTA_TU_MISC -c "$CS/ta_kernels.hip"
# affine-gap extension (fill + traceback kernels and its plan driver)
cc "$B/ta_affine.o" "$CS/ta_affine.hip" "$HIPCC" "${FLAGS[@]}" -c "$CS/ta_affine.hip"
cc "$B/ta_api.o" "$CS/ta_api.hip" "$HIPCC" "${FLAGS[@]}" -c "$CS/ta_api.hip"
cc "$B/ta_server.o" "$CS/ta_server.cpp" "$HIPCC" "${FLAGS[@]}" -x hip -c "$CS/ta_server.cpp"
cc "$B/shim.o" "$CS/team_alignment_shim.cpp" "$HIPCC" "${FLAGS[@]}" -x c++ -c "$CS/team_alignment_shim.cpp"
# host planner: plain C++ (also built with g++ under ASan/UBSan/TSan by tests/test_host_sanitizers.py)
cc "$B/ta_planner.o" "$CS/ta_planner.cpp" g++ -O2 -std=c++17 -fPIC -Wall -c "$CS/ta_planner.cpp"
# mapper stages (libteam_mapper.so) and the team_mapper_amd CLI
if [ "${TA_LIB_ONLY:-0}" != 1 ]; then
for f in tm_minimizers tm_match tm_chain; do
  cc "$B/$f.o" "$CS/$f.hip" "$HIPCC" "${FLAGS[@]}" -c "$CS/$f.hip"
done
for f in tm_api tm_fastx; do
  cc "$B/$f.o" "$CS/$f.cpp" "$HIPCC" "${FLAGS[@]}" -x hip -c "$CS/$f.cpp"
done
cc "$B/tm_main.o" "$CS/tm_main.cpp" "$HIPCC" "${FLAGS[@]}" -x c++ -c "$CS/tm_main.cpp"
fi
for p in "${pids[@]}"; do wait "$p"; done
"$HIPCC" -shared -fPIC --offload-arch=gfx950 "$B"/ta_fill_{0,1,2}{0,1}.o "$B"/ta_dual_{0,1,2}{0,1}.o "$B/ta_dual_blk.o" "$B"/ta_dual_ck_{0,1,2}.o "$B/ta_walk_ck.o" "$B"/ta_flex_{0,1,2}{0,1}.o "$B"/ta_flex_ck_{0,1,2}.o "$B/ta_misc.o" "$B/ta_affine.o" "$B/ta_api.o" "$B/ta_server.o" "$B/ta_planner.o" "$B/shim.o" \
  -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib -o "$OUT"
if [ "${TA_LIB_ONLY:-0}" = 1 ]; then echo "built $OUT"; exit 0; fi
PKG="$ROOT/bioinfo1_amd"
"$HIPCC" -shared -fPIC --offload-arch=gfx950 "$B"/tm_{minimizers,match,chain,api,fastx}.o -L"$PKG" -lteam_alignment -lz \
  -Wl,-rpath,'$ORIGIN' -o "$PKG/libteam_mapper.so"
"$HIPCC" --offload-arch=gfx950 "$B/tm_main.o" -L"$PKG" -lteam_mapper -lteam_alignment -Wl,-rpath,'$ORIGIN' \
  -o "$PKG/team_mapper_amd"
# the drop-in single-call measurement (bench.py --workload dropin), our side
g++ -std=c++17 -O3 -pthread -I"$ROOT/include" "$ROOT/scripts/dropin_bench.cpp" -L"$PKG" -lteam_alignment \
  -Wl,-rpath,"$PKG" -Wl,-rpath,'$ORIGIN/../bioinfo1_amd' -o "$B/dropin_amd"
make -s -C "$ROOT/oracle" >/dev/null
echo "built $OUT"
