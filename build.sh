#!/usr/bin/env bash
# Builds libteam_alignment.so (gfx950 HIP kernels + C-ABI + team::Align shim)
# in-tree, and the test-only oracle libraries.  Used by __graft_entry__.build().
set -euo pipefail
ROOT="$(cd "$(dirname "$0")" && pwd)"
CS="$ROOT/bioinfo1_amd/csrc"
OUT="$ROOT/bioinfo1_amd/libteam_alignment.so"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
mkdir -p "$ROOT/build"
FLAGS=(-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result)
"$HIPCC" "${FLAGS[@]}" -c "$CS/ta_kernels.hip" -o "$ROOT/build/ta_kernels.o" &
"$HIPCC" "${FLAGS[@]}" -c "$CS/ta_api.hip" -o "$ROOT/build/ta_api.o" &
"$HIPCC" "${FLAGS[@]}" -x c++ -c "$CS/team_alignment_shim.cpp" -o "$ROOT/build/shim.o" &
wait %1 && wait %2 && wait %3
"$HIPCC" -shared -fPIC --offload-arch=gfx950 "$ROOT/build/ta_kernels.o" "$ROOT/build/ta_api.o" "$ROOT/build/shim.o" -o "$OUT"
make -s -C "$ROOT/oracle" >/dev/null
echo "built $OUT"
