#!/usr/bin/env bash
# Quick rocprofv3 passes of bench.py (GPU box): kernel trace + two SQ counter
# passes -> gpurun_out/<tag>/.   scripts/exp/prof_quick.sh <tag> [bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
TAG="${1:-q}"; shift || true
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BARGS=(--steps 3 --warmup 1 --no-cpu --no-parity --no-host --no-score-only "$@")
step() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 "$ROOT/bench.py" "${BARGS[@]}" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
step trace --kernel-trace --stats
step sq --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES
step sq2 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM
python3 "$ROOT/scripts/exp/prof_quick_sum.py" "$OUT"
