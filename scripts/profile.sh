#!/usr/bin/env bash
# rocprofv3 evidence for bench.py's default workload (run on the GPU box):
#   kernel trace + stats, then one --pmc pass per counter group (the guide's
#   rule: FETCH_SIZE and WRITE_SIZE in separate passes; no --pmc together
#   with trace domains).  Summaries -> gpurun_out/<tag>/prof_*/.
# Usage: scripts/profile.sh <tag> [bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-p}"; shift || true
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
# --serial: one batch after the other, so that no two kernels' durations and
# counters overlap (the pipelined steps run a walk beside the next fill)
BARGS=(--steps 20 --warmup 3 --serial --no-cpu --no-parity --no-host --no-score-only "$@")
step() { # name timeout args...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a "$OUT/profile.log"
  timeout -k 10 "$to" rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 "$ROOT/bench.py" "${BARGS[@]}" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/profile.log"
  case $rc in 0) ;; *) echo "stopping after $name" | tee -a "$OUT/profile.log"; exit $rc ;; esac
}
step prof_trace 600 --kernel-trace --stats
step prof_fetch 600 --pmc FETCH_SIZE
step prof_write 600 --pmc WRITE_SIZE
step prof_sq 600 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES
step prof_busy 600 --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_WR
step prof_wait 600 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY
echo "profile done" | tee -a "$OUT/profile.log"
