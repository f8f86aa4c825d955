#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel trace.
# Every GPU step has its own timeout; a crash / fault / timeout ends the
# session (no further GPU work), ordinary test failures do not.
# Usage: scripts/gpu_session.sh [tag]      (outputs under gpurun_out/<tag>/)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-s}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
fatal() { # exit codes that mean the GPU step crashed or hung
  case "$1" in 0|1|2|3|4|5) return 1 ;; *) return 0 ;; esac
}
run() { # run NAME TIMEOUT cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -5 "$OUT/$name.log" | tee -a "$OUT/session.log"
  if fatal $rc; then echo "FATAL step $name rc=$rc; stopping" | tee -a "$OUT/session.log"; exit $rc; fi
  return 0
}
rocminfo 2>/dev/null | grep -m1 -E 'gfx9[0-9]+' > "$OUT/gpu.txt" || true
run pytest_gpu 1200 python -m pytest tests -m gpu -q -rf
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps 10 --warmup 2
if [ "${SKIP_PROF:-0}" != 1 ]; then
  cd /tmp
  run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu --no-parity
  cd "$ROOT"
fi
echo "session done" | tee -a "$OUT/session.log"
