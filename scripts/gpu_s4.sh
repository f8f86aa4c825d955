#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/s4
rocprofv3 -L > gpurun_out/s4/counters.txt 2>&1 || true
SKIP_PROF=1 bash scripts/gpu_session.sh s4 && bash scripts/profile.sh p4
