#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
SKIP_PROF=1 bash scripts/gpu_session.sh s3 && bash scripts/profile.sh p3
