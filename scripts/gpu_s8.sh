#!/usr/bin/env bash
# s8: PMC profile of the dual fill kernel alone (unfused) and of the default (fused) path
set -u
cd "${GRAFT_REPO_ROOT:-.}"
TA_FUSED_TRACEBACK=0 bash scripts/profile.sh s8_unfused || exit $?
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/profile.sh s8_fused || exit $?
echo s8 done
