#!/usr/bin/env bash
# s10: PMC profile of the bit-plane dual fill (unfused) and score-only
set -u
cd "${GRAFT_REPO_ROOT:-.}"
TA_FUSED_TRACEBACK=0 bash scripts/profile.sh s10_unfused || exit $?
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/profile.sh s10_nocigar --no-cigar || exit $?
echo s10 done
