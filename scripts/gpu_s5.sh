#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
SKIP_PROF=1 bash scripts/gpu_session.sh s5 || exit $?
TA_FUSED_TRACEBACK=0 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/s5/bench_unfused.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --related > gpurun_out/s5/bench_related.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-cigar > gpurun_out/s5/bench_nocigar.log 2>&1 || exit $?
bash scripts/profile.sh p5
