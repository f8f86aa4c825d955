#!/usr/bin/env bash
# s13: packed branch-free best tracking, hoisted chunk reloads, unfused default for dual plans
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s13; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
B="timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu"
$B > $O/bench.log 2>&1 || exit $?
$B --no-parity --mode semiGlobal > $O/bench_semi.log 2>&1 || exit $?
$B --no-parity --mode global > $O/bench_global.log 2>&1 || exit $?
$B --related > $O/bench_related.log 2>&1 || exit $?
$B --no-parity --no-cigar > $O/bench_nocigar.log 2>&1 || exit $?
TA_DUAL=0 $B --no-parity > $O/bench_nodual.log 2>&1 || exit $?
TA_DUAL=0 TA_FUSED_TRACEBACK=0 $B --no-parity > $O/bench_nodual_unfused.log 2>&1 || exit $?
echo s13 done
