#!/usr/bin/env bash
# s9: bit-plane pointer layout (VALU-only codes in the dual fill): parity, benches
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s9; mkdir -p $O
SKIP_PROF=1 bash scripts/gpu_session.sh s9 || exit $?
grep -q ' passed' $O/pytest_gpu.log && ! grep -q 'failed' $O/pytest_gpu.log || { echo "parity failures; stop"; exit 0; }
B="timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-parity"
TA_DUAL=0 $B > $O/bench_nodual.log 2>&1 || exit $?
TA_FUSED_TRACEBACK=0 $B > $O/bench_unfused.log 2>&1 || exit $?
$B --no-cigar > $O/bench_nocigar.log 2>&1 || exit $?
$B --mode global > $O/bench_global.log 2>&1 || exit $?
$B --mode semiGlobal > $O/bench_semi.log 2>&1 || exit $?
echo s9 done
