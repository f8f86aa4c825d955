#!/usr/bin/env bash
# s11: batched run writer + branch-light traceback: parity, fused/unfused benches, traceback profile
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s11; mkdir -p $O
SKIP_PROF=1 bash scripts/gpu_session.sh s11 || exit $?
grep -q ' passed' $O/pytest_gpu.log && ! grep -q 'failed' $O/pytest_gpu.log || { echo "parity failures; stop"; exit 0; }
B="timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-parity"
TA_FUSED_TRACEBACK=0 $B > $O/bench_unfused.log 2>&1 || exit $?
TA_FUSED_TRACEBACK=0 $B --related > $O/bench_unfused_related.log 2>&1 || exit $?
$B --related > $O/bench_related.log 2>&1 || exit $?
TA_FUSED_TRACEBACK=0 $B --mode global > $O/bench_unfused_global.log 2>&1 || exit $?
cd /tmp && TA_FUSED_TRACEBACK=0 timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_sq -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu --no-parity > $GRAFT_REPO_ROOT/$O/pmc_sq.log 2>&1 || exit $?
echo s11 done
