#!/usr/bin/env bash
# s12: branch-free traceback iteration: parity + traceback timing/PMC
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s12; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
B="timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-parity"
$B > $O/bench.log 2>&1 || exit $?
TA_FUSED_TRACEBACK=0 $B > $O/bench_unfused.log 2>&1 || exit $?
TA_FUSED_TRACEBACK=0 $B --related > $O/bench_unfused_related.log 2>&1 || exit $?
cd /tmp && TA_FUSED_TRACEBACK=0 timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_sq -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu --no-parity > $GRAFT_REPO_ROOT/$O/pmc_sq.log 2>&1 || exit $?
echo s12 done
