#!/usr/bin/env bash
# s7: dual kernel with '-' fallback + waves_per_eu(5): parity, benches, 2-rank gloo rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s7; mkdir -p $O
SKIP_PROF=1 bash scripts/gpu_session.sh s7 || exit $?
grep -q ' passed' $O/pytest_gpu.log && ! grep -q 'failed' $O/pytest_gpu.log || { echo "parity failures; stop"; exit 0; }
B="timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-parity"
TA_DUAL=0 $B > $O/bench_nodual.log 2>&1 || exit $?
TA_FUSED_TRACEBACK=0 $B > $O/bench_unfused.log 2>&1 || exit $?
$B --no-cigar > $O/bench_nocigar.log 2>&1 || exit $?
$B --related > $O/bench_related.log 2>&1 || exit $?
$B --mode global > $O/bench_global.log 2>&1 || exit $?
$B --mode semiGlobal > $O/bench_semi.log 2>&1 || exit $?
TA_BENCH_ONE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu > $O/trun2.log 2>&1 || exit $?
echo s7 done
