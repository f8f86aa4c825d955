#!/usr/bin/env bash
# s6: dual-kernel parity + benches (dual on/off, score-only), torchrun rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s6; mkdir -p $O
SKIP_PROF=1 bash scripts/gpu_session.sh s6 || exit $?
grep -q ' passed' $O/pytest_gpu.log && ! grep -q 'failed' $O/pytest_gpu.log || { echo "parity failures; stop"; exit 0; }
TA_DUAL=0 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $O/bench_nodual.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-cigar > $O/bench_nocigar.log 2>&1 || exit $?
TA_DUAL=0 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-cigar > $O/bench_nocigar_nodual.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu > $O/trun1.log 2>&1 || exit $?
TA_BENCH_ONE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu > $O/trun2.log 2>&1 || exit $?
echo s6 done
