#!/usr/bin/env bash
# s34: N>1 bench path rehearsal on one GPU (2 ranks, gloo, TA_BENCH_ONE_GPU=1), plain and --pipeline
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/s34; mkdir -p $O
export TA_BENCH_ONE_GPU=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo > $O/bench_n2.json 2> $O/bench_n2.err || { tail -30 $O/bench_n2.err; exit 1; }
tail -1 $O/bench_n2.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --pipeline > $O/bench_n2_pipe.json 2> $O/bench_n2_pipe.err || { tail -30 $O/bench_n2_pipe.err; exit 1; }
tail -1 $O/bench_n2_pipe.json
echo s34 done
