#!/usr/bin/env bash
# s19: 2-rank gloo rehearsal of the config-4 mapper path on one GPU; kernel trace of cfg3map
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s19; mkdir -p $O
export TA_BENCH_ONE_GPU=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --workload cfg3map --pairs 400 --steps 2 --warmup 1 --dist-backend gloo > $O/bench_cfg4_gloo2.log 2>&1 || { tail -30 $O/bench_cfg4_gloo2.log; exit 1; }
tail -1 $O/bench_cfg4_gloo2.log
unset TA_BENCH_ONE_GPU
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg3map -o run -- python3 bench.py --workload cfg3map --steps 2 --warmup 1 --no-cpu > $O/prof_cfg3map.log 2>&1 || { tail -30 $O/prof_cfg3map.log; exit 1; }
tail -1 $O/prof_cfg3map.log
find $O/prof_cfg3map -name "*kernel_stats.csv" | head -3
echo s19 done
