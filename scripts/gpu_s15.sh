#!/usr/bin/env bash
# s15: config 3 / config 5 property + digest tests, bench lines for cfg2 / cfg3 / cfg5
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s15; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 400 python bench.py --workload cfg3 --steps 3 --warmup 1 > $O/bench_cfg3.log 2>&1 || { tail -20 $O/bench_cfg3.log; exit 1; }
tail -1 $O/bench_cfg3.log
timeout -k 10 400 python bench.py --workload cfg5 --steps 3 --warmup 1 > $O/bench_cfg5.log 2>&1 || { tail -20 $O/bench_cfg5.log; exit 1; }
tail -1 $O/bench_cfg5.log
echo s15 done
