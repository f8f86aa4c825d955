#!/usr/bin/env bash
# s18: workspace cached in the context + dynamic budget; device CIGAR compaction in the mapper
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s18; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
B="timeout -k 10 600 python bench.py"
$B > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
$B --workload cfg3 --steps 3 --warmup 1 --no-cpu > $O/bench_cfg3.log 2>&1 || { tail -20 $O/bench_cfg3.log; exit 1; }
tail -1 $O/bench_cfg3.log
$B --workload cfg3map --steps 3 --warmup 1 > $O/bench_cfg3map.log 2>&1 || { tail -30 $O/bench_cfg3map.log; exit 1; }
tail -1 $O/bench_cfg3map.log
echo s18 done
