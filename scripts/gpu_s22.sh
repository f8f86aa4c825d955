#!/usr/bin/env bash
# s22: int32 singles beside the packed fill (aux stream); cfg3 benches + kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s22; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1 || { tail -40 $O/pytest_parity.log; exit 1; }
tail -1 $O/pytest_parity.log
B="timeout -k 10 600 python bench.py --no-cpu"
$B --workload cfg3 --steps 3 --warmup 1 > $O/bench_cfg3.log 2>&1 || { tail -20 $O/bench_cfg3.log; exit 1; }
tail -1 $O/bench_cfg3.log | cut -c1-300
$B --workload cfg3map --steps 3 --warmup 1 > $O/bench_cfg3map.log 2>&1 || { tail -20 $O/bench_cfg3map.log; exit 1; }
tail -1 $O/bench_cfg3map.log | cut -c1-300
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg3 -o run -- python3 bench.py --workload cfg3 --steps 1 --warmup 0 --no-cpu --no-parity > $O/prof_cfg3.log 2>&1 || { tail -30 $O/prof_cfg3.log; exit 1; }
echo s22 done
