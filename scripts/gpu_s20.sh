#!/usr/bin/env bash
# s20: flexible dual fill (ragged couples, rebased int16): parity + benches
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s20; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "flex" > $O/pytest_flex.log 2>&1 || { tail -40 $O/pytest_flex.log; exit 1; }
tail -2 $O/pytest_flex.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
B="timeout -k 10 600 python bench.py --no-cpu"
$B > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
$B --workload cfg3 --steps 3 --warmup 1 > $O/bench_cfg3.log 2>&1 || { tail -20 $O/bench_cfg3.log; exit 1; }
tail -1 $O/bench_cfg3.log | cut -c1-400
$B --workload cfg3map --steps 3 --warmup 1 > $O/bench_cfg3map.log 2>&1 || { tail -30 $O/bench_cfg3map.log; exit 1; }
tail -1 $O/bench_cfg3map.log
$B --workload cfg5 --steps 3 --warmup 1 > $O/bench_cfg5.log 2>&1 || { tail -20 $O/bench_cfg5.log; exit 1; }
tail -1 $O/bench_cfg5.log | cut -c1-400
echo s20 done
