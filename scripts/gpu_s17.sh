#!/usr/bin/env bash
# s17: mapper tests (two-size chain kernel) + config 3 end-to-end mapper bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s17; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_mapper_gpu.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_mapper.log 2>&1 || { tail -40 $O/pytest_mapper.log; exit 1; }
tail -3 $O/pytest_mapper.log
timeout -k 10 600 python bench.py --workload cfg3map --steps 3 --warmup 1 > $O/bench_cfg3map.log 2>&1 || { tail -30 $O/bench_cfg3map.log; exit 1; }
tail -1 $O/bench_cfg3map.log
echo s17 done
