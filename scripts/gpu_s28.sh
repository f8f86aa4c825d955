#!/usr/bin/env bash
# s28: fresh-container re-verification: full -m gpu suite, smoke, default bench, affine config-5 bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s28; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail -30 $O/bench_cfg2.err; exit 1; }
tail -1 $O/bench_cfg2.json
timeout -k 10 400 python -u bench.py --workload cfg5 --gap-open 2 --steps 3 --warmup 1 > $O/bench_cfg5_affine.json 2> $O/bench_cfg5_affine.err || { tail -30 $O/bench_cfg5_affine.err; exit 1; }
tail -1 $O/bench_cfg5_affine.json
echo s28 done
