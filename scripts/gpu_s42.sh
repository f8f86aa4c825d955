#!/usr/bin/env bash
# s42: round-end check of the final code: full -m gpu suite, smoke, default bench, config-2 profile
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/s42; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail -30 $O/bench_cfg2.err; exit 1; }
tail -1 $O/bench_cfg2.json | cut -c1-200
bash scripts/profile.sh s42/r01n_cfg2 || exit 1
echo s42 done
