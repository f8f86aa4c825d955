#!/usr/bin/env bash
# s14: re-entry sanity on the restored tree: gpu parity tests, smoke, default bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s14; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
echo s14 done
