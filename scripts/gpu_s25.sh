#!/usr/bin/env bash
# s25: multi-pass equal-shape couples through the pipelined flexible fill (config 5)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s25; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "flex" > $O/pytest_flex.log 2>&1 || { tail -40 $O/pytest_flex.log; exit 1; }
tail -1 $O/pytest_flex.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
B="timeout -k 10 600 python bench.py --no-cpu"
for w in cfg5 cfg2; do
  $B --workload $w --steps 3 --warmup 1 > $O/bench_$w.log 2>&1 || { tail -20 $O/bench_$w.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$w.log').read().strip().splitlines()[-1]); print('$w', d['value'], d['ms_per_step'], d.get('fill_ms'), d.get('stage_ms'), d.get('parity'))"
done
echo s25 done
