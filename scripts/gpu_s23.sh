#!/usr/bin/env bash
# s23: staged plans (traceback stage k beside fill stage k+1): parity + cfg2 bench over TA_STAGES
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s23; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for st in 1 2 4 8; do
  TA_STAGES=$st timeout -k 10 300 python bench.py --no-cpu > $O/bench_st$st.log 2>&1 || { tail -20 $O/bench_st$st.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_st$st.log').read().strip().splitlines()[-1]); print('stages $st', d['value'], d['ms_per_step'], d['fill_ms'], d['traceback_ms'], d['chunks'], d['parity'])"
done
echo s23 done
