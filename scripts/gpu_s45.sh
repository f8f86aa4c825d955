#!/usr/bin/env bash
# s45: flexible fill polls each record chunk just in time (no next-chunk prefetch): flex parity, config 3
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/s45; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_mapper_gpu.py -m gpu -x -v -k "flex or digest or config3 or config5 or stale or mapper or paf" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --workload cfg3 --steps 3 --warmup 1 --no-cpu > $O/cfg3.json 2> $O/cfg3.err || { tail -30 $O/cfg3.err; exit 1; }
tail -1 $O/cfg3.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg3', d['value'], d['fill_ms'], d['traceback_ms'], d['parity'])"
echo s45 done
