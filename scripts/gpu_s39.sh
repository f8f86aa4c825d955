#!/usr/bin/env bash
# s39: affine M-run jumping walk + SGPR-base code stores: affine GPU tests, config-5 affine bench
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/s39; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_affine_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_affine.log 2>&1 || { tail -60 $O/pytest_affine.log; exit 1; }
tail -1 $O/pytest_affine.log
timeout -k 10 400 python -u bench.py --workload cfg5 --gap-open -2 --steps 3 --warmup 1 > $O/cfg5_affine.json 2> $O/cfg5_affine.err || { tail -30 $O/cfg5_affine.err; exit 1; }
tail -1 $O/cfg5_affine.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['fill_ms'], d['traceback_ms'], d['parity'])"
echo s39 done
