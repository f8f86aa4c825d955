#!/usr/bin/env bash
# s35: packed two-pair affine fill: affine GPU tests, then config-5 affine bench (open -2) dual vs int32
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/s35; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_affine_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_affine.log 2>&1 || { tail -60 $O/pytest_affine.log; exit 1; }
tail -1 $O/pytest_affine.log
timeout -k 10 400 python -u bench.py --workload cfg5 --gap-open -2 --steps 3 --warmup 1 > $O/cfg5_affine.json 2> $O/cfg5_affine.err || { tail -30 $O/cfg5_affine.err; exit 1; }
tail -1 $O/cfg5_affine.json
TA_AFFINE_DUAL=0 timeout -k 10 400 python -u bench.py --workload cfg5 --gap-open -2 --steps 3 --warmup 1 --no-cpu > $O/cfg5_affine_int32.json 2> $O/cfg5_affine_int32.err || { tail -30 $O/cfg5_affine_int32.err; exit 1; }
tail -1 $O/cfg5_affine_int32.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('int32', d['value'], d['fill_ms'], d['traceback_ms'])"
echo s35 done
