#!/usr/bin/env bash
# s40: local walks track the cost (no STOP codes in the packed local fill): full -m gpu suite, smoke, bench
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/s40; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail -30 $O/bench_cfg2.err; exit 1; }
tail -1 $O/bench_cfg2.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['fill_ms'], d['traceback_ms'], d['parity'])"
timeout -k 10 400 python -u bench.py --related --no-cpu > $O/bench_cfg2_related.json 2> $O/bench_cfg2_related.err || { tail -30 $O/bench_cfg2_related.err; exit 1; }
tail -1 $O/bench_cfg2_related.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('related', d['value'], d['fill_ms'], d['traceback_ms'], d['parity'])"
echo s40 done
