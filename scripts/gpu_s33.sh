#!/usr/bin/env bash
# s33: stale-record fix: the failing digest sequence first (fresh process), then the full -m gpu suite,
# smoke, default bench, profile r01n
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/s33; mkdir -p $O
timeout -k 10 300 python -u scripts/diag/digest_seq.py > $O/diag.log 2>&1 || { tail -40 $O/diag.log; exit 1; }
grep -c "bad 0" $O/diag.log; grep "bad [1-9]" $O/diag.log
for k in 1; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "pipelined or staged or device_plan or digest or stale" --timeout 200 --timeout-method thread > $O/pytest_digest_$k.log 2>&1 || { tail -40 $O/pytest_digest_$k.log; exit 1; }
  tail -1 $O/pytest_digest_$k.log
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail -30 $O/bench_cfg2.err; exit 1; }
tail -1 $O/bench_cfg2.json
timeout -k 10 400 python -u bench.py --workload cfg3 --steps 3 --warmup 1 --no-cpu > $O/bench_cfg3.json 2> $O/bench_cfg3.err || { tail -30 $O/bench_cfg3.err; exit 1; }
tail -1 $O/bench_cfg3.json
bash scripts/profile.sh s33/r01n_cfg2 || exit 1
echo s33 done
