#!/usr/bin/env bash
# s46: full -m gpu suite, config 3 / 3-mapper / 5 benches with the pass-major flex tickets, config-3 profile
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/s46; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py --workload cfg3 --steps 3 --warmup 1 > $O/cfg3.json 2> $O/cfg3.err || { tail -30 $O/cfg3.err; exit 1; }
tail -1 $O/cfg3.json | cut -c1-200
timeout -k 10 500 python -u bench.py --workload cfg3map --steps 3 --warmup 1 > $O/cfg3map.json 2> $O/cfg3map.err || { tail -30 $O/cfg3map.err; exit 1; }
tail -1 $O/cfg3map.json | cut -c1-200
timeout -k 10 400 python -u bench.py --workload cfg5 --steps 3 --warmup 1 > $O/cfg5.json 2> $O/cfg5.err || { tail -30 $O/cfg5.err; exit 1; }
tail -1 $O/cfg5.json | cut -c1-200
timeout -k 10 400 python -u bench.py --workload cfg5 --gap-open -2 --steps 3 --warmup 1 > $O/cfg5_affine.json 2> $O/cfg5_affine.err || { tail -30 $O/cfg5_affine.err; exit 1; }
tail -1 $O/cfg5_affine.json | cut -c1-200
bash scripts/profile.sh s46/r01n_cfg3 --workload cfg3 || exit 1
echo s46 done
