#!/usr/bin/env bash
# s41: final config-2 profile (trace + PMC) of the round's code, then the default bench line
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/s41; mkdir -p $O
bash scripts/profile.sh s41/r01n_cfg2 || exit 1
cd "$R"
timeout -k 10 400 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail -30 $O/bench_cfg2.err; exit 1; }
tail -1 $O/bench_cfg2.json | cut -c1-200
echo s41 done
