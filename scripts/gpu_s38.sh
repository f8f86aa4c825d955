#!/usr/bin/env bash
# s38: config-5 linear profile (traffic/valu), then the round's bench set with CPU baselines
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/s38; mkdir -p $O
bash scripts/profile.sh s38/r01n_cfg5 --workload cfg5 || exit 1
cd "$R"
timeout -k 10 400 python -u bench.py --workload cfg5 --steps 3 --warmup 1 > $O/cfg5.json 2> $O/cfg5.err || { tail -30 $O/cfg5.err; exit 1; }
tail -1 $O/cfg5.json | cut -c1-300
timeout -k 10 400 python -u bench.py --workload cfg3 --steps 3 --warmup 1 > $O/cfg3.json 2> $O/cfg3.err || { tail -30 $O/cfg3.err; exit 1; }
tail -1 $O/cfg3.json | cut -c1-300
timeout -k 10 500 python -u bench.py --workload cfg3map --steps 3 --warmup 1 > $O/cfg3map.json 2> $O/cfg3map.err || { tail -30 $O/cfg3map.err; exit 1; }
tail -1 $O/cfg3map.json | cut -c1-300
timeout -k 10 400 python -u bench.py --workload cfg2 --related > $O/cfg2_related.json 2> $O/cfg2_related.err || { tail -30 $O/cfg2_related.err; exit 1; }
tail -1 $O/cfg2_related.json | cut -c1-300
timeout -k 10 400 python -u bench.py --workload cfg2 --no-cigar --no-cpu > $O/cfg2_score.json 2> $O/cfg2_score.err || { tail -30 $O/cfg2_score.err; exit 1; }
tail -1 $O/cfg2_score.json | cut -c1-300
echo s38 done
