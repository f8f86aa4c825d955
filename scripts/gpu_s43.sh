#!/usr/bin/env bash
# s43: config-5 slice size (occupancy): 2000 vs 4096 vs 8192 pairs, linear and affine
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/s43; mkdir -p $O
for P in 4096 8192; do
  timeout -k 10 400 python -u bench.py --workload cfg5 --pairs $P --steps 3 --warmup 1 --no-cpu > $O/cfg5_$P.json 2> $O/cfg5_$P.err || { tail -20 $O/cfg5_$P.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/cfg5_$P.json').read().strip().splitlines()[-1]); print('lin', $P, d['value'], d['fill_ms'], d['traceback_ms'], d['chunks'], d['workspace_gb'], d['parity'])"
  timeout -k 10 400 python -u bench.py --workload cfg5 --gap-open -2 --pairs $P --steps 3 --warmup 1 --no-cpu > $O/cfg5a_$P.json 2> $O/cfg5a_$P.err || { tail -20 $O/cfg5a_$P.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/cfg5a_$P.json').read().strip().splitlines()[-1]); print('aff', $P, d['value'], d['fill_ms'], d['traceback_ms'], d['chunks'], d['workspace_gb'])"
done
echo s43 done
