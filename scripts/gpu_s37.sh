#!/usr/bin/env bash
# s37: traceback time vs pair count (tail effect of 8 waves/SIMD x 1024 SIMDs = 8192 resident walks)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/s37; mkdir -p $O
for P in 2048 4096 8192 10000 12288 16384 20480; do
  timeout -k 10 200 python -u bench.py --pairs $P --no-cpu --no-parity --steps 5 > $O/p$P.json 2> $O/p$P.err || { tail -20 $O/p$P.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/p$P.json').read().strip().splitlines()[-1]); print($P, d['value'], d['fill_ms'], d['traceback_ms'])"
done
echo s37 done
