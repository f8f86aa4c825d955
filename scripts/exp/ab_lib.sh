#!/usr/bin/env bash
# A/B of an experiment build (build/exp/libteam_alignment.so) against the
# in-tree library on one bench command: scripts/exp/ab_lib.sh <bench args...>
set -u
cp bioinfo1_amd/libteam_alignment.so build/exp/base.so
for v in base exp base exp; do
  if [ $v = base ]; then cp build/exp/base.so bioinfo1_amd/libteam_alignment.so; else cp build/exp/libteam_alignment.so bioinfo1_amd/libteam_alignment.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-host --no-score-only "$@" > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "fail $v"; tail -3 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab_$v.json') if l.startswith('{')][-1]); print('$v', d['value'], 'fill', d['fill_ms'], 'tb', d['traceback_ms'], (d.get('parity') or {}).get('bit_exact'))"
done
cp build/exp/base.so bioinfo1_amd/libteam_alignment.so
