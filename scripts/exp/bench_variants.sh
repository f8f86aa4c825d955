#!/usr/bin/env bash
# Bench each build/exp/<name>.so in place of the in-tree library (GPU box):
#   scripts/exp/bench_variants.sh "<bench args>" name...
set -u
ARGS=$1; shift
LIB=bioinfo1_amd/libteam_alignment.so
cp $LIB build/exp/_orig.so
for v in "$@"; do
  cp build/exp/$v.so $LIB
  timeout -k 10 300 python -u bench.py --no-cpu --no-host --no-score-only $ARGS > gpurun_out/v_$v.json 2> gpurun_out/v_$v.err
  rc=$?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/v_$v.json') if l.startswith('{')][-1]); print('$v', d['value'], 'fill', d['fill_ms'], 'tb', d['traceback_ms'], (d.get('parity') or {}).get('bit_exact'))" || { echo "$v rc=$rc"; tail -3 gpurun_out/v_$v.err; }
  [ $rc -le 1 ] || break
done
cp build/exp/_orig.so $LIB
