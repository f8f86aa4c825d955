set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cp bioinfo1_amd/libteam_alignment.so /tmp/base.so
for r in 1 2; do
  for v in base w6; do
    if [ $v = base ]; then cp /tmp/base.so bioinfo1_amd/libteam_alignment.so; else cp build/exp/w6.so bioinfo1_amd/libteam_alignment.so; fi
    timeout -k 10 300 python -u bench.py --no-cpu --no-host --no-score-only > gpurun_out/ab_${v}_$r.json 2> gpurun_out/ab_${v}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_${v}_$r.json').read().strip().splitlines()[-1]); p=d['pipeline']; print('$v $r', d['value'], d['ms_per_step'], 'fill', d['fill_ms'], 'tb', d['traceback_ms'], 'serial', p['serial_value'], 'parity', d['parity']['bit_exact'], p['slots_bit_exact'])"
  done
done
