# config 2 pipelined bench with the default library and experiment variants (build/exp/<name>.so)
set -o pipefail
mkdir -p gpurun_out
for v in default "$@" default "$@"; do
  lib=bioinfo1_amd/libteam_alignment.so; [ "$v" = default ] || lib=build/exp/$v.so
  timeout -k 10 200 python -u -c "
import sys, runpy
import bioinfo1_amd.align as A
A.LIB_PATH = '$lib'
sys.argv = ['bench.py', '--steps', '30', '--warmup', '3', '--no-cpu', '--no-host', '--no-score-only']
runpy.run_path('bench.py', run_name='__main__')
" > gpurun_out/prio.json 2> gpurun_out/prio.err
  rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/prio.err; exit $rc; }
  grep '^{' gpurun_out/prio.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['pipeline']; print('$v', d['ms_per_step'], 'serial', p['serial_ms_per_step'], 'fill', d['fill_ms'], 'tb', d['traceback_ms'], p['slots_bit_identical'], d['parity']['bit_exact'])"
done
