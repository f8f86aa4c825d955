#!/usr/bin/env bash
# s26: cfg2 repeatability + PMC (VALU instructions, HBM bytes) of the config-3 flexible fill
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s26; mkdir -p $O
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg2_$k.log 2>&1 || { tail -20 $O/bench_cfg2_$k.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_cfg2_$k.log').read().strip().splitlines()[-1]); print('cfg2', d['value'], d['ms_per_step'], d['fill_ms'], d['traceback_ms'])"
done
export TMPDIR=/tmp
BA="bench.py --workload cfg3 --steps 1 --warmup 0 --no-cpu --no-parity"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o run -- python3 $BA > $O/prof_trace.log 2>&1 || { tail -20 $O/prof_trace.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/prof_sq -o run -- python3 $BA > $O/prof_sq.log 2>&1 || { tail -20 $O/prof_sq.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- python3 $BA > $O/prof_fetch.log 2>&1 || { tail -20 $O/prof_fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- python3 $BA > $O/prof_write.log 2>&1 || { tail -20 $O/prof_write.log; exit 1; }
echo s26 done
