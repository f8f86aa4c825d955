#!/usr/bin/env bash
# One GPU call, several steps, each under its own time limit; stops at the first failure.
#   scripts/gpu_step.sh "ubench" "pytest:<pytest -k expr>:<files>" "bench:<tag>:<bench args>" ...
# Logs and bench lines go to gpurun_out/ (merged back by gpurun).
set -u
mkdir -p gpurun_out/bench
for spec in "$@"; do
  kind="${spec%%:*}"
  case "$kind" in
    ubench)
      # built on the box from its source (the binary is git- and gpurun-ignored)
      /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 scripts/exp/ubench/valu_rates.hip -o scripts/exp/ubench/valu_rates \
        || { echo "ubench build failed"; exit 1; }
      timeout -k 10 180 ./scripts/exp/ubench/valu_rates > gpurun_out/valu_rates.txt 2>&1 || { echo "ubench failed"; exit 1; }
      echo "ubench ok" ;;
    pytest)
      rest="${spec#pytest:}"; expr="${rest%%:*}"; files="${rest#*:}"
      timeout -k 10 1100 python -u -m pytest $files -m gpu -x -v --timeout 400 --timeout-method thread -k "$expr" \
        > gpurun_out/pytest_$(date +%s).log 2>&1
      rc=$?; echo "pytest [$expr] rc=$rc"; tail -2 gpurun_out/pytest_*.log | tail -1
      [ $rc -eq 0 ] || exit 1 ;;
    bench)
      rest="${spec#bench:}"; tag="${rest%%:*}"; args="${rest#*:}"
      timeout -k 10 600 python -u bench.py $args > gpurun_out/bench/$tag.json 2> gpurun_out/bench/$tag.err
      rc=$?; echo "bench $tag rc=$rc"
      python3 -c "import json; d=json.loads(open('gpurun_out/bench/$tag.json').read().strip().splitlines()[-1]); print('  value', d.get('value'), 'fill', d.get('fill_ms'), 'tb', d.get('traceback_ms'), 'parity', (d.get('parity') or {}).get('bit_exact'))" 2>/dev/null
      [ $rc -le 1 ] || exit 1 ;;
  esac
done
