#!/usr/bin/env bash
# s29: pipelined batches (traceback of batch k beside fill of batch k+1): parity, then bench variants
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s29; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "pipelined or staged or device_plan" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="python -u bench.py --no-cpu"
timeout -k 10 300 $B > $O/cfg2_pipe.json 2> $O/cfg2_pipe.err || { tail -30 $O/cfg2_pipe.err; exit 1; }
tail -1 $O/cfg2_pipe.json
timeout -k 10 300 $B --no-pipeline > $O/cfg2_seq.json 2> $O/cfg2_seq.err || { tail -30 $O/cfg2_seq.err; exit 1; }
tail -1 $O/cfg2_seq.json
for w in 1 3 0; do
  TA_TB_WAVES_PER_SIMD=$w timeout -k 10 300 $B --no-parity > $O/cfg2_pipe_w$w.json 2> $O/cfg2_pipe_w$w.err || { tail -30 $O/cfg2_pipe_w$w.err; exit 1; }
  echo "w=$w"; tail -1 $O/cfg2_pipe_w$w.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
timeout -k 10 300 $B --steps 20 > $O/cfg2_pipe_k20.json 2> $O/cfg2_pipe_k20.err || { tail -30 $O/cfg2_pipe_k20.err; exit 1; }
echo k20; tail -1 $O/cfg2_pipe_k20.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
timeout -k 10 400 $B --workload cfg5 --steps 3 --warmup 2 > $O/cfg5_pipe.json 2> $O/cfg5_pipe.err || { tail -30 $O/cfg5_pipe.err; exit 1; }
tail -1 $O/cfg5_pipe.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-parity > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }

# re-run of the digest sequence that failed once in the first s29 call (ragged_global scores, 2/2000 pairs)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "digest" --timeout 200 --timeout-method thread > $GRAFT_REPO_ROOT/$O/pytest_digest_rerun.log 2>&1
tail -1 $GRAFT_REPO_ROOT/$O/pytest_digest_rerun.log
echo s29 done
