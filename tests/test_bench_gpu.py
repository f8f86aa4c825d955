"""bench.py's multi-GPU code path on the one-GPU box: `--gpus 2` starts two
ranks itself (torch.distributed.run), both on device 0 (TA_BENCH_ONE_GPU=1,
gloo), and (config 4) range-splits ONE read set by cells, aligns the halves,
gathers records + CIGAR bytes every step and compares the gathered result
with the 1-GPU result of the whole set and the reference digest
(SURVEY.md §8e); (config 2) gathers every rank's 1 kb pairs and checks rank
0's slice.  The 8-GPU run is the driver's."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=300):
    env = dict(os.environ, TA_BENCH_ONE_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_cfg4_two_ranks_gathered_equals_one_gpu():
    out = _bench("--gpus", "2", "--workload", "cfg4", "--pairs", "300", "--dist-backend", "gloo", "--steps", "2",
                 "--warmup", "1", "--no-cpu", "--workspace-gb", "8")
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"
    g = out["gather"]
    assert g["bit_exact"] and g["pairs"] == 300 and g["digest"]["bit_exact"], g
    assert out["parity"]["bit_exact"]


def test_cfg2_two_ranks_gather():
    out = _bench("--gpus", "2", "--pairs", "600", "--dist-backend", "gloo", "--steps", "2", "--warmup", "1",
                 "--no-cpu")
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    assert out["gather"]["bit_exact"] and out["gather"]["pairs_gathered"] == 1200, out["gather"]


def test_rccl_gather_world_one():
    """The RCCL branch of ResultGather (gather on a side stream, then
    point-to-point CIGAR bytes) with a world of one under
    torch.distributed.run: the only RCCL run a one-GPU box allows."""
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, TA_BENCH_FORCE_DIST="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "1", "--dist-backend", "nccl", "--pairs", "600", "--steps", "2", "--warmup", "1",
                        "--no-cpu", "--no-host", "--no-score-only"], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    g = out["gather"]
    assert g["bit_exact"] and g["pairs_gathered"] == 600 and g["cigar_bytes"] > 0, g
