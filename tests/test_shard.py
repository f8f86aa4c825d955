"""Multi-rank path on CPU: world_size-2 (and 3) gloo process groups.  Each
rank aligns its cell-balanced range with the CPU checker standing in for its
GPU, the results are gathered with bioinfo1_amd.shard.gather_results, and
the gathered batch must equal the single-process result byte for byte."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from bioinfo1_amd import shard, synth


def test_range_split_balanced_and_contiguous():
    b = synth.ragged_batch(200, 0, 500, seed=5)
    cells = b.qlen.astype(np.int64) * b.tlen.astype(np.int64)
    for world in (1, 2, 3, 8):
        rs = shard.range_split(cells, world)
        assert rs[0][0] == 0 and rs[-1][1] == 200
        assert all(rs[k][1] == rs[k + 1][0] for k in range(world - 1))
        per = [cells[lo:hi].sum() for lo, hi in rs]
        assert max(per) - min(per) <= cells.max() + 1


def test_range_split_edge_cases():
    assert shard.range_split(np.zeros(0, np.int64), 4) == [(0, 0)] * 4
    assert shard.range_split(np.zeros(5, np.int64), 2) == [(0, 2), (2, 5)]
    rs = shard.range_split(np.array([10, 0, 0, 0], np.int64), 2)
    assert rs[0][0] == 0 and rs[-1][1] == 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from oracle.pyoracle import Oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = synth.ragged_batch(60, 0, 200, seed=9, alphabet=b"ACGT-")
    cells = b.qlen.astype(np.int64) * b.tlen.astype(np.int64)
    lo, hi = shard.range_split(cells, world)[rank]
    part = b.slice(lo, hi)
    r = Oracle().align_batch(part, 2, 2, -1, -1, True, n_threads=1)
    cig = b"".join(r.cigar(p) for p in range(part.n_pairs))
    out = shard.gather_results(dist, torch.from_numpy(r.scores), torch.from_numpy(r.target_begins.view(np.int32)),
                               torch.from_numpy(r.cigar_lens.view(np.int32)),
                               torch.from_numpy(np.frombuffer(cig, np.uint8).copy()))
    if rank == 0:
        q.put((out[0].tolist(), out[1].tolist(), out[2].tolist(), out[3].tobytes()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gloo_gather_matches_single_process(world):
    from oracle.pyoracle import Oracle

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    b = synth.ragged_batch(60, 0, 200, seed=9, alphabet=b"ACGT-")
    full = Oracle().align_batch(b, 2, 2, -1, -1, True)
    assert got[0] == full.scores.tolist()
    assert got[1] == full.target_begins.tolist()
    assert got[2] == full.cigar_lens.tolist()
    assert got[3] == b"".join(full.cigars())
