"""Multi-GPU sharding of a pair batch.

Pairs are independent, so the batch is range-split by pair index into
contiguous, cell-balanced ranges (prefix sum of n*m), one per rank; each
rank aligns its range on its own GPU and the results are gathered back in
pair order.  The gather is the only collective: fixed-size per-pair records
(score, target_begin, cigar_len) with one all_gather, then the CIGAR bytes
with a second, padded all_gather (RCCL has no gatherv).  Over xGMI these are
KB-MB transfers -- latency-bound, not bandwidth-bound.

Works with any torch.distributed backend: "nccl" (= RCCL on ROCm) with
device tensors on the GPU box, "gloo" with CPU tensors in the CPU tests.
"""
from __future__ import annotations

import numpy as np


def range_split(cells: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous [lo, hi) pair ranges with ~equal total cells per rank.

    Rank r takes the pairs whose cell prefix sum (exclusive) falls in
    [r*T/world, (r+1)*T/world).  Order is preserved, so gathering the ranks'
    results in rank order reproduces the batch order."""
    P = int(cells.shape[0])
    if world <= 1 or P == 0:
        return [(0, P)] + [(P, P)] * max(world - 1, 0)
    c = np.asarray(cells, dtype=np.float64)
    excl = np.concatenate([[0.0], np.cumsum(c)[:-1]])
    total = float(c.sum())
    if total == 0:
        bounds = [round(P * r / world) for r in range(world + 1)]
    else:
        bounds = [0] + [int(np.searchsorted(excl, total * r / world, side="left")) for r in range(1, world)] + [P]
    return [(bounds[r], max(bounds[r], bounds[r + 1])) for r in range(world)]


def gather_results(dist, scores, target_begins, cigar_lens, cigar_bytes, device=None):
    """All-gather one rank's results; returns the concatenation over ranks.

    scores/target_begins/cigar_lens: 1-D int tensors of this rank's pairs;
    cigar_bytes: 1-D uint8 tensor, this rank's CIGARs back to back (may be
    None for score-only).  Returns (scores, target_begins, cigar_lens,
    cigar_bytes) as numpy arrays in global pair order."""
    import torch

    world = dist.get_world_size()
    dev = scores.device if device is None else device
    P = torch.tensor([scores.numel(), 0 if cigar_bytes is None else cigar_bytes.numel()], dtype=torch.int64,
                     device=dev)
    sizes = [torch.zeros_like(P) for _ in range(world)]
    dist.all_gather(sizes, P)
    sizes = torch.stack(sizes).cpu().numpy()
    pmax, bmax = int(sizes[:, 0].max()), int(sizes[:, 1].max())
    rec = torch.zeros((3, max(pmax, 1)), dtype=torch.int32, device=dev)
    n = scores.numel()
    rec[0, :n] = scores.to(torch.int32)
    rec[1, :n] = target_begins.to(torch.int32)
    rec[2, :n] = cigar_lens.to(torch.int32)
    recs = [torch.zeros_like(rec) for _ in range(world)]
    dist.all_gather(recs, rec)
    out = [torch.cat([recs[r][k, : sizes[r, 0]] for r in range(world)]).cpu().numpy() for k in range(3)]
    cig = None
    if cigar_bytes is not None:
        # gloo has no uint8 all_gather on every build: move bytes as int32 words
        words = (bmax + 3) // 4
        buf = torch.zeros(max(words, 1) * 4, dtype=torch.uint8, device=dev)
        buf[: cigar_bytes.numel()] = cigar_bytes
        bufw = buf.view(torch.int32)
        bufs = [torch.zeros_like(bufw) for _ in range(world)]
        dist.all_gather(bufs, bufw)
        cig = np.concatenate([bufs[r].view(torch.uint8)[: sizes[r, 1]].cpu().numpy() for r in range(world)])
    return out[0], out[1].view(np.uint32), out[2].view(np.uint32), cig
