"""Synthetic read-vs-window batches for tests and bench.

The generator is splitmix64, seeded per pair with ``seed ^ p`` so the same
batch is reproduced bit-for-bit here, on the GPU box and by the golden-vector
script (tests/golden/make_golden.py).  Bases are ``"ACGT"[x >> 62]``.

A batch is a :class:`PairBatch`: concatenated query / target bytes plus
uint64 offsets and uint32 lengths (the SoA layout the C-ABI takes,
include/team_align_c.h).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def splitmix64_next(state: np.ndarray) -> np.ndarray:
    """Advance ``state`` (uint64 array, in place) and return the outputs."""
    with np.errstate(over="ignore"):
        state += _GOLDEN
        z = state.copy()
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def draws(seed: int, n_pairs: int, count: int, first_pair: int = 0) -> np.ndarray:
    """``count`` splitmix64 outputs per pair -> uint64 array [n_pairs, count]."""
    st = np.uint64(seed) ^ np.arange(first_pair, first_pair + n_pairs, dtype=np.uint64)
    out = np.empty((n_pairs, count), dtype=np.uint64)
    for k in range(count):
        out[:, k] = splitmix64_next(st)
    return out


@dataclass
class PairBatch:
    qbytes: np.ndarray  # uint8, concatenated queries
    qoff: np.ndarray  # uint64 [P]
    qlen: np.ndarray  # uint32 [P]
    tbytes: np.ndarray  # uint8, concatenated targets
    toff: np.ndarray  # uint64 [P]
    tlen: np.ndarray  # uint32 [P]

    @property
    def n_pairs(self) -> int:
        return int(self.qlen.shape[0])

    @property
    def cells(self) -> int:
        return int(np.dot(self.qlen.astype(np.uint64), self.tlen.astype(np.uint64)))

    def query(self, p: int) -> bytes:
        o = int(self.qoff[p])
        return self.qbytes[o : o + int(self.qlen[p])].tobytes()

    def target(self, p: int) -> bytes:
        o = int(self.toff[p])
        return self.tbytes[o : o + int(self.tlen[p])].tobytes()

    def slice(self, lo: int, hi: int) -> "PairBatch":
        """Pairs [lo, hi) as a self-contained batch (used by the range split)."""
        return from_pairs([(self.query(p), self.target(p)) for p in range(lo, hi)])


def from_pairs(pairs) -> PairBatch:
    """Build a batch from an iterable of (query: bytes, target: bytes)."""
    pairs = list(pairs)
    ql = np.array([len(q) for q, _ in pairs], dtype=np.uint32)
    tl = np.array([len(t) for _, t in pairs], dtype=np.uint32)
    qoff = np.zeros(len(pairs), dtype=np.uint64)
    toff = np.zeros(len(pairs), dtype=np.uint64)
    if len(pairs):
        qoff[1:] = np.cumsum(ql[:-1], dtype=np.uint64)
        toff[1:] = np.cumsum(tl[:-1], dtype=np.uint64)
    qb = np.frombuffer(b"".join(q for q, _ in pairs), dtype=np.uint8).copy()
    tb = np.frombuffer(b"".join(t for _, t in pairs), dtype=np.uint8).copy()
    return PairBatch(qb, qoff, ql, tb, toff, tl)


def uniform_batch(n_pairs: int, qlen: int, tlen: int, seed: int = 0x5EED, first_pair: int = 0) -> PairBatch:
    """Config-2 shape: i.i.d. uniform ACGT, query then target from one stream."""
    d = draws(seed, n_pairs, qlen + tlen, first_pair)
    bases = ACGT[(d >> np.uint64(62)).astype(np.intp)]
    q = np.ascontiguousarray(bases[:, :qlen]).reshape(-1)
    t = np.ascontiguousarray(bases[:, qlen:]).reshape(-1)
    qoff = np.arange(n_pairs, dtype=np.uint64) * np.uint64(qlen)
    toff = np.arange(n_pairs, dtype=np.uint64) * np.uint64(tlen)
    return PairBatch(q, qoff, np.full(n_pairs, qlen, np.uint32), t, toff, np.full(n_pairs, tlen, np.uint32))


def related_batch(n_pairs: int, qlen: int, tlen: int, seed: int = 0x5EED, rate: float = 0.05,
                  first_pair: int = 0) -> PairBatch:
    """Config-2 "related" variant: target = query with ``rate`` substitutions,
    insertions and deletions each, trimmed / padded (random bases) to tlen.
    Per pair the stream yields qlen query bases, then 2 draws per query base
    (event, base), then tlen padding bases."""
    d = draws(seed, n_pairs, qlen + 2 * qlen + tlen, first_pair)
    top = (d >> np.uint64(62)).astype(np.intp)
    q = ACGT[top[:, :qlen]]
    ev = (d[:, qlen : 3 * qlen : 2] >> np.uint64(11)).astype(np.float64) * (1.0 / 2**53)
    eb = ACGT[top[:, qlen + 1 : 3 * qlen : 2]]
    pad = ACGT[top[:, 3 * qlen :]]
    out = []
    for p in range(n_pairs):
        e = ev[p]
        sub = e < rate
        ins = (e >= rate) & (e < 2 * rate)
        dele = (e >= 2 * rate) & (e < 3 * rate)
        base = np.where(sub, eb[p], q[p])
        # each query position emits: [inserted base] + [base unless deleted]
        emit_ins = ins
        emit_base = ~dele
        cnt = emit_ins.astype(np.intp) + emit_base.astype(np.intp)
        seq = np.empty(int(cnt.sum()), dtype=np.uint8)
        pos = np.cumsum(cnt) - cnt
        seq[pos[emit_ins]] = eb[p][emit_ins]
        seq[(pos + emit_ins)[emit_base]] = base[emit_base]
        if seq.shape[0] >= tlen:
            seq = seq[:tlen]
        else:
            seq = np.concatenate([seq, pad[p][: tlen - seq.shape[0]]])
        out.append(seq)
    t = np.concatenate(out) if out else np.zeros(0, np.uint8)
    qf = np.ascontiguousarray(q).reshape(-1)
    qoff = np.arange(n_pairs, dtype=np.uint64) * np.uint64(qlen)
    toff = np.arange(n_pairs, dtype=np.uint64) * np.uint64(tlen)
    return PairBatch(qf, qoff, np.full(n_pairs, qlen, np.uint32), t, toff, np.full(n_pairs, tlen, np.uint32))


def ragged_batch(n_pairs: int, min_len: int, max_len: int, seed: int = 0x5EED, alphabet: bytes = b"ACGT",
                 first_pair: int = 0) -> PairBatch:
    """Independent random lengths in [min_len, max_len] for query and target,
    bases drawn uniformly from ``alphabet`` (used for edge-case parity)."""
    alpha = np.frombuffer(alphabet, dtype=np.uint8)
    d = draws(seed, n_pairs, 2 + 2 * max_len, first_pair)
    span = np.uint64(max_len - min_len + 1)
    ql = (d[:, 0] % span).astype(np.int64) + min_len
    tl = (d[:, 1] % span).astype(np.int64) + min_len
    sym = alpha[((d[:, 2:] >> np.uint64(32)) % np.uint64(len(alpha))).astype(np.intp)]
    pairs = []
    for p in range(n_pairs):
        pairs.append((sym[p, : ql[p]].tobytes(), sym[p, max_len : max_len + tl[p]].tobytes()))
    return from_pairs(pairs)
