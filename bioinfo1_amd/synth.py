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


def _mix(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def stream(state0, k0: int, count: int) -> np.ndarray:
    """Outputs ``k0 .. k0+count-1`` of the splitmix64 stream that starts from
    ``state0`` (closed form: output k = mix(state0 + (k+1) * golden)).
    ``state0`` may be an array (one stream per row)."""
    st = np.asarray(state0, dtype=np.uint64)[..., None]
    k = np.arange(k0 + 1, k0 + 1 + count, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return _mix(st + k * _GOLDEN)


def draws(seed: int, n_pairs: int, count: int, first_pair: int = 0) -> np.ndarray:
    """``count`` splitmix64 outputs per pair -> uint64 array [n_pairs, count]
    (pair p's stream starts from state ``seed ^ p``)."""
    st = np.uint64(seed) ^ np.arange(first_pair, first_pair + n_pairs, dtype=np.uint64)
    return stream(st, 0, count).reshape(n_pairs, count)


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
    (event, base), then tlen padding bases.  (related_batch_torch makes the
    same bytes on the GPU, for config 5's 100k pairs.)"""
    block = max(1, (64 << 20) // (8 * (3 * qlen + tlen) + 1))  # bound the draw matrix to ~64 MB
    if n_pairs > block:
        parts = [related_batch(min(block, n_pairs - k), qlen, tlen, seed, rate, first_pair + k)
                 for k in range(0, n_pairs, block)]
        return _concat(parts)
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


def _concat(parts) -> PairBatch:
    qb = np.concatenate([b.qbytes for b in parts])
    tb = np.concatenate([b.tbytes for b in parts])
    ql = np.concatenate([b.qlen for b in parts])
    tl = np.concatenate([b.tlen for b in parts])
    qoff = np.zeros(ql.shape[0], np.uint64)
    toff = np.zeros(tl.shape[0], np.uint64)
    if ql.shape[0]:
        qoff[1:] = np.cumsum(ql[:-1], dtype=np.uint64)
        toff[1:] = np.cumsum(tl[:-1], dtype=np.uint64)
    return PairBatch(qb, qoff, ql, tb, toff, tl)


# --- the same generators on the GPU (torch int64, two's-complement wrap) ----

def _i64(x: int) -> int:
    return x - (1 << 64) if x >= 1 << 63 else x


def _torch_mix(z):
    """splitmix64's output mix on an int64 tensor (logical shifts by masking)."""
    import torch

    def shr(v, k):
        return (v >> k) & ((1 << (64 - k)) - 1)

    z = (z ^ shr(z, 30)) * _i64(int(_M1))
    z = (z ^ shr(z, 27)) * _i64(int(_M2))
    return z ^ shr(z, 31)


def draws_torch(seed: int, n_pairs: int, count: int, first_pair: int, device):
    """``draws`` on ``device`` as int64 (bit patterns of the uint64 outputs)."""
    import torch

    st = torch.arange(first_pair, first_pair + n_pairs, dtype=torch.int64, device=device) ^ _i64(seed)
    k = torch.arange(1, count + 1, dtype=torch.int64, device=device) * _i64(int(_GOLDEN))
    return _torch_mix(st[:, None] + k[None, :])


def related_batch_torch(n_pairs: int, qlen: int, tlen: int, seed: int = 0x5EED, rate: float = 0.05,
                        first_pair: int = 0, device="cuda", block: int = 256):
    """related_batch generated on the GPU: returns (query bytes, target bytes)
    as uint8 device tensors [n_pairs * qlen], [n_pairs * tlen] -- the pairs
    of a fixed-shape batch back to back (offsets p*qlen, p*tlen), the same
    bytes as related_batch (tests/test_synth.py)."""
    import torch

    acgt = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=device)
    Q = torch.empty(n_pairs * qlen, dtype=torch.uint8, device=device)
    T = torch.empty(n_pairs * tlen, dtype=torch.uint8, device=device)
    W = max(2 * qlen, tlen)
    for k0 in range(0, n_pairs, block):
        B = min(block, n_pairs - k0)
        d = draws_torch(seed, B, 3 * qlen + tlen, first_pair + k0, device)
        top = ((d >> 62) & 3).long()
        q = acgt[top[:, :qlen]]
        ev = ((d[:, qlen:3 * qlen:2] >> 11) & ((1 << 53) - 1)).double() * (1.0 / 2**53)
        eb = acgt[top[:, qlen + 1:3 * qlen:2]]
        pad = acgt[top[:, 3 * qlen:]]
        del d, top
        sub = ev < rate
        ins = (ev >= rate) & (ev < 2 * rate)
        dele = (ev >= 2 * rate) & (ev < 3 * rate)
        base = torch.where(sub, eb, q)
        emit_base = ~dele
        cnt = ins.long() + emit_base.long()
        pos = torch.cumsum(cnt, 1) - cnt
        L = cnt.sum(1)
        seq = torch.zeros((B, W), dtype=torch.uint8, device=device)
        rows = torch.arange(B, device=device)[:, None].expand(B, qlen)
        seq[rows[ins], pos[ins]] = eb[ins]
        pb = pos + ins.long()
        seq[rows[emit_base], pb[emit_base]] = base[emit_base]
        col = torch.arange(tlen, device=device)[None, :]
        padded = torch.gather(pad, 1, (col - L[:, None]).clamp(min=0))
        t = torch.where(col < L[:, None], seq[:, :tlen], padded)
        Q[k0 * qlen:(k0 + B) * qlen] = q.reshape(-1)
        T[k0 * tlen:(k0 + B) * tlen] = t.reshape(-1)
    return Q, T


def related_pairs_at(indices, qlen: int, tlen: int, seed: int = 0x5EED, rate: float = 0.05) -> PairBatch:
    """The pairs at stream positions ``indices`` of related_batch's stream (pair p
    depends only on ``seed ^ p``): the stratified samples of config 5's 100k-pair
    stream that the golden digests pin (tests/golden/make_golden.py)."""
    return _concat([related_batch(1, qlen, tlen, seed, rate, first_pair=int(p)) for p in indices])


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


# --- config 3 / 4 stand-in: a genome and ONT-like reads -----

COMPLEMENT = np.arange(256, dtype=np.uint8)
for _a, _b in (b"AT", b"TA", b"CG", b"GC"):
    COMPLEMENT[_a] = _b


def reverse_complement(seq: np.ndarray) -> np.ndarray:
    """A<->T, C<->G, reversed; other bytes pass through (team_mapper.cpp:47-63)."""
    return COMPLEMENT[seq[::-1]]


def genome(length: int, seed: int = 0xEC011) -> np.ndarray:
    """i.i.d. uniform ACGT genome (the E. coli K-12 stand-in is 4,641,652 bp)."""
    out = np.empty(length, dtype=np.uint8)
    step = 1 << 22
    for k0 in range(0, length, step):
        c = min(step, length - k0)
        out[k0 : k0 + c] = ACGT[(stream(seed, k0, c) >> np.uint64(62)).astype(np.intp)]
    return out


@dataclass
class ReadSet:
    """Reads sampled from a genome: concatenated bytes + offsets/lengths, and
    where each came from (forward-strand start, segment length, strand)."""

    bytes: np.ndarray  # uint8
    off: np.ndarray  # uint64 [R]
    len: np.ndarray  # uint32 [R]
    start: np.ndarray  # uint64 [R], forward coordinates
    seg_len: np.ndarray  # uint32 [R]
    rev: np.ndarray  # bool [R]

    @property
    def n_reads(self) -> int:
        return int(self.len.shape[0])

    def read(self, r: int) -> bytes:
        o = int(self.off[r])
        return self.bytes[o : o + int(self.len[r])].tobytes()


def _mutate(seg: np.ndarray, d: np.ndarray, rate: float) -> np.ndarray:
    ev = (d[0::2] >> np.uint64(11)).astype(np.float64) * (1.0 / 2**53)
    eb = ACGT[(d[1::2] >> np.uint64(62)).astype(np.intp)]
    r3 = rate / 3.0
    sub = ev < r3
    ins = (ev >= r3) & (ev < 2 * r3)
    emit_base = ~((ev >= 2 * r3) & (ev < rate))
    base = np.where(sub, eb, seg)
    cnt = ins.astype(np.intp) + emit_base.astype(np.intp)
    out = np.empty(int(cnt.sum()), dtype=np.uint8)
    pos = np.cumsum(cnt) - cnt
    out[pos[ins]] = eb[ins]
    out[(pos + ins)[emit_base]] = base[emit_base]
    return out


def ont_reads(n_reads: int, ref: np.ndarray, seed: int = 0x0E7, median: float = 9000.0, sigma: float = 0.5,
              min_len: int = 1000, max_len: int = 20000, error: float = 0.10, first_read: int = 0,
              indices=None) -> ReadSet:
    """ONT-like reads: log-normal segment lengths (median ``median``, clamped to
    [min_len, max_len]), uniform start, 50 % reverse-complement strand, then
    ``error`` total substitution/insertion/deletion rate (a third each).
    Read r's stream starts from state ``seed ^ r``: 4 header draws (two for the
    length, start, strand), then 2 draws per segment base.  ``indices``: the
    reads at these stream positions instead of ``first_read ..`` (each read is
    independent of the others, so read r is the same bytes in any set)."""
    G = int(ref.shape[0])
    max_len = min(max_len, G)
    chunks, lens, starts, segs, revs = [], [], [], [], []
    idx = range(first_read, first_read + n_reads) if indices is None else [int(r) for r in indices]
    n_reads = len(idx)
    for r in idx:
        st = np.uint64(seed) ^ np.uint64(r)
        h = stream(st, 0, 4)
        u1 = (float(h[0] >> np.uint64(11)) + 1.0) * (1.0 / 2**53)
        u2 = float(h[1] >> np.uint64(11)) * (1.0 / 2**53)
        z = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)
        L = int(min(max(round(median * np.exp(sigma * z)), min_len), max_len))
        s = int(h[2] % np.uint64(G - L + 1))
        rev = bool(h[3] >> np.uint64(63))
        seg = ref[s : s + L]
        if rev:
            seg = reverse_complement(seg)
        rd = _mutate(seg, stream(st, 4, 2 * L), error)
        chunks.append(rd)
        lens.append(rd.shape[0])
        starts.append(s)
        segs.append(L)
        revs.append(rev)
    ln = np.array(lens, dtype=np.uint32)
    off = np.zeros(n_reads, dtype=np.uint64)
    if n_reads:
        off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    b = np.concatenate(chunks) if chunks else np.zeros(0, np.uint8)
    return ReadSet(b, off, ln, np.array(starts, dtype=np.uint64), np.array(segs, dtype=np.uint32),
                   np.array(revs, dtype=bool))


def origin_batch(reads: ReadSet, ref: np.ndarray) -> PairBatch:
    """Config-3 stand-in pairs: each read against its true origin window, in
    the read's orientation (a window of the reverse-complement reference for
    reverse reads, as team_mapper.cpp:674-678 aligns them)."""
    tgt = []
    for r in range(reads.n_reads):
        s, L = int(reads.start[r]), int(reads.seg_len[r])
        seg = ref[s : s + L]
        tgt.append(reverse_complement(seg) if reads.rev[r] else seg)
    tl = reads.seg_len.copy()
    toff = np.zeros(reads.n_reads, dtype=np.uint64)
    if reads.n_reads:
        toff[1:] = np.cumsum(tl[:-1], dtype=np.uint64)
    tb = np.concatenate(tgt) if tgt else np.zeros(0, np.uint8)
    return PairBatch(reads.bytes, reads.off.copy(), reads.len.copy(), tb, toff, tl)


ECOLI_LEN = 4_641_652  # NC_000913.3


def cfg3_batch(n_reads: int = 10000, first_read: int = 0, genome_seed: int = 0xEC011, read_seed: int = 0x0E7,
               indices=None):
    """Config 3 stand-in: reads of a 4.64 Mb i.i.d. genome against
    their true-origin windows.  Returns (PairBatch, ReadSet, genome).
    ``indices``: only the reads at these positions of the read stream."""
    g = genome(ECOLI_LEN, genome_seed)
    rs = ont_reads(n_reads, g, read_seed, first_read=first_read, indices=indices)
    return origin_batch(rs, g), rs, g


# stratified digest positions (tests/golden/make_golden.py): pairs from every chunk of the
# stated-size runs, not only the first ones
CFG5_STRIDED = np.arange(128, dtype=np.int64) * 781   # 0 .. 99,187 of config 5's 100,000 pairs
CFG3_STRIDED = np.arange(256, dtype=np.int64) * 39    # 0 .. 9,945 of config 3's 10,000 reads
