"""CPU restatement of the mapper stages around team::Align (TEST
INFRASTRUCTURE ONLY -- only tests/ and the golden-vector scripts use it).

* ``minimize``        -- team::KMER::Minimize (team_minimizers/
                         team_minimizers.cpp:122-225), entry for entry
* ``first_occurrences`` -- remove_duplicates (team_mapper.cpp:26-42)
* ``find_lis``        -- FindLIS (team_mapper.cpp:283-316)
* ``RefMapper``       -- ctypes over oracle/_ref/libref_mapper.so (the
                         reference's own Minimize compiled from source, and the
                         restated FindLIS), present only where it was built
* ``ref_mapper_binary`` -- oracle/_ref/ref_mapper: the reference Minimize +
                         Align with the restated team_mapper.cpp glue (PAF)

Parity: ``minimize`` is pinned to the reference Minimize through
tests/golden/mapper/minimizers.json (made by oracle/_ref) and, where _ref is
built, fresh random sequences (tests/test_mapper_oracle.py).  The mapper glue
(index ban order, matching, chaining, PAF) has no reference build here
(team_mapper.cpp needs the absent bioparser): its pin is the restatement in
oracle/ref_mapper.cpp, so end-to-end mapper parity is "glue restated".
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_MAPPER_SO = os.path.join(HERE, "_ref", "libref_mapper.so")
REF_MAPPER_BIN = os.path.join(HERE, "_ref", "ref_mapper")

_CODE = np.zeros(256, dtype=np.uint32)
_CODE[ord("C")] = 0
_CODE[ord("A")] = 1
_CODE[ord("T")] = 2
_CODE[ord("G")] = 3
UINT_MAX = 0xFFFFFFFF


def kmer_code(seq: bytes, i: int, k: int) -> int:
    """MappSeqCharPointerToBit (:66-86): 2-bit fold in uint32; bytes past the
    end read as NUL (the reference reads past the end of the string there)."""
    c = 0
    for t in range(k):
        b = seq[i + t] if i + t < len(seq) else 0
        c = ((c << 2) | int(_CODE[b])) & UINT_MAX
    return c


def _window_min(codes, lo, hi, is_fwd):
    """GetTupleWithMinFirst (:103-118) over k-mers lo..hi inclusive."""
    best, tup = UINT_MAX, (0, 0, False)  # default-constructed tuple if nothing is < UINT_MAX
    for i in range(lo, hi + 1):
        if codes(i) < best:
            best = codes(i)
            tup = (best, i + 1, is_fwd)
    return tup


def minimize(seq: bytes, k: int, w: int, is_fwd: bool = True):
    """team::KMER::Minimize -> list of (hash, 1-based pos, strand)."""
    L = len(seq)
    out = []
    if L < k or w == 0:
        return out
    cache = {}

    def codes(i):
        if i not in cache:
            cache[i] = kmer_code(seq, i, k)
        return cache[i]

    for u in range(k, w + k - 1):  # leading end-minimizers (:141-169)
        out.append(_window_min(codes, 0, u - k, is_fwd))
    for i in range(0, L - k + 1):  # full windows (:172-198)
        if i >= w - 1:
            out.append(_window_min(codes, i - w + 1, i, is_fwd))
    for u in range(k, w + k - 1):  # trailing end-minimizers (:201-222)
        if L < u:
            break
        out.append(_window_min(codes, L - u, L - k, is_fwd))
    return out


def first_occurrences(mins):
    seen, out = set(), []
    for m in mins:
        if m not in seen:
            seen.add(m)
            out.append(m)
    return out


def find_lis(hits):
    """FindLIS over [(fragment pos, reference pos)] -> chain list."""
    n = len(hits)
    if n == 0:
        return []
    lis = [1] * n
    prev = [-1] * n
    for i in range(1, n):
        fi, ri = hits[i]
        for j in range(i):
            fj, rj = hits[j]
            if ri > rj and lis[i] < lis[j] + 1 and fi != fj and ((fi - fj) & UINT_MAX) < 5000 and (
                    (ri - rj) & UINT_MAX) < 5000:
                lis[i] = lis[j] + 1
                prev[i] = j
    best = max(range(n), key=lambda i: (lis[i], -i))
    chain = []
    i = best
    while i >= 0:
        chain.append(hits[i])
        i = prev[i]
    return chain[::-1]


class RefMapper:
    """The reference's own Minimize (compiled from /root/reference by
    oracle/Makefile) and the restated FindLIS, through ctypes."""

    @staticmethod
    def available() -> bool:
        return os.path.exists(REF_MAPPER_SO)

    def __init__(self):
        L = C.CDLL(REF_MAPPER_SO)
        L.ref_minimize.restype = C.c_int
        L.ref_minimize.argtypes = [C.c_char_p, C.c_uint, C.c_uint, C.c_uint, C.c_int, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
        L.ref_find_lis.restype = C.c_int
        L.ref_find_lis.argtypes = [C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_size_t)]
        self.lib = L

    def minimize(self, seq: bytes, k: int, w: int, is_fwd: bool = True):
        cap = len(seq) + 2 * w + 4
        h = np.zeros(cap, np.uint32)
        p = np.zeros(cap, np.uint32)
        s = np.zeros(cap, np.uint8)
        n, u = C.c_size_t(0), C.c_size_t(0)
        r = self.lib.ref_minimize(seq, len(seq), k, w, int(is_fwd), h.ctypes.data, p.ctypes.data, s.ctypes.data,
                                  cap, C.byref(n), C.byref(u))
        assert r == 0
        return [(int(h[i]), int(p[i]), bool(s[i])) for i in range(n.value)], u.value

    def find_lis(self, hits):
        n = len(hits)
        f = np.array([h[0] for h in hits], np.uint32) if n else np.zeros(1, np.uint32)
        r = np.array([h[1] for h in hits], np.uint32) if n else np.zeros(1, np.uint32)
        of = np.zeros(max(n, 1), np.uint32)
        orr = np.zeros(max(n, 1), np.uint32)
        m = C.c_size_t(0)
        self.lib.ref_find_lis(n, f.ctypes.data, r.ctypes.data, of.ctypes.data, orr.ctypes.data, C.byref(m))
        return [(int(of[i]), int(orr[i])) for i in range(m.value)]
