"""Python host-side mirror of the mapper stages around team::Align, over the
extern "C" ABI of libteam_mapper.so (include/team_mapper_c.h) -- the gfx950
kernels do the work; there is no CPU fallback (a missing library or GPU
raises).

Reference names are kept where the reference has them:
  ``KMER(is_fwd).Minimize(seq, k, w)``   team_minimizers.cpp:122-225
  ``remove_duplicates(mins)``             team_mapper.cpp:26-42 (device dedup)
  ``FindLIS(hits)``                       team_mapper.cpp:283-316
  ``map_files(ref, reads, ...)``          team_mapper.cpp main (PAF lines)
and batched forms (``minimize_batch``, ``chain_batch``, ``Index`` +
``map_batch``) are what the mapper driver itself uses.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

from . import align as _align

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libteam_mapper.so")
CLI_PATH = os.path.join(HERE, "team_mapper_amd")

TM_OK = 0

# Every symbol include/team_mapper_c.h declares (checked by tests/test_abi.py).
ABI_SYMBOLS = ["tm_status_string", "tm_last_error", "tm_context_create", "tm_context_destroy", "tm_minimizer_bound",
               "tm_minimize_batch", "tm_chain_batch", "tm_index_create", "tm_index_destroy", "tm_index_stats",
               "tm_map_batch", "tm_stage_times", "tm_align_plan_stats", "tm_map_files"]

_lib = None


class Options(C.Structure):
    """tm_options: team_mapper.cpp:321-387 defaults (global, 1/-1/-1, k 15, w 5, f 0.001)."""

    _fields_ = [("type", C.c_int), ("match", C.c_int), ("mismatch", C.c_int), ("gap", C.c_int), ("k", C.c_uint32),
                ("w", C.c_uint32), ("f", C.c_double), ("want_cigar", C.c_int), ("fastq_rules", C.c_int)]

    @classmethod
    def make(cls, type=0, match=1, mismatch=-1, gap=-1, k=15, w=5, f=0.001, want_cigar=False, fastq_rules=False):
        return cls(int(type), match, mismatch, gap, k, w, f, int(bool(want_cigar)), int(bool(fastq_rules)))


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    _align.lib()  # one HIP runtime (torch's) and libteam_alignment.so first
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    vp, u32p, u64p, i32p, u8p = C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), C.POINTER(C.c_int32), \
        C.POINTER(C.c_uint8)
    L.tm_status_string.restype = C.c_char_p
    L.tm_status_string.argtypes = [C.c_int]
    L.tm_last_error.restype = C.c_char_p
    L.tm_last_error.argtypes = [vp]
    L.tm_context_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.tm_context_destroy.argtypes = [vp]
    L.tm_context_destroy.restype = None
    L.tm_minimizer_bound.restype = C.c_uint64
    L.tm_minimizer_bound.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
    L.tm_minimize_batch.argtypes = [vp, C.c_uint32, vp, u64p, u32p, C.c_uint32, C.c_uint32, C.c_int, u64p, u32p,
                                    u32p, C.c_uint64]
    L.tm_chain_batch.argtypes = [vp, C.c_uint32, u64p, u32p, u32p, u32p, u32p, u32p, u32p, u32p]
    L.tm_index_create.argtypes = [vp, C.c_char_p, vp, C.c_uint64, C.c_uint32, C.c_uint32, C.c_double, C.POINTER(vp)]
    L.tm_index_destroy.argtypes = [vp]
    L.tm_index_destroy.restype = None
    L.tm_index_stats.argtypes = [vp, u64p, u64p, u64p, u64p, u32p, u32p]
    L.tm_map_batch.argtypes = [vp, vp, C.c_uint32, vp, u64p, u32p, C.POINTER(Options), u8p, u8p, u32p, u32p, u32p,
                               u32p, i32p, vp, C.c_uint64, u64p, u32p]
    L.tm_stage_times.argtypes = [vp, C.POINTER(C.c_double), C.c_uint32, u64p]
    L.tm_align_plan_stats.argtypes = [vp, u64p]
    L.tm_map_files.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(Options), C.c_char_p, C.c_int]
    _lib = L
    return L


def _p(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))


def _check(r, ctx=None):
    if r != TM_OK:
        L = lib()
        msg = L.tm_status_string(r).decode()
        detail = L.tm_last_error(ctx).decode() if ctx else ""
        raise RuntimeError(f"{msg}: {detail}" if detail else msg)


def _soa(seqs):
    """(bytes uint8[], off uint64[], len uint32[]) -- also accepts that tuple as is."""
    if isinstance(seqs, tuple) and len(seqs) == 3 and isinstance(seqs[0], np.ndarray):
        return seqs
    seqs = [bytes(s) for s in seqs]
    ln = np.array([len(s) for s in seqs], dtype=np.uint32)
    off = np.zeros(len(seqs), dtype=np.uint64)
    if len(seqs):
        off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    b = np.frombuffer(b"".join(seqs) or b"\0", dtype=np.uint8).copy()
    return b, off, ln


def soa(seqs):
    """Pack sequences once into the SoA layout map_batch takes."""
    return _soa(seqs)


class Mapper:
    """A device context for the mapper stages (one gfx950 GPU)."""

    def __init__(self, device: int = 0):
        L = lib()
        h = C.c_void_p()
        _check(L.tm_context_create(device, C.byref(h)))
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            lib().tm_context_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- minimizers ---------------------------------------------------------
    def minimize_batch(self, seqs, k: int, w: int, dedup: bool = False):
        """Per sequence: (hash uint32[], 1-based pos uint32[]) in Minimize order."""
        L = lib()
        b, off, ln = _soa(seqs)
        cap = int(sum(L.tm_minimizer_bound(int(x), k, w) for x in ln))
        oo = np.zeros(len(ln) + 1, np.uint64)
        h = np.zeros(max(cap, 1), np.uint32)
        p = np.zeros(max(cap, 1), np.uint32)
        _check(L.tm_minimize_batch(self._h, len(ln), b.ctypes.data, _p(off, C.c_uint64), _p(ln, C.c_uint32), k, w,
                                   int(dedup), _p(oo, C.c_uint64), _p(h, C.c_uint32), _p(p, C.c_uint32), cap),
               self._h)
        return [(h[int(oo[s]):int(oo[s + 1])].copy(), p[int(oo[s]):int(oo[s + 1])].copy()) for s in range(len(ln))]

    STAGES = ["upload", "minimizers", "matching", "chaining", "windows_plan", "align", "results", "total"]

    def stage_times(self):
        """Per-stage wall ms of the last map_batch on this context, and its aligned cells."""
        ms = (C.c_double * 8)()
        cells = C.c_uint64()
        _check(lib().tm_stage_times(self._h, ms, 8, C.byref(cells)))
        return dict(zip(self.STAGES, list(ms))), cells.value

    def align_plan_stats(self):
        """The alignment plan of the last map_batch (ta_plan_* counts)."""
        out = (C.c_uint64 * 5)()
        _check(lib().tm_align_plan_stats(self._h, out))
        return dict(zip(["pairs", "chunks", "dual_pairs", "flex_pairs", "workspace_bytes"], list(out)))

    # -- chaining -----------------------------------------------------------
    def chain_batch(self, lists):
        """FindLIS over each [(fpos, rpos)] list -> (len, first (f, r), last (f, r)) per list."""
        L = lib()
        n = len(lists)
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum([len(x) for x in lists], dtype=np.uint64)
        tot = int(off[-1])
        f = np.zeros(max(tot, 1), np.uint32)
        r = np.zeros(max(tot, 1), np.uint32)
        for i, x in enumerate(lists):
            if len(x):
                a = np.asarray(x, dtype=np.uint32).reshape(-1, 2)
                f[int(off[i]):int(off[i + 1])] = a[:, 0]
                r[int(off[i]):int(off[i + 1])] = a[:, 1]
        out = [np.zeros(max(n, 1), np.uint32) for _ in range(5)]
        _check(L.tm_chain_batch(self._h, n, _p(off, C.c_uint64), _p(f, C.c_uint32), _p(r, C.c_uint32),
                                *[_p(o, C.c_uint32) for o in out]), self._h)
        return [(int(out[0][i]), (int(out[1][i]), int(out[2][i])), (int(out[3][i]), int(out[4][i])))
                for i in range(n)]


class KMER:
    """team::KMER mirror: ``KMER(is_fwd).Minimize(seq, k, w)`` -> [(hash, pos, strand)]."""

    _mapper: Mapper | None = None

    def __init__(self, is_fwd: bool = True):
        self.is_fwd = bool(is_fwd)

    def Minimize(self, sequence: bytes, kmer_len: int, window_len: int):
        if KMER._mapper is None:
            KMER._mapper = Mapper(0)
        h, p = KMER._mapper.minimize_batch([sequence], kmer_len, window_len, False)[0]
        return [(int(a), int(b), self.is_fwd) for a, b in zip(h, p)]


def FindLIS(hits):
    """Chain summary of FindLIS on the GPU: (length, first hit, last hit)."""
    if KMER._mapper is None:
        KMER._mapper = Mapper(0)
    return KMER._mapper.chain_batch([hits])[0]


@dataclass
class MapResult:
    mapped: np.ndarray
    strand_fwd: np.ndarray
    q_begin: np.ndarray
    q_end: np.ndarray
    t_begin: np.ndarray
    t_end: np.ndarray
    scores: np.ndarray
    cigar_off: np.ndarray
    cigar_len: np.ndarray
    arena: np.ndarray

    def cigar(self, r):
        o = int(self.cigar_off[r])
        return self.arena[o:o + int(self.cigar_len[r])].tobytes()


class Index:
    """Reference minimizer index (both strands) resident in HBM."""

    def __init__(self, mapper: Mapper, name: str, seq: bytes, k=15, w=5, f=0.001):
        L = lib()
        self.mapper = mapper
        self.seq = np.frombuffer(bytes(seq) or b"\0", np.uint8).copy()
        h = C.c_void_p()
        _check(L.tm_index_create(mapper._h, name.encode(), self.seq.ctypes.data, len(seq), k, w, f, C.byref(h)),
               mapper._h)
        self._h = h
        self.k, self.w = k, w

    def stats(self):
        v = [C.c_uint64() for _ in range(4)] + [C.c_uint32() for _ in range(2)]
        _check(lib().tm_index_stats(self._h, *[C.byref(x) for x in v]))
        return dict(zip(["fwd_keys", "rev_keys", "fwd_positions", "rev_positions", "banned_fwd", "banned_rev"],
                        [x.value for x in v]))

    def map_batch(self, reads, opt: Options) -> MapResult:
        """reads: sequences, or a prepared (bytes, off, len) tuple (see soa())."""
        L = lib()
        b, off, ln = _soa(reads)
        n = len(ln)
        out = dict(mapped=np.zeros(n, np.uint8), strand_fwd=np.zeros(n, np.uint8), q_begin=np.zeros(n, np.uint32),
                   q_end=np.zeros(n, np.uint32), t_begin=np.zeros(n, np.uint32), t_end=np.zeros(n, np.uint32),
                   scores=np.zeros(n, np.int32), cigar_off=np.zeros(n, np.uint64), cigar_len=np.zeros(n, np.uint32))
        cap = int((4 * ln.astype(np.uint64) + 2).sum()) if n else 0
        arena = np.zeros(max(cap, 1), np.uint8)
        _check(L.tm_map_batch(self.mapper._h, self._h, n, b.ctypes.data, _p(off, C.c_uint64), _p(ln, C.c_uint32),
                              C.byref(opt), _p(out["mapped"], C.c_uint8), _p(out["strand_fwd"], C.c_uint8),
                              _p(out["q_begin"], C.c_uint32), _p(out["q_end"], C.c_uint32),
                              _p(out["t_begin"], C.c_uint32), _p(out["t_end"], C.c_uint32),
                              _p(out["scores"], C.c_int32), arena.ctypes.data, cap, _p(out["cigar_off"], C.c_uint64),
                              _p(out["cigar_len"], C.c_uint32)), self.mapper._h)
        return MapResult(arena=arena, **out)

    def close(self):
        if getattr(self, "_h", None):
            lib().tm_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def map_files(reference: str, reads: str, out: str = "-", device: int = 0, **opts) -> None:
    """The whole mapper on files, in process (tm_map_files)."""
    o = Options.make(**opts)
    _check(lib().tm_map_files(reference.encode(), reads.encode(), C.byref(o), out.encode(), device))


def run_cli(args, **kw) -> subprocess.CompletedProcess:
    """bioinfo1_amd/team_mapper_amd with the reference CLI's arguments."""
    return subprocess.run([CLI_PATH] + list(args), capture_output=True, **kw)
