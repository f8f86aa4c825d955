"""Python host-side mirror of the team_alignment interface.

``align()`` mirrors ``team::Align`` (/root/reference/team_alignment/
team_alignment.hpp:14-23): same arguments, same results -- the int score, the
CIGAR bytes the reference assigns to ``*cigar`` (``None`` when no CIGAR is
requested, like passing ``cigar = nullptr``) and ``*target_begin`` -- and the
same error: an unknown type raises ``ValueError("Unknown AlignmentType
provided.")`` (the reference's ``std::invalid_argument``).

``Aligner.align_batch()`` is the batched form (host memory in and out) and
``DevicePlan`` the device-resident form (torch CUDA tensors in HBM) used by
bench.py.  Everything goes through the extern "C" ABI of
``libteam_alignment.so`` (include/team_align_c.h) into the gfx950 HIP
kernels; there is no CPU fallback -- if the library or a gfx950 GPU is
missing, these raise.
"""
from __future__ import annotations

import ctypes as C
import enum
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libteam_alignment.so")

TA_OK, TA_ERR_BAD_TYPE, TA_ERR_CIGAR, TA_ERR_ARG, TA_ERR_DEVICE, TA_ERR_CAPACITY, TA_ERR_RANGE, TA_ERR_UNSERVED = range(8)
# ta_plan_create flags (include/team_align_c.h): kernel selection, same results
TA_PLAN_INT32_ONLY, TA_PLAN_NO_FLEX, TA_PLAN_UNFUSED, TA_PLAN_WALK1, TA_PLAN_WALK2 = 1, 2, 4, 8, 16
TA_PLAN_SERIAL_PASSES, TA_PLAN_PASS_MAJOR, TA_PLAN_NO_BLK, TA_PLAN_NO_CK, TA_PLAN_CK = 32, 64, 128, 256, 512
TA_PLAN_NO_FLEX_CK = 1024


class AlignmentType(enum.IntEnum):
    """team::AlignmentType (team_alignment.hpp:8-12), underlying int."""

    global_ = 0
    local = 1
    semiGlobal = 2


class DeviceError(RuntimeError):
    pass


_lib = None


def lib() -> C.CDLL:
    """Load libteam_alignment.so (fails loudly if it was not built).

    torch, when importable, is imported first so that the process has a single
    HIP runtime (torch's libamdhip64 satisfies the library's dependency)."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    u32p, u64p, i32p = C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), C.POINTER(C.c_int32)
    L.ta_status_string.restype = C.c_char_p
    L.ta_status_string.argtypes = [C.c_int]
    L.ta_last_error.restype = C.c_char_p
    L.ta_last_error.argtypes = [C.c_void_p]
    L.ta_context_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.ta_context_destroy.argtypes = [C.c_void_p]
    L.ta_context_destroy.restype = None
    L.ta_cigar_slot_bytes.restype = C.c_uint64
    L.ta_cigar_slot_bytes.argtypes = [C.c_uint32, C.c_uint32]
    L.ta_align_batch.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, u64p, u32p, C.c_void_p, u64p, u32p, C.c_int,
                                 C.c_int, C.c_int, C.c_int, C.c_int, i32p, u32p, C.c_void_p, C.c_uint64, u64p, u32p]
    L.ta_align_batch_flags.argtypes = L.ta_align_batch.argtypes + [C.c_uint32]
    L.ta_context_release.argtypes = [C.c_void_p]
    L.ta_context_release.restype = None
    L.ta_context_held_bytes.argtypes = [C.c_void_p]
    L.ta_context_held_bytes.restype = C.c_uint64
    L.ta_set_default_device.argtypes = [C.c_int]
    L.ta_set_thread_device.argtypes = [C.c_int]
    L.ta_plan_create.argtypes = [C.c_void_p, C.c_uint32, u32p, u32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_uint64, C.c_uint32, C.POINTER(C.c_void_p)]
    L.ta_plan_destroy.argtypes = [C.c_void_p]
    L.ta_plan_destroy.restype = None
    for f in ("ta_plan_cigar_slots_bytes", "ta_plan_workspace_bytes"):
        getattr(L, f).restype = C.c_uint64
        getattr(L, f).argtypes = [C.c_void_p]
    L.ta_plan_chunks.restype = C.c_uint32
    L.ta_plan_chunks.argtypes = [C.c_void_p]
    L.ta_plan_dual_pairs.restype = C.c_uint32
    L.ta_plan_dual_pairs.argtypes = [C.c_void_p]
    L.ta_plan_flex_pairs.restype = C.c_uint32
    L.ta_plan_flex_pairs.argtypes = [C.c_void_p]
    L.ta_plan_fused.argtypes = [C.c_void_p]
    L.ta_plan_walk.argtypes = [C.c_void_p]
    L.ta_plan_pair_chunks.argtypes = [C.c_void_p, u32p]
    L.ta_affine_plan_pair_chunks.argtypes = [C.c_void_p, u32p]
    L.ta_plan_execute.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.ta_plan_check.argtypes = [C.c_void_p]
    L.ta_compact_cigars.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_void_p]
    L.ta_plan_execute_fill.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]
    L.ta_plan_execute_traceback.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]
    # affine-gap extension (include/team_align_c.h, no reference counterpart)
    L.ta_align_batch_affine.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, u64p, u32p, C.c_void_p, u64p, u32p,
                                        C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, i32p, u32p, C.c_void_p,
                                        C.c_uint64, u64p, u32p]
    L.ta_affine_plan_create.argtypes = [C.c_void_p, C.c_uint32, u32p, u32p, C.c_int, C.c_int, C.c_int, C.c_int,
                                        C.c_int, C.c_int, C.c_uint64, C.c_uint32, C.POINTER(C.c_void_p)]
    L.ta_affine_plan_destroy.argtypes = [C.c_void_p]
    L.ta_affine_plan_destroy.restype = None
    for f in ("ta_affine_plan_cigar_slots_bytes", "ta_affine_plan_workspace_bytes"):
        getattr(L, f).restype = C.c_uint64
        getattr(L, f).argtypes = [C.c_void_p]
    L.ta_affine_plan_chunks.restype = C.c_uint32
    L.ta_affine_plan_chunks.argtypes = [C.c_void_p]
    L.ta_affine_plan_dual_pairs.restype = C.c_uint32
    L.ta_affine_plan_dual_pairs.argtypes = [C.c_void_p]
    L.ta_affine_plan_execute.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.ta_affine_plan_execute_fill.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]
    L.ta_affine_plan_execute_traceback.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]
    L.ta_affine_plan_check.argtypes = [C.c_void_p]
    # the low-latency single-pair server (ta_server_*)
    L.ta_server_create.argtypes = [C.c_int, C.c_int, C.c_uint32, C.POINTER(C.c_void_p)]
    L.ta_server_destroy.argtypes = [C.c_void_p]
    L.ta_server_destroy.restype = None
    L.ta_server_fits.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_int]
    L.ta_server_running.argtypes = [C.c_void_p]
    L.ta_server_last_times.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_double)]
    L.ta_server_align.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32, C.c_int, C.c_int,
                                  C.c_int, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_uint32), C.c_void_p,
                                  C.c_uint64, C.POINTER(C.c_uint32)]
    _lib = L
    return L


# Every symbol include/team_align_c.h declares (checked by tests/test_abi.py).
ABI_SYMBOLS = [
    "ta_status_string", "ta_last_error", "ta_context_create", "ta_context_destroy", "ta_context_release",
    "ta_context_held_bytes", "ta_set_default_device", "ta_set_thread_device", "ta_current_device", "ta_device_count",
    "ta_cigar_slot_bytes", "ta_align_batch", "ta_align_batch_flags", "ta_plan_create", "ta_plan_destroy", "ta_plan_cigar_slots_bytes",
    "ta_plan_workspace_bytes", "ta_plan_chunks", "ta_plan_dual_pairs", "ta_plan_flex_pairs", "ta_plan_fused", "ta_plan_walk",
    "ta_plan_execute", "ta_plan_check", "ta_plan_execute_fill", "ta_plan_pair_chunks", "ta_affine_plan_pair_chunks", "ta_plan_execute_traceback", "ta_compact_cigars",
    "ta_affine_plan_create", "ta_affine_plan_destroy", "ta_affine_plan_cigar_slots_bytes",
    "ta_affine_plan_workspace_bytes", "ta_affine_plan_chunks", "ta_affine_plan_dual_pairs", "ta_affine_plan_execute", "ta_affine_plan_execute_fill",
    "ta_affine_plan_execute_traceback", "ta_affine_plan_check", "ta_align_batch_affine",
    "ta_server_create", "ta_server_destroy", "ta_server_fits", "ta_server_align", "ta_server_running",
    "ta_server_last_times", "ta_server_pause", "ta_server_resume",
]
# The drop-in C++ entry point (team_alignment.hpp), g++/libstdc++ cxx11 mangling.
TEAM_ALIGN_SYMBOL = ("_ZN4team5AlignEPKcjS1_jNS_13AlignmentTypeEiiiPNSt7__cxx1112basic_stringIcSt11char_traitsIcESaIcEEEPj")


def _check_type(type) -> int:
    t = int(type)
    if t not in (0, 1, 2):
        raise ValueError("Unknown AlignmentType provided.")
    return t


def _raise(status: int, ctx=None):
    L = lib()
    msg = L.ta_status_string(status).decode()
    if status in (TA_ERR_BAD_TYPE, TA_ERR_CIGAR, TA_ERR_RANGE):
        raise ValueError(msg)
    detail = L.ta_last_error(ctx).decode() if ctx else ""
    raise DeviceError(f"{msg}: {detail}" if detail else msg)


def _p(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))


@dataclass
class BatchResult:
    scores: np.ndarray  # int32 [P]
    target_begins: np.ndarray  # uint32 [P]
    cigar_offsets: np.ndarray | None  # uint64 [P]
    cigar_lens: np.ndarray | None  # uint32 [P]
    arena: np.ndarray | None  # uint8

    def cigar(self, p: int) -> bytes | None:
        if self.arena is None:
            return None
        o = int(self.cigar_offsets[p])
        return self.arena[o : o + int(self.cigar_lens[p])].tobytes()

    def cigars(self):
        return [self.cigar(p) for p in range(len(self.scores))]


class Aligner:
    """A device context (HIP stream + staging buffers) on one gfx950 GPU."""

    def __init__(self, device: int = 0):
        L = lib()
        h = C.c_void_p()
        r = L.ta_context_create(device, C.byref(h))
        if r != TA_OK:
            raise DeviceError(f"ta_context_create(device={device}): {L.ta_status_string(r).decode()}")
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            lib().ta_context_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def release(self):
        """ta_context_release: free the cached device workspace and staging."""
        lib().ta_context_release(self._h)

    def align_batch(self, batch, type, match: int, mismatch: int, gap: int, want_cigar: bool = True) -> BatchResult:
        """Batched team::Align over a bioinfo1_amd.synth.PairBatch."""
        return self._batch(batch, type, (match, mismatch, gap), want_cigar, affine=False)

    def align_batch_affine(self, batch, type, match: int, mismatch: int, gap_open: int, gap_extend: int,
                           want_cigar: bool = True) -> BatchResult:
        """The affine-gap extension (ta_align_batch_affine): a gap of length L costs
        gap_open + L*gap_extend.  No reference counterpart; gap_open == 0 gives
        exactly team::Align with gap = gap_extend."""
        return self._batch(batch, type, (match, mismatch, gap_open, gap_extend), want_cigar, affine=True)

    def _batch(self, batch, type, scoring, want_cigar, affine) -> BatchResult:
        L = lib()
        t = _check_type(type)
        P = batch.n_pairs
        sc = np.zeros(P, np.int32)
        tb = np.zeros(P, np.uint32)
        coff = clen = arena = None
        cap = 0
        if want_cigar:
            cap = int((2 * (batch.qlen.astype(np.uint64) + batch.tlen.astype(np.uint64)) + 2).sum()) if P else 0
            arena = np.zeros(max(cap, 1), np.uint8)
            coff = np.zeros(P, np.uint64)
            clen = np.zeros(P, np.uint32)
        qb = batch.qbytes if batch.qbytes.size else np.zeros(1, np.uint8)
        tbb = batch.tbytes if batch.tbytes.size else np.zeros(1, np.uint8)
        fn = L.ta_align_batch_affine if affine else L.ta_align_batch
        r = fn(
            self._h, P, qb.ctypes.data, _p(batch.qoff, C.c_uint64), _p(batch.qlen, C.c_uint32), tbb.ctypes.data,
            _p(batch.toff, C.c_uint64), _p(batch.tlen, C.c_uint32), t, *scoring, int(bool(want_cigar)),
            _p(sc, C.c_int32), _p(tb, C.c_uint32), arena.ctypes.data if want_cigar else None, cap,
            _p(coff, C.c_uint64) if want_cigar else None, _p(clen, C.c_uint32) if want_cigar else None)
        if r != TA_OK:
            _raise(r, self._h)
        return BatchResult(sc, tb, coff, clen, arena)


_default: Aligner | None = None


def default_aligner() -> Aligner:
    global _default
    if _default is None:
        _default = Aligner(0)
    return _default


def align(query: bytes, target: bytes, type, match: int, mismatch: int, gap: int, want_cigar: bool = True):
    """team::Align for one pair -> (score, cigar bytes or None, target_begin)."""
    from .synth import from_pairs

    _check_type(type)
    res = default_aligner().align_batch(from_pairs([(bytes(query), bytes(target))]), type, match, mismatch, gap,
                                        want_cigar)
    return int(res.scores[0]), res.cigar(0), int(res.target_begins[0])


def align_affine(query: bytes, target: bytes, type, match: int, mismatch: int, gap_open: int, gap_extend: int,
                 want_cigar: bool = True):
    """The affine-gap extension for one pair -> (score, cigar bytes or None, target_begin)."""
    from .synth import from_pairs

    _check_type(type)
    res = default_aligner().align_batch_affine(from_pairs([(bytes(query), bytes(target))]), type, match, mismatch,
                                               gap_open, gap_extend, want_cigar)
    return int(res.scores[0]), res.cigar(0), int(res.target_begins[0])


class Server:
    """The low-latency single-pair path (ta_server_*): a resident kernel, one
    wave per slot, serves one team::Align call at a time per slot -- what the
    drop-in team::Align uses for pairs up to 4096 x 16384.  align() returns
    (score, cigar bytes or None, target_begin) like align(); a pair outside
    the server's limits raises LookupError (the caller takes a batch)."""

    def __init__(self, device: int, type, slots: int = 32):
        L = lib()
        h = C.c_void_p()
        r = L.ta_server_create(device, _check_type(type), slots, C.byref(h))
        if r != TA_OK:
            _raise(r)
        self._h = h
        self.type = int(type)

    def fits(self, n: int, m: int, match: int, mismatch: int, gap: int) -> bool:
        return bool(lib().ta_server_fits(self._h, n, m, match, mismatch, gap))

    def running(self) -> bool:
        return bool(lib().ta_server_running(self._h))

    def last_times(self, slot: int = 0):
        """Device phase times (us) of slot's last request: request + bytes to HBM,
        fill + walk, results out, 0 (the release store of `done` is the fence)."""
        out = (C.c_double * 4)()
        r = lib().ta_server_last_times(self._h, slot, out)
        if r != TA_OK:
            _raise(r)
        return list(out)

    def align(self, query: bytes, target: bytes, match: int, mismatch: int, gap: int, want_cigar: bool = True):
        query, target = bytes(query), bytes(target)
        cap = 2 * (len(query) + len(target)) + 2
        buf = C.create_string_buffer(cap) if want_cigar else None
        sc, tb, cl = C.c_int32(0), C.c_uint32(0), C.c_uint32(0)
        r = lib().ta_server_align(self._h, query, len(query), target, len(target), match, mismatch, gap,
                                  int(bool(want_cigar)), C.byref(sc), C.byref(tb), buf, cap, C.byref(cl))
        if r == TA_ERR_UNSERVED:
            raise LookupError("pair outside the single-pair server's limits")
        if r != TA_OK:
            _raise(r)
        return sc.value, (buf.raw[: cl.value] if want_cigar else None), tb.value

    def close(self):
        if getattr(self, "_h", None):
            lib().ta_server_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _DeviceIO(C.Structure):
    _fields_ = [("query_bytes", C.c_void_p), ("query_off", C.c_void_p), ("target_bytes", C.c_void_p),
                ("target_off", C.c_void_p), ("score", C.c_void_p), ("target_begin", C.c_void_p),
                ("cigar_slots", C.c_void_p), ("cigar_start", C.c_void_p), ("cigar_len", C.c_void_p)]


def _results(o) -> BatchResult:
    o.torch.cuda.synchronize(o.dev)
    sc = o.score.cpu().numpy()
    tb = o.target_begin.cpu().numpy().view(np.uint32)
    if not o.want_cigar:
        return BatchResult(sc, tb, None, None, None)
    start = o.cigar_start.cpu().numpy().view(np.uint64)
    ln = o.cigar_len.cpu().numpy().view(np.uint32)
    slots = o.slots.cpu().numpy()
    return BatchResult(sc, tb, start, ln, slots)


class DevicePlan:
    """Device-resident batch: inputs and outputs are torch tensors in HBM.

    Mirrors the mapper-side batching of SURVEY §8f: lengths and scoring are
    fixed at plan time; ``run()`` enqueues the fill + traceback kernels on the
    current torch stream (asynchronous)."""

    def __init__(self, aligner: Aligner, batch, type, match, mismatch, gap, want_cigar=True, device=None,
                 workspace_budget: int = 0, gap_open=None, flags: int = 0, inputs=None, records=None):
        """gap_open=None: team::Align's linear gap.  gap_open=o: the affine-gap
        extension (ta_affine_plan_*) with gap_extend = gap.  flags: TA_PLAN_*
        kernel selection (tests / measurements; same results).  inputs: the
        batch already in HBM as (query bytes, query offsets, target bytes,
        target offsets) tensors -- then only batch.qlen / batch.tlen are read.
        records: an int32 device tensor of >= 3 * P entries that receives the
        scores, target_begins and CIGAR lengths back to back (one download)."""
        import torch

        L = lib()
        t = _check_type(type)
        self.torch = torch
        self.dev = torch.device("cuda", aligner.device) if device is None else device
        self.P = batch.n_pairs
        self.want_cigar = bool(want_cigar)
        self.affine = gap_open is not None
        self._fn = (lambda name: getattr(L, name.replace("ta_plan_", "ta_affine_plan_"))) if self.affine else \
            (lambda name: getattr(L, name))
        h = C.c_void_p()
        scoring = (match, mismatch, gap_open, gap) if self.affine else (match, mismatch, gap)
        r = self._fn("ta_plan_create")(aligner.handle, self.P, _p(batch.qlen, C.c_uint32),
                                       _p(batch.tlen, C.c_uint32), t, *scoring, int(self.want_cigar),
                                       workspace_budget, flags, C.byref(h))
        if r != TA_OK:
            _raise(r, aligner.handle)
        self._h = h
        self._ctx = aligner.handle
        if inputs is None:
            f = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.dev)  # noqa: E731
            self.qbytes = f(batch.qbytes if batch.qbytes.size else np.zeros(1, np.uint8))
            self.tbytes = f(batch.tbytes if batch.tbytes.size else np.zeros(1, np.uint8))
            self.qoff = f(batch.qoff.view(np.int64))
            self.toff = f(batch.toff.view(np.int64))
        else:
            self.qbytes, self.qoff, self.tbytes, self.toff = inputs
        if records is not None:
            assert records.dtype == torch.int32 and records.numel() >= 3 * self.P and records.is_contiguous()
            self.score, self.target_begin = records[:self.P], records[self.P:2 * self.P]
        else:
            self.score = torch.zeros(self.P, dtype=torch.int32, device=self.dev)
            self.target_begin = torch.zeros(self.P, dtype=torch.int32, device=self.dev)
        self.slots_bytes = int(self._fn("ta_plan_cigar_slots_bytes")(h))
        self.slots = torch.zeros(max(self.slots_bytes, 1) if self.want_cigar else 1, dtype=torch.uint8,
                                 device=self.dev)
        self.cigar_start = torch.zeros(self.P, dtype=torch.int64, device=self.dev)
        self.cigar_len = (records[2 * self.P:3 * self.P] if records is not None
                          else torch.zeros(self.P, dtype=torch.int32, device=self.dev))
        self.io = _DeviceIO(self.qbytes.data_ptr(), self.qoff.data_ptr(), self.tbytes.data_ptr(),
                            self.toff.data_ptr(), self.score.data_ptr(), self.target_begin.data_ptr(),
                            self.slots.data_ptr(), self.cigar_start.data_ptr(), self.cigar_len.data_ptr())
        self.workspace_bytes = int(self._fn("ta_plan_workspace_bytes")(h))
        self.chunks = int(self._fn("ta_plan_chunks")(h))
        self.dual_pairs = int(L.ta_affine_plan_dual_pairs(h)) if self.affine else int(L.ta_plan_dual_pairs(h))
        self.flex_pairs = 0 if self.affine else int(L.ta_plan_flex_pairs(h))
        self.fused = False if self.affine else bool(L.ta_plan_fused(h))
        w = -1 if self.affine else int(L.ta_plan_walk(h))
        self.walk, self.blk, self.ck = (w & 0xFF, bool(w & 0x100), bool(w & 0x200)) if w >= 0 else (None, False, False)
        self.aligner = aligner

    def _stream(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.dev).cuda_stream)

    def set_inputs(self, inputs):
        """Point the plan at another batch of the same shapes already in HBM:
        (query bytes, query offsets, target bytes, target offsets) tensors --
        pair p must keep its planned lengths.  Takes effect for the launches
        enqueued after the call; the caller keeps the tensors unmodified until
        those launches are done."""
        q, qo, t, to = inputs
        assert q.device == self.dev and t.device == self.dev and qo.numel() >= self.P and to.numel() >= self.P
        self.qbytes, self.qoff, self.tbytes, self.toff = q, qo, t, to
        self.io.query_bytes, self.io.query_off = q.data_ptr(), qo.data_ptr()
        self.io.target_bytes, self.io.target_off = t.data_ptr(), to.data_ptr()

    def run(self):
        r = self._fn("ta_plan_execute")(self._h, C.byref(self.io), self._stream())
        if r != TA_OK:
            _raise(r, self._ctx)

    def run_fill(self, chunk: int = 0):
        r = self._fn("ta_plan_execute_fill")(self._h, C.byref(self.io), self._stream(), chunk)
        if r != TA_OK:
            _raise(r, self._ctx)

    def run_traceback(self, chunk: int = 0):
        r = self._fn("ta_plan_execute_traceback")(self._h, C.byref(self.io), self._stream(), chunk)
        if r != TA_OK:
            _raise(r, self._ctx)

    def check(self):
        """ta_plan_check after synchronising: raises DeviceError if a kernel reported an internal failure."""
        self.torch.cuda.synchronize(self.dev)
        r = self._fn("ta_plan_check")(self._h)
        if r != TA_OK:
            _raise(r, self._ctx)

    def compact_cigars(self, out=None):
        """The CIGARs packed back to back on the device (ta_compact_cigars on
        the current stream): returns (bytes uint8 tensor, int64 offsets
        tensor [P+1]) -- what a rank hands to an RCCL gather.  ``out``: a
        (bytes, offsets) pair from compact_buffers() to fill instead of fresh
        tensors (a pipeline reusing them per slot)."""
        torch = self.torch
        lens = self.cigar_len.to(torch.int64)
        if out is None:
            off = torch.zeros(self.P + 1, dtype=torch.int64, device=self.dev)
            # a device-side bound keeps this free of host syncs: every CIGAR fits its slot
            dst = torch.empty(max(self.slots_bytes, 1), dtype=torch.uint8, device=self.dev)
        else:
            dst, off = out
        torch.cumsum(lens, 0, out=off[1:])
        r = lib().ta_compact_cigars(self._ctx, self.P, self.slots.data_ptr(), self.cigar_start.data_ptr(),
                                    self.cigar_len.data_ptr(), off.data_ptr(), dst.data_ptr(), self._stream())
        if r != TA_OK:
            _raise(r, self._ctx)
        return dst, off

    def compact_buffers(self):
        """Buffers for compact_cigars(out=...): (bytes, offsets with offsets[0] = 0)."""
        torch = self.torch
        return (torch.empty(max(self.slots_bytes, 1), dtype=torch.uint8, device=self.dev),
                torch.zeros(self.P + 1, dtype=torch.int64, device=self.dev))

    def pair_chunks(self) -> np.ndarray:
        """uint32 [P]: the chunk each pair ran in (ta_plan_pair_chunks)."""
        out = np.zeros(max(self.P, 1), np.uint32)
        r = self._fn("ta_plan_pair_chunks")(self._h, _p(out, C.c_uint32))
        if r != TA_OK:
            _raise(r, self._ctx)
        return out[: self.P]

    def results_at(self, indices) -> BatchResult:
        """Synchronise, check and copy the results of the pairs ``indices`` only
        (the stratified parity checks of a stated-size run): a BatchResult whose
        k-th entry is pair indices[k]."""
        torch = self.torch
        self.check()
        idx = torch.as_tensor(np.asarray(indices, np.int64), device=self.dev)
        sc = self.score[idx].cpu().numpy()
        tb = self.target_begin[idx].cpu().numpy().view(np.uint32)
        if not self.want_cigar:
            return BatchResult(sc, tb, None, None, None)
        start = self.cigar_start[idx].cpu().numpy()
        ln = self.cigar_len[idx].cpu().numpy().view(np.uint32)
        parts, offs, o = [], np.zeros(len(ln), np.uint64), 0
        for k in range(len(ln)):
            parts.append(self.slots[int(start[k]):int(start[k]) + int(ln[k])].cpu().numpy())
            offs[k] = o
            o += int(ln[k])
        arena = np.concatenate(parts) if parts else np.zeros(1, np.uint8)
        return BatchResult(sc, tb, offs, ln, arena)

    def results(self) -> BatchResult:
        """Synchronise, check and copy results to host (CIGARs unpacked from slots)."""
        self.check()
        return _results(self)

    def close(self):
        if getattr(self, "_h", None):
            self._fn("ta_plan_destroy")(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DevicePipeline:
    """Device-resident batches aligned back to back with batch k's traceback
    running beside batch k+1's fill.

    The traceback of a batch is one long serial walk per pair -- latency-bound,
    about one wave per SIMD -- while the fill is VALU-bound with
    many waves per SIMD, so the two overlap well on one GPU.  Each slot is a
    DevicePlan on its own Aligner context: the context owns the workspace the
    fill writes and the walk reads, and ta_plan_execute_fill / _traceback order
    one context's launches across streams (a slot's traceback waits for its
    fill, its next fill for that traceback).  Fills run on the pipeline's fill
    stream, tracebacks on its high-priority walk stream, and the caller's
    current stream waits for each step's traceback, so whatever the caller
    enqueues after step() on its stream (a compaction, a gather, the next
    upload into this step's input buffers) follows it; a slot's next fill also
    waits for that.

    Inputs: every step may align another batch of the planned shapes
    (step(inputs=...), tensors in HBM); the step's fill waits for the
    ``ready`` event (recorded after the batch's upload, e.g. on a copy stream).
    Without ``ready`` the inputs must already be resident (written before the
    pipeline was built, or synchronised): waiting on the caller's stream would
    also wait for the previous step's traceback and serialise the pipeline.  A
    step without inputs realigns the slot's last batch (at construction: the
    shared first batch).  Memory: ``depth`` workspaces."""

    def __init__(self, device: int, batch, type, match, mismatch, gap, want_cigar=True, depth: int = 2,
                 workspace_budget: int = 0, gap_open=None, flags: int = 0, inputs=None, first=None):
        """first: an existing DevicePlan (on its own Aligner) to use as slot 0;
        the other slots then start on its inputs."""
        import torch

        self.torch = torch
        self.dev = torch.device("cuda", device)
        self.aligners, self.plans = [], []
        for k in range(depth):
            if k == 0 and first is not None:
                self.plans.append(first)
                continue
            al = Aligner(device)
            self.aligners.append(al)
            shared = inputs if not self.plans else (self.plans[0].qbytes, self.plans[0].qoff,
                                                    self.plans[0].tbytes, self.plans[0].toff)
            self.plans.append(DevicePlan(al, batch, type, match, mismatch, gap, want_cigar,
                                         workspace_budget=workspace_budget, gap_open=gap_open, flags=flags,
                                         inputs=shared))
        # the tracebacks on a high-priority stream: HIP gives it a hardware queue
        # of its own (streams of one priority share GPU_MAX_HW_QUEUES queues, and
        # the kernels of one queue run one after the other)
        self.fill = torch.cuda.Stream(self.dev)
        self.walk = torch.cuda.Stream(self.dev, priority=-1)
        for st in (self.fill, self.walk):
            st.wait_stream(torch.cuda.current_stream(self.dev))  # (the inputs' uploads)
        self.walked = [torch.cuda.Event() for _ in range(depth)]
        self.done = [torch.cuda.Event() for _ in range(depth)]
        self.used = [False] * depth
        self.k = 0
        self.last = None

    @property
    def chunks(self):
        return self.plans[0].chunks

    def step(self, inputs=None, ready=None):
        """Enqueue one batch: its fill on the fill stream, its traceback on the
        walk stream (the current stream waits for it).  inputs: this batch's
        (query bytes, query offsets, target bytes, target offsets) tensors in
        HBM, same shapes as planned; ready: an event the fill waits for first
        (None: the inputs are resident).  Returns the slot's
        DevicePlan (its results are ready on the current stream after the call;
        the inputs may be overwritten by work enqueued on it after the call)."""
        torch = self.torch
        cur = torch.cuda.current_stream(self.dev)
        depth = len(self.plans)
        if self.last is not None:  # the previous slot's traceback and what the caller queued after it
            self.done[self.last].record(cur)
        i = self.k % depth
        self.k += 1
        plan = self.plans[i]
        if self.used[i]:
            self.fill.wait_event(self.done[i])
        if inputs is not None:
            plan.set_inputs(inputs)
            if ready is not None:
                self.fill.wait_event(ready)
        for c in range(plan.chunks):
            with torch.cuda.stream(self.fill):
                plan.run_fill(c)
            with torch.cuda.stream(self.walk):
                plan.run_traceback(c)  # (waits for the fill: the slot's context orders them)
        self.walked[i].record(self.walk)
        cur.wait_event(self.walked[i])
        self.used[i] = True
        self.last = i
        return plan

    def check(self):
        for p in self.plans:
            p.check()

    def close(self):
        for p in self.plans:
            p.close()
        for al in self.aligners:
            al.close()


class HostBatchRunner:
    """Repeated host-memory batches (ta_align_batch) over one batch whose
    inputs and outputs live in pinned host memory (torch pin_memory, i.e.
    hipHostMalloc): what a caller that keeps its reads in pinned buffers gets
    host-to-host.  run() is one call: upload, kernels, download, sync."""

    def __init__(self, aligner: Aligner, batch, type, match, mismatch, gap, want_cigar=True):
        import torch

        self.t = _check_type(type)
        self.sc = (match, mismatch, gap)
        self.want_cigar = bool(want_cigar)
        self.aligner = aligner
        self.P = P = batch.n_pairs

        def pinned(a):
            a = np.ascontiguousarray(a)
            t = torch.empty(max(a.nbytes, 1), dtype=torch.uint8, pin_memory=True)
            v = t.numpy()[: a.nbytes].view(a.dtype)
            v[...] = a.reshape(-1)
            return t, v

        self._keep = []
        for name, a in (("qb", batch.qbytes if batch.qbytes.size else np.zeros(1, np.uint8)), ("qoff", batch.qoff),
                        ("qlen", batch.qlen), ("tb", batch.tbytes if batch.tbytes.size else np.zeros(1, np.uint8)),
                        ("toff", batch.toff), ("tlen", batch.tlen), ("score", np.zeros(P, np.int32)),
                        ("tbeg", np.zeros(P, np.uint32)), ("coff", np.zeros(P, np.uint64)),
                        ("clen", np.zeros(P, np.uint32))):
            t, v = pinned(a)
            self._keep.append(t)
            setattr(self, name, v)
        cap = int((2 * (batch.qlen.astype(np.uint64) + batch.tlen.astype(np.uint64)) + 2).sum()) if P else 1
        t, self.arena = pinned(np.zeros(max(cap, 1), np.uint8))
        self._keep.append(t)
        self.cap = cap

    def run(self):
        L = lib()
        r = L.ta_align_batch(
            self.aligner.handle, self.P, self.qb.ctypes.data, _p(self.qoff, C.c_uint64), _p(self.qlen, C.c_uint32),
            self.tb.ctypes.data, _p(self.toff, C.c_uint64), _p(self.tlen, C.c_uint32), self.t, *self.sc,
            int(self.want_cigar), _p(self.score, C.c_int32), _p(self.tbeg, C.c_uint32), self.arena.ctypes.data,
            self.cap, _p(self.coff, C.c_uint64), _p(self.clen, C.c_uint32))
        if r != TA_OK:
            _raise(r, self.aligner.handle)

    def results(self) -> BatchResult:
        if not self.want_cigar:
            return BatchResult(self.score.copy(), self.tbeg.copy(), None, None, None)
        return BatchResult(self.score.copy(), self.tbeg.copy(), self.coff.copy(), self.clen.copy(), self.arena.copy())


class HostPipeline:
    """Host-resident batches aligned back to back with the PCIe transfers hidden:
    batch k's upload runs on an upload stream and batch k-1's download on a
    download stream while the kernels run on the compute stream.  Inputs are the
    batch's bytes in pinned host memory; every step uploads them, runs the plan,
    compacts the CIGARs on the device and brings the records and the compacted
    CIGAR bytes back into pinned host memory (host inputs to host
    results).

    Two DevicePlans alternate (double-buffered device inputs and outputs), each
    on an Aligner context of its own (the given one and a second), so that, as
    in DevicePipeline, batch k's traceback (high-priority walk stream) runs
    beside batch k+1's fill (fill stream).  Step k enqueues its upload and
    kernels, then waits for step k-1's kernels and downloads step k-1's records
    (12 bytes per pair) and exactly its CIGAR bytes.  Every copy is posted only
    once its data is ready: a copy enqueued ahead of its data (waiting on an
    event) holds its DMA engine, and an upload queued behind it then waits for
    a whole plan (measured: a 0.45 ms bubble every other step)."""

    def __init__(self, aligner: Aligner, batch, type, match, mismatch, gap, want_cigar=True, workspace_budget=0,
                 overlap: bool = True):
        """overlap=False: both slots on ``aligner``'s context, one stream for
        the kernels (each batch's fill after the previous traceback)."""
        import torch

        self.torch = torch
        self.P = P = batch.n_pairs
        self.want_cigar = bool(want_cigar)
        dev = torch.device("cuda", aligner.device)
        self.dev = dev
        qb = batch.qbytes if batch.qbytes.size else np.zeros(1, np.uint8)
        tb = batch.tbytes if batch.tbytes.size else np.zeros(1, np.uint8)
        # query and target bytes in one pinned buffer and one device buffer per
        # slot: one H2D copy per step
        nq = int(qb.size)
        self.h_qt = torch.from_numpy(np.concatenate([np.ascontiguousarray(qb), np.ascontiguousarray(tb)])).pin_memory()
        qoff = torch.from_numpy(batch.qoff.view(np.int64).copy()).to(dev)
        toff = torch.from_numpy(batch.toff.view(np.int64).copy()).to(dev)
        self.d_qt = [torch.empty_like(self.h_qt, device=dev) for _ in range(2)]
        self.d_q = [self.d_qt[i][:nq] for i in range(2)]
        self.d_t = [self.d_qt[i][nq:] for i in range(2)]
        # per slot: scores, target_begins, CIGAR lengths (written there by the plan) + the CIGAR byte total
        self.d_rec = [torch.zeros(3 * P + 1, dtype=torch.int32, device=dev) for _ in range(2)]
        self.second = Aligner(aligner.device) if overlap else None
        self.plans = [DevicePlan(al, batch, type, match, mismatch, gap, want_cigar,
                                 workspace_budget=workspace_budget, inputs=(self.d_q[i], qoff, self.d_t[i], toff),
                                 records=self.d_rec[i])
                      for i, al in enumerate((aligner, self.second or aligner))]
        self.fill, self.up, self.down = (torch.cuda.Stream(dev) for _ in range(3))
        # tracebacks + compaction (DevicePipeline.walk); without overlap the fills run there too
        self.compute = torch.cuda.Stream(dev, priority=-1) if overlap else self.fill
        self.h_rec = [torch.empty(3 * P + 1, dtype=torch.int32, pin_memory=True) for _ in range(2)]
        cap = max(self.plans[0].slots_bytes, 1)
        self.h_cig = [torch.empty(cap, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        E = lambda: [torch.cuda.Event() for _ in range(2)]  # noqa: E731
        self.ev_in, self.ev_done, self.ev_rec, self.ev_cig = E(), E(), E(), E()
        # per slot: the compacted CIGAR bytes and offsets, allocated once
        self.cbuf = [self.plans[i].compact_buffers() for i in range(2)] if self.want_cigar else [None, None]
        self.used = [False, False]  # slot has a step in flight (its downloads may still run)
        self.prev = None            # (slot, device CIGAR bytes) of the previous step
        self.last = None
        self.k = 0

    def _download(self, i, dst):
        """Slot i's step, once its kernels are done: the records, then exactly
        its CIGAR bytes (posted only now that their data is ready)."""
        torch = self.torch
        self.ev_done[i].synchronize()  # the step's kernels are done
        with torch.cuda.stream(self.down):
            self.h_rec[i].copy_(self.d_rec[i], non_blocking=True)
            self.ev_rec[i].record(self.down)
        if self.want_cigar:
            self.ev_rec[i].synchronize()
            nbytes = int(self.h_rec[i][3 * self.P])
            with torch.cuda.stream(self.down):
                if nbytes:
                    self.h_cig[i][:nbytes].copy_(dst[:nbytes], non_blocking=True)
                self.ev_cig[i].record(self.down)
        else:
            self.ev_cig[i] = self.ev_rec[i]
        self.last = i

    def step(self):
        torch, P = self.torch, self.P
        i = self.k % 2
        self.k += 1
        # inputs of this step: the kernels of two steps ago (slot i) are done (the
        # host saw them finish during the previous step)
        with torch.cuda.stream(self.up):
            self.d_qt[i].copy_(self.h_qt, non_blocking=True)
            self.ev_in[i].record(self.up)
        plan = self.plans[i]
        with torch.cuda.stream(self.fill):
            self.fill.wait_event(self.ev_in[i])
            if self.used[i]:  # the slot's results of two steps ago are down (a wait on the device)
                self.fill.wait_event(self.ev_cig[i])
            for c in range(plan.chunks):
                plan.run_fill(c)
                with torch.cuda.stream(self.compute):
                    plan.run_traceback(c)  # (after its fill: the slot's context orders them)
        with torch.cuda.stream(self.compute):
            rec = self.d_rec[i]
            dst = None
            if self.want_cigar:
                dst, off = plan.compact_cigars(out=self.cbuf[i])
                rec[3 * P:].copy_(off[-1:], non_blocking=True)
            self.ev_done[i].record(self.compute)
        self.used[i] = True
        if self.prev is not None:  # the previous step's results (its kernels end as this step's begin)
            self._download(*self.prev)
        self.prev = (i, dst)

    def drain(self):
        if self.prev is not None:
            self._download(*self.prev)
            self.prev = None
        self.torch.cuda.synchronize(self.dev)

    def results(self) -> BatchResult:
        """The last drained step's results (host copies)."""
        i, P = self.last, self.P
        rec = self.h_rec[i].numpy()
        sc = rec[:P].copy()
        tb = rec[P:2 * P].copy().view(np.uint32)
        if not self.want_cigar:
            return BatchResult(sc, tb, None, None, None)
        ln = rec[2 * P:3 * P].copy().view(np.uint32)
        off = np.zeros(P, np.uint64)
        if P:
            off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
        return BatchResult(sc, tb, off, ln, self.h_cig[i].numpy()[:int(rec[3 * P])].copy())

    def close(self):
        for p in self.plans:
            p.close()
        if self.second:
            self.second.close()
