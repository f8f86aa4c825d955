"""Experiment: host-to-host latency of small ta_align_batch_flags batches
(200x200 and 1000x1000 local pairs) under plan flags (BL_FLAGS, default
"1,0": the int32-fused plan vs the default plan; "0,128": the default plan vs
TA_PLAN_NO_BLK, the [step][lane] layout and lane walks)."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from bioinfo1_amd import synth  # noqa: E402
from bioinfo1_amd.align import Aligner, lib  # noqa: E402

L = lib()
al = Aligner(0)


def p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


for shape in [int(x) for x in os.environ.get("BL_SHAPES", "200,1000").split(",")]:
    for n in [int(x) for x in os.environ.get("BL_N", "1,2,4,8,16,64").split(",")]:
        b = synth.uniform_batch(n, shape, shape)
        cap = int((2 * (b.qlen.astype(np.uint64) + b.tlen.astype(np.uint64)) + 2).sum())
        arena = np.zeros(cap, np.uint8)
        sc = np.zeros(n, np.int32); tb = np.zeros(n, np.uint32); coff = np.zeros(n, np.uint64); clen = np.zeros(n, np.uint32)
        for flags in [int(x) for x in os.environ.get("BL_FLAGS", "1,0").split(",")]:
            ts = []
            for it in range(30):
                t0 = time.perf_counter()
                r = L.ta_align_batch_flags(al._h, n, b.qbytes.ctypes.data, p(b.qoff, C.c_uint64), p(b.qlen, C.c_uint32),
                                           b.tbytes.ctypes.data, p(b.toff, C.c_uint64), p(b.tlen, C.c_uint32), 1, 1, -1, -1,
                                           1, p(sc, C.c_int32), p(tb, C.c_uint32), arena.ctypes.data, cap,
                                           p(coff, C.c_uint64), p(clen, C.c_uint32), flags)
                ts.append(time.perf_counter() - t0)
                assert r == 0
            print(f"{shape}x{shape} n={n:3d} flags={flags}: p50 {1e6 * np.median(ts[5:]):8.1f} us", flush=True)
