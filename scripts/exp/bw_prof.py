"""Experiment: phase clock totals of the band walk (library built with -DTA_BW_PROF)."""
import ctypes as C
import sys

import torch

sys.path.insert(0, ".")
from bioinfo1_amd import synth  # noqa: E402
from bioinfo1_amd.align import Aligner, DevicePlan, lib  # noqa: E402

related = "--related" in sys.argv
b = synth.related_batch(10000, 1000, 1000) if related else synth.uniform_batch(10000, 1000, 1000)
al = Aligner(0)
plan = DevicePlan(al, b, 1, 1, -1, -1, True)
L = lib()
buf = (C.c_ulonglong * 8)()
for it in range(3):
    L.ta_bw_prof(buf, 1)
    plan.run()
    torch.cuda.synchronize()
    L.ta_bw_prof(buf, 1)
    waves = (10000 + 63) // 64
    v = list(buf)
    print("iter", it, "related" if related else "uniform", "per wave: commit %.0f issue %.0f flush %.0f walk %.0f total %.0f"
          " rounds %.1f | per pair: walk iters %.0f stalled iters %.0f" %
          (v[0] / waves, v[1] / waves, v[2] / waves, v[3] / waves, v[4] / waves, v[5] / waves, v[7] / 10000, v[6] / 10000))
