"""Experiment: phase clock totals of the lane walk (library built with -DTA_LW_PROF)."""
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
    L.ta_lw_prof(buf, 1)
    plan.run()
    torch.cuda.synchronize()
    L.ta_lw_prof(buf, 1)
    waves = (10000 + 3) // 4
    v = list(buf)
    print("iter", it, "per wave: service-A %.0f  cells %.0f  service-B %.0f  total %.0f  outer-iters %.1f" %
          (v[0] / waves, v[1] / waves, v[2] / waves, v[3] / waves, v[4] / waves))
