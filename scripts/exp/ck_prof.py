"""Experiment: phase clock totals of the recomputing walk (library built with
-DTA_CK_PROF: scripts/exp/build_variant.sh ckprof walk_ck -DTA_CK_PROF)."""
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
import os
lanes = int(os.environ.get("CK_LANES", "16"))
waves = (10000 + 64 // lanes - 1) // (64 // lanes)
for it in range(3):
    L.ta_ck_prof(buf, 1)
    plan.run()
    torch.cuda.synchronize()
    L.ta_ck_prof(buf, 1)
    v = list(buf)
    print("iter", it, "related" if related else "uniform",
          "per wave: setup %.0f sweep %.0f walk %.0f total %.0f cycles | windows %.1f, walk iterations %.1f; counters 6, 7: %d %d" %
          (v[0] / waves, v[1] / waves, v[2] / waves, v[3] / waves, v[4] / waves, v[5] / waves, v[6], v[7]))
