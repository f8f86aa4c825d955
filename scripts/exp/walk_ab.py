"""Experiment: fill / traceback time of config 2 under plan flags (default =
blocked layout + band walks; TA_PLAN_NO_BLK = the [step][lane] layout and the
lane walks), HIP events around each phase, 20 reps after warmup; also the
related-pairs variant.  Prints one line per (batch, flags)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from bioinfo1_amd import synth  # noqa: E402
from bioinfo1_amd.align import TA_PLAN_NO_BLK, Aligner, DevicePlan  # noqa: E402

al = Aligner(0)
for name, b in (("uniform", synth.uniform_batch(10000, 1000, 1000, 0x5EED)),
                ("related", synth.related_batch(10000, 1000, 1000, 0x5EED))):
    for flags in (0, TA_PLAN_NO_BLK):
        plan = DevicePlan(al, b, 1, 1, -1, -1, True, flags=flags)
        for _ in range(3):
            plan.run()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ft, tt = [], []
        for _ in range(20):
            ev[0].record()
            plan.run_fill(0)
            ev[1].record()
            plan.run_traceback(0)
            ev[2].record()
            torch.cuda.synchronize()
            ft.append(ev[0].elapsed_time(ev[1]))
            tt.append(ev[1].elapsed_time(ev[2]))
        r = plan.results()
        print(f"{name} flags={flags} blk={plan.blk} walk={plan.walk} fill {np.median(ft):.4f} ms "
              f"traceback {np.median(tt):.4f} ms  cigar bytes {int(r.cigar_lens.sum())}", flush=True)
        plan.close()
