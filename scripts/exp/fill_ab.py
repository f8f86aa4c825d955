"""Experiment: config-2 fill time alone (HIP events, 20 reps after warmup) of
the library in place; results are not read (checkpoint prototypes store no
codes)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from bioinfo1_amd import synth  # noqa: E402
from bioinfo1_amd.align import Aligner, DevicePlan  # noqa: E402

al = Aligner(0)
b = synth.uniform_batch(10000, 1000, 1000, 0x5EED)
for cigar in (True, False):
    plan = DevicePlan(al, b, 1, 1, -1, -1, cigar)
    for _ in range(3):
        plan.run_fill(0)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ft = []
    for _ in range(20):
        ev[0].record()
        plan.run_fill(0)
        ev[1].record()
        torch.cuda.synchronize()
        ft.append(ev[0].elapsed_time(ev[1]))
    print(f"cigar={cigar} blk={plan.blk} fill {np.median(ft):.4f} ms (min {min(ft):.4f})", flush=True)
    plan.close()
