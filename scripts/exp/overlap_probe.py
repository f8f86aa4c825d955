"""Experiment: does a pinned host->device copy on its own stream overlap with
the fill kernels (config 2 plan)?  Times 10 plan runs alone, the copies alone,
and both together."""
import sys
import time

import torch

sys.path.insert(0, ".")
from bioinfo1_amd import synth  # noqa: E402
from bioinfo1_amd.align import Aligner, DevicePlan  # noqa: E402

b = synth.uniform_batch(10000, 1000, 1000, 0x5EED)
al = Aligner(0)
plan = DevicePlan(al, b, 1, 1, -1, -1, True)
cs, us, ds = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
h = torch.empty(20_000_000, dtype=torch.uint8).pin_memory()
d = torch.empty(20_000_000, dtype=torch.uint8, device="cuda")
hd = torch.empty(9_000_000, dtype=torch.uint8).pin_memory()
dd = torch.empty(9_000_000, dtype=torch.uint8, device="cuda")


def run(k, plan_on, up_on, down_on):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        if plan_on:
            with torch.cuda.stream(cs):
                plan.run()
        if up_on:
            with torch.cuda.stream(us):
                d.copy_(h, non_blocking=True)
        if down_on:
            with torch.cuda.stream(ds):
                hd.copy_(dd, non_blocking=True)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


for _ in range(2):
    run(3, True, True, True)
print("plan alone        %.3f ms" % run(10, True, False, False))
print("H2D 20 MB alone   %.3f ms" % run(10, False, True, False))
print("D2H 9 MB alone    %.3f ms" % run(10, False, False, True))
print("plan + H2D        %.3f ms" % run(10, True, True, False))
print("plan + H2D + D2H  %.3f ms" % run(10, True, True, True))
