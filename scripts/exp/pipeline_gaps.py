"""Experiment: GPU-side gaps in align.HostPipeline (config 2), unprofiled.
Events on the compute stream at each plan's start and end give the kernels'
busy time per step; host timestamps around the blocking waits show where the
host thread sleeps."""
import sys
import time

import torch

sys.path.insert(0, ".")
from bioinfo1_amd import synth  # noqa: E402
from bioinfo1_amd.align import Aligner, HostPipeline  # noqa: E402

b = synth.uniform_batch(10000, 1000, 1000, 0x5EED)
al = Aligner(0)
hp = HostPipeline(al, b, 1, 1, -1, -1, True)
for _ in range(3):
    hp.step()
hp.drain()
starts, ends = [], []
orig_run = [p.run for p in hp.plans]


def wrap(k):
    def run():
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(hp.compute)
        orig_run[k]()
        e1.record(hp.compute)
        starts.append(e0)
        ends.append(e1)
    return run


for k, p in enumerate(hp.plans):
    p.run = wrap(k)
waits = []
o_dl = hp._download


def dl(i, dst):
    t0 = time.perf_counter()
    o_dl(i, dst)
    waits.append((time.perf_counter() - t0) * 1e3)


hp._download = dl
t0 = time.perf_counter()
for _ in range(20):
    hp.step()
hp.drain()
dt = (time.perf_counter() - t0) / 20
busy = [s.elapsed_time(e) for s, e in zip(starts, ends)]
gap = [ends[k].elapsed_time(starts[k + 1]) for k in range(len(starts) - 1)]
print("pipeline %.3f ms/step" % (dt * 1e3))
print("plan busy (ms):", " ".join("%.2f" % x for x in busy))
print("gap to next plan (ms):", " ".join("%.2f" % x for x in gap))
print("host download waits (ms):", " ".join("%.2f" % x for x in waits))
