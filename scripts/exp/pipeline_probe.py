"""Experiment: where align.HostPipeline's steps spend host time (config 2)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from bioinfo1_amd import synth  # noqa: E402
from bioinfo1_amd.align import Aligner, DevicePlan, HostPipeline  # noqa: E402

b = synth.uniform_batch(10000, 1000, 1000, 0x5EED)
al = Aligner(0)
hp = HostPipeline(al, b, 1, 1, -1, -1, True)
for _ in range(3):
    hp.step()
hp.drain()
orig = hp._download
waits = []


def timed(i, dst):
    t0 = time.perf_counter()
    orig(i, dst)
    waits.append(time.perf_counter() - t0)


hp._download = timed
t0 = time.perf_counter()
steps = []
for _ in range(10):
    s0 = time.perf_counter()
    hp.step()
    steps.append(time.perf_counter() - s0)
hp.drain()
dt = (time.perf_counter() - t0) / 10
print("pipeline %.3f ms/step; host step calls (ms):" % (dt * 1e3), " ".join("%.2f" % (x * 1e3) for x in steps))
print("download waits (ms):", " ".join("%.2f" % (x * 1e3) for x in waits))
# the plans alone, back to back on one stream
p = hp.plans[0]
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    with torch.cuda.stream(hp.compute):
        p.run()
        p.compact_cigars()
torch.cuda.synchronize()
print("plan+compact alone %.3f ms" % ((time.perf_counter() - t0) / 10 * 1e3))
t0 = time.perf_counter()
for k in range(10):
    with torch.cuda.stream(hp.compute):
        hp.plans[k % 2].run()
torch.cuda.synchronize()
print("two plans alternating %.3f ms" % ((time.perf_counter() - t0) / 10 * 1e3))
