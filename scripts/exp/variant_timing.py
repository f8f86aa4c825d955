"""Config-2 step times with one input batch vs three rotated input batches in turn
(bench.py input_variants), serial (DevicePlan.run) and pipelined (DevicePipeline)."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

import bench  # noqa: E402
from bioinfo1_amd import synth  # noqa: E402
from bioinfo1_amd.align import Aligner, DevicePipeline, DevicePlan  # noqa: E402

b = synth.uniform_batch(10000, 1000, 1000, 0x5EED)
al = Aligner(0)
plan = DevicePlan(al, b, 1, 1, -1, -1, True)
var = bench.input_variants(plan, b)
torch.cuda.synchronize()


def timed(f, n=20):
    for _ in range(3):
        f(0)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for k in range(n):
        f(k)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


print("serial, one batch        %.3f ms" % timed(lambda k: plan.run()))
print("serial, same set_inputs  %.3f ms" % timed(lambda k: (plan.set_inputs(var[0][0]), plan.run())))
print("serial, rotated in turn  %.3f ms" % timed(lambda k: (plan.set_inputs(var[k % 3][0]), plan.run())))
plan.set_inputs(var[0][0])
pipe = DevicePipeline(0, b, 1, 1, -1, -1, True, first=plan)
print("pipelined, one batch     %.3f ms" % timed(lambda k: pipe.step()))
print("pipelined, rotated       %.3f ms" % timed(lambda k: pipe.step(inputs=var[k % 3][0])))
print("serial again, one batch  %.3f ms" % timed(lambda k: plan.run()))
print("serial again, rotated    %.3f ms" % timed(lambda k: (plan.set_inputs(var[k % 3][0]), plan.run())))
