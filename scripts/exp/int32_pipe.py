"""Experiment: the int32 fill's passes one after another on one wave
(TA_PLAN_SERIAL_PASSES) vs one wave per (pair, pass) (fill_pipe_kernel), on
batches whose pairs go to the int32 fill: local pairs past flex_local_fits.

Prints one line per (batch, flags): ms per plan run (fill + traceback, inputs
and results in HBM) and GCUPS; score/CIGAR equality between the two is
checked on every batch."""
import sys
import time

import torch

sys.path.insert(0, ".")
from bioinfo1_amd import synth  # noqa: E402
from bioinfo1_amd.align import TA_PLAN_SERIAL_PASSES, Aligner, DevicePlan  # noqa: E402

al = Aligner(0)
SC = (1, -1, -1)  # local: a 30 kb pair's score passes the int16 range
cases = [
    ("1 x 30kb x 30kb", synth.related_batch(1, 30000, 30000, seed=11)),
    ("16 x 20kb x 20kb (ma 2)", synth.related_batch(16, 20000, 20000, seed=12)),
    ("256 x 20kb x 20kb (ma 2)", synth.related_batch(256, 20000, 20000, seed=13)),
    ("2048 x 16kb x 16kb (ma 2)", synth.related_batch(2048, 16000, 16000, seed=14)),
]
for name, b in cases:
    sc = SC if b.n_pairs == 1 else (2, -1, -1)
    cells = float(sum(int(b.qlen[p]) * int(b.tlen[p]) for p in range(b.n_pairs)))
    res = {}
    for label, flags in (("serial", TA_PLAN_SERIAL_PASSES), ("pipelined", 0)):
        plan = DevicePlan(al, b, 1, *sc, True, flags=flags)
        assert plan.dual_pairs == 0, plan.dual_pairs
        plan.run()
        torch.cuda.synchronize()
        reps = 3 if cells > 1e11 else 10
        t0 = time.perf_counter()
        for _ in range(reps):
            plan.run()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        r = plan.results()
        res[label] = (r.scores.copy(), [r.cigar(p) for p in range(min(b.n_pairs, 64))])
        plan.check()
        plan.close()
        print("%-26s %-9s %9.2f ms  %7.1f GCUPS" % (name, label, ms, cells / ms / 1e6), flush=True)
    assert (res["serial"][0] == res["pipelined"][0]).all() and res["serial"][1] == res["pipelined"][1], name
# affine-gap local (the affine packed fill takes global / semi only: every local pair is an int32 single)
for name, b in (("affine local 16 x 10kb", synth.related_batch(16, 10000, 10000, seed=21)),
                ("affine local 1024 x 10kb", synth.related_batch(1024, 10000, 10000, seed=22))):
    cells = float(sum(int(b.qlen[p]) * int(b.tlen[p]) for p in range(b.n_pairs)))
    res = {}
    for label, flags in (("serial", TA_PLAN_SERIAL_PASSES), ("pipelined", 0)):
        plan = DevicePlan(al, b, 1, 2, -3, -1, True, gap_open=-5, flags=flags)
        plan.run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            plan.run()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 3 * 1e3
        r = plan.results()
        res[label] = (r.scores.copy(), [r.cigar(p) for p in range(min(b.n_pairs, 64))])
        plan.check()
        plan.close()
        print("%-26s %-9s %9.2f ms  %7.1f GCUPS" % (name, label, ms, cells / ms / 1e6), flush=True)
    assert (res["serial"][0] == res["pipelined"][0]).all() and res["serial"][1] == res["pipelined"][1], name
print("pipelined == serial on every batch")
