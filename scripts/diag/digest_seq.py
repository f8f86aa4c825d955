"""Diagnostic: the digest sequence of tests/test_gpu_parity.py::test_digest on
one context, then ragged_global again; prints mismatching pairs."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from conftest import digest_batch, load_digest  # noqa: E402

from bioinfo1_amd.align import Aligner, DevicePlan  # noqa: E402

al = Aligner(0)
seq = ["cfg2_local", "cfg2_related_local", "g1k_global", "s1k_semi", "ragged_local", "ragged_semi",
       "ragged_global", "ragged_global", "ragged_global"]
if len(sys.argv) > 1:
    seq = sys.argv[1].split(",")
for name in seq:
    meta, d = load_digest(name)
    b = digest_batch(name)
    for cig in (True, False):
        r = al.align_batch(b, meta["type"], meta["match"], meta["mismatch"], meta["gap"], cig)
        bad = np.nonzero(r.scores != d["scores"])[0]
        print(name, "cigar", cig, "bad", len(bad), flush=True)
        for p in bad[:8]:
            q = b.qbytes[b.qoff[p]:b.qoff[p] + b.qlen[p]].tobytes()
            t = b.tbytes[b.toff[p]:b.toff[p] + b.tlen[p]].tobytes()
            print("   pair", int(p), "n", int(b.qlen[p]), "m", int(b.tlen[p]), "got", int(r.scores[p]),
                  "want", int(d["scores"][p]), "qdash", b"-" in q, "tdash", b"-" in t, flush=True)
    if name == "ragged_global":
        pl = DevicePlan(al, b, meta["type"], meta["match"], meta["mismatch"], meta["gap"], True)
        print("   plan dual_pairs", pl.dual_pairs, "flex_pairs", pl.flex_pairs, "chunks", pl.chunks, flush=True)
        pl.close()
