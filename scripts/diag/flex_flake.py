"""Diagnostic: repeat the ragged digest batches and report mismatching pairs
(index, lengths) per run, with the flexible fill on and off."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from conftest import digest_batch, load_digest  # noqa: E402

from bioinfo1_amd.align import Aligner  # noqa: E402

al = Aligner(0)
for name in ("ragged_global", "ragged_semi"):
    meta, d = load_digest(name)
    b = digest_batch(name)
    for flex in ("1", "0"):
        os.environ["TA_FLEX"] = flex
        bad_runs = 0
        for it in range(12):
            for cig in (True, False):
                r = al.align_batch(b, meta["type"], meta["match"], meta["mismatch"], meta["gap"], cig)
                bad = np.nonzero(r.scores != d["scores"])[0]
                if len(bad):
                    bad_runs += 1
                    print(name, "flex", flex, "it", it, "cigar", cig, "bad", [(int(p), int(b.qlen[p]), int(b.tlen[p]),
                          int(r.scores[p]), int(d["scores"][p])) for p in bad[:6]], flush=True)
        print(name, "flex", flex, "bad runs", bad_runs, "of 24", flush=True)
