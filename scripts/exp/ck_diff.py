"""Experiment: which pairs of test_band_walk case 1 (and a config-2 slice) differ
from the oracle under the library in place; prints pair, shape, got, want."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from bioinfo1_amd import synth  # noqa: E402
from bioinfo1_amd.align import Aligner  # noqa: E402
from conftest import run_plan  # noqa: E402
import test_gpu_parity as T  # noqa: E402

al = Aligner(0)
for case in (0, 1, 2):
    sc, qa, ta, shapes, walk = T.BAND_CASES[case]
    rng = np.random.default_rng(0xBA4D + case)
    qa, ta = np.frombuffer(qa, np.uint8), np.frombuffer(ta, np.uint8)
    pairs = []
    for k in range(2 * len(shapes) * 4):
        n, m = shapes[(k // 2) % len(shapes)]
        pairs.append((qa[rng.integers(len(qa), size=n)].tobytes(), ta[rng.integers(len(ta), size=m)].tobytes()))
    b = synth.from_pairs(pairs)
    got = run_plan(al, b, 1, sc, True, 0)
    want = run_plan(al, b, 1, sc, True, T.TA_PLAN_NO_CK)
    bad = [p for p in range(b.n_pairs) if got.cigar(p) != want.cigar(p)]
    print("case", case, "pairs", b.n_pairs, "bad", len(bad), flush=True)
    for p in bad[:12]:
        print("  ", p, b.qlen[p], b.tlen[p], got.scores[p], got.cigar(p)[:40], want.cigar(p)[:40], flush=True)
