"""The CPU restatement of the mapper stages (oracle/pymapper.py) is pinned to
the reference: minimizers.json was produced by the reference's own
team::KMER::Minimize (compiled from /root/reference into oracle/_ref by
oracle/Makefile, tests/golden/make_mapper_golden.py); where oracle/_ref is
built, fresh random sequences and hit lists are compared too."""
import json
import os
import random

import pytest
from conftest import GOLDEN

from oracle import pymapper as pm

MG = os.path.join(GOLDEN, "mapper")


def minimizer_cases():
    with open(os.path.join(MG, "minimizers.json")) as f:
        return json.load(f)["cases"]


def test_minimize_matches_reference_fixtures():
    cases = minimizer_cases()
    assert len(cases) > 300
    for c in cases:
        s = c["seq"].encode("latin1")
        got = pm.minimize(s, c["k"], c["w"], c["is_fwd"])
        want = list(zip(c["hash"], c["pos"], [bool(x) for x in c["strand"]]))
        assert got == want, (c["source"], c["k"], c["w"])
        assert len(set(want)) == c["n_unique"]


def test_mapper_fixtures_present():
    with open(os.path.join(MG, "runs.json")) as f:
        runs = json.load(f)["runs"]
    assert len(runs) >= 9
    for r in runs:
        assert os.path.exists(os.path.join(MG, r["paf"]))
        assert open(os.path.join(MG, r["paf"]), "rb").read().count(b"\n") == r["lines"]


def test_slide17_published_paf_fixture():
    """run9 is the reference's published mapper run (pptx slide 16/17,
    `-a local -m 2 -n -1 -g 2 -k 3 -w 2 -c ref.fasta seq.fasta.txt`): its PAF
    fixture holds the two published lines literally."""
    with open(os.path.join(MG, "runs.json")) as f:
        r = [x for x in json.load(f)["runs"] if x["genome"] == "demo_ref9.fasta"][0]
    assert r["args"] == ["-a", "local", "-m", "2", "-n", "-1", "-g", "2", "-k", "3", "-w", "2", "-c"]
    lines = open(os.path.join(MG, r["paf"]), "rb").read().splitlines()
    assert b"seq1\t6\t1\t6\t-\tref\t9\t0\t5\t18\t5\t60\tcg:Z:1M4D4I" in lines
    assert b"seq2\t7\t0\t5\t+\tref\t9\t3\t8\t18\t5\t60\tcg:Z:1M4D4I" in lines
    if pm.RefMapper.available():  # the reference build (oracle/_ref/ref_mapper) reproduces the fixture
        import subprocess

        res = subprocess.run([pm.REF_MAPPER_BIN] + r["args"] + [os.path.join(MG, r["genome"]),
                                                                os.path.join(MG, r["reads"])],
                             capture_output=True, check=True, timeout=60)
        assert res.stdout.splitlines() == lines


@pytest.mark.skipif(not pm.RefMapper.available(), reason="oracle/_ref not built (reference sources absent)")
def test_restatement_vs_reference_fuzz():
    ref = pm.RefMapper()
    rng = random.Random(77)
    for t in range(300):
        L = rng.randint(0, 80)
        alpha = rng.choice([b"ACGT", b"AC", b"ACGTN", b"acgtACGT", b"G"])
        s = bytes(rng.choice(alpha) for _ in range(L))
        k, w = rng.randint(1, 16), rng.randint(1, 9)
        if L >= k and L < w + k - 2:
            continue  # the reference reads past the end of its string there (UB)
        for fwd in (True, False):
            m, u = ref.minimize(s, k, w, fwd)
            assert pm.minimize(s, k, w, fwd) == m, (s, k, w)
            assert len(set(m)) == u
    for t in range(200):
        n = rng.randint(0, 60)
        hits = [(rng.randint(1, 12000), rng.randint(1, 12000)) for _ in range(n)]
        if t % 2:
            hits.sort(key=lambda h: h[0])
        assert pm.find_lis(hits) == ref.find_lis(hits)
