"""GPU parity of the mapper stages against the reference's
outputs: minimizers (gfx950 kernel) vs the reference Minimize fixtures and
the restatement; FindLIS chains (gfx950 kernel) vs the restated FindLIS; and
the whole mapper CLI (team_mapper_amd) byte-for-byte against the PAF lines
of oracle/_ref/ref_mapper on the committed inputs."""
import json
import os
import random

import numpy as np
import pytest
from conftest import GOLDEN

from bioinfo1_amd import mapper as M
from bioinfo1_amd import synth
from oracle import pymapper as pm

pytestmark = pytest.mark.gpu
MG = os.path.join(GOLDEN, "mapper")


@pytest.fixture(scope="module")
def mp():
    return M.Mapper(0)


def test_minimizers_vs_reference_fixtures(mp):
    with open(os.path.join(MG, "minimizers.json")) as f:
        cases = [c for c in json.load(f)["cases"] if c["is_fwd"]]
    seqs = [c["seq"].encode("latin1") for c in cases]
    by_kw = {}
    for i, c in enumerate(cases):
        by_kw.setdefault((c["k"], c["w"]), []).append(i)
    n = 0
    for (k, w), idx in by_kw.items():
        full = mp.minimize_batch([seqs[i] for i in idx], k, w, dedup=False)
        ded = mp.minimize_batch([seqs[i] for i in idx], k, w, dedup=True)
        for j, i in enumerate(idx):
            c = cases[i]
            assert full[j][0].tolist() == c["hash"] and full[j][1].tolist() == c["pos"], (c["source"], k, w)
            fo = pm.first_occurrences(list(zip(c["hash"], c["pos"])))
            assert list(zip(ded[j][0].tolist(), ded[j][1].tolist())) == fo, (c["source"], k, w)
            n += 1
    assert n > 150


@pytest.mark.parametrize("k,w", [(15, 5), (10, 8), (3, 2), (5, 1), (12, 20), (1, 64)])
def test_minimizers_long_and_ragged(mp, k, w):
    rng = random.Random(k * 100 + w)
    seqs = []
    for i in range(24):
        L = rng.choice([0, 1, k - 1, k, k + w, 1023, 1024 + k, 2500, rng.randint(0, 4000)])
        alpha = [b"ACGT", b"AC", b"ACGTN", b"GGGGT"][i % 4]
        if L >= k and L < w + k - 2:
            L = w + k - 2  # keep clear of the reference's read-past-the-end case
        seqs.append(bytes(rng.choice(alpha) for _ in range(max(L, 0))))
    full = mp.minimize_batch(seqs, k, w, dedup=False)
    ded = mp.minimize_batch(seqs, k, w, dedup=True)
    for s, (h, p), (dh, dp) in zip(seqs, full, ded):
        want = pm.minimize(s, k, w, True)
        assert list(zip(h.tolist(), p.tolist(), [True] * len(h))) == want, (len(s), k, w)
        assert list(zip(dh.tolist(), dp.tolist())) == [(a, b) for a, b, _ in pm.first_occurrences(want)]


def _oracle_lis():
    return pm.RefMapper().find_lis if pm.RefMapper.available() else pm.find_lis


def _summary(chain):
    return (len(chain), chain[0] if chain else (0, 0), chain[-1] if chain else (0, 0))


def test_chain_vs_findlis(mp):
    rng = random.Random(99)
    lists = []
    for t in range(160):
        n = rng.choice([0, 1, 2, 5, 50, 300, rng.randint(0, 900)])
        span = rng.choice([3000, 20000, 200000])
        hits = [(rng.randint(1, span), rng.randint(1, span)) for _ in range(n)]
        if t % 3:
            hits.sort(key=lambda h: h[0])
            if t % 3 == 2 and hits:  # unsorted tail, like trailing end-minimizers
                hits += [(rng.randint(1, span), rng.randint(1, span)) for _ in range(4)]
        if t % 7 == 0:  # a colinear chain with noise and repeated positions
            hits = sorted(hits + [(10 * i + 1, 7 * i + 100) for i in range(n)] + [(10 * i + 1, 7 * i + 101) for i in
                                                                                   range(n // 3)])
        lists.append(hits)
    got = mp.chain_batch(lists)
    lis = _oracle_lis()
    for i, hits in enumerate(lists):
        assert got[i] == _summary(lis(hits)), (i, len(hits))


def test_chain_long_lists_global_path(mp):
    # 3072 < n <= 12288: the large-LDS instantiation; > 12288: global scratch
    rng = random.Random(5)
    lists = [[(i + 1, i + 1) for i in range(3072)]]
    for n in (3073, 5000, 12289):
        f = sorted(rng.randint(1, 40000) for _ in range(n))
        lists.append([(x, x + rng.randint(-30, 30) + 1000) for x in f])
    got = mp.chain_batch(lists)
    lis = _oracle_lis()
    for i, hits in enumerate(lists):
        assert got[i] == _summary(lis(hits))


def _runs():
    with open(os.path.join(MG, "runs.json")) as f:
        return json.load(f)["runs"]


@pytest.mark.parametrize("run", range(10))
def test_mapper_cli_matches_reference_paf(run):
    r = _runs()[run]
    for line in r.get("published_lines", []):  # run9: the reference's own slide-17 lines, literally
        assert line.encode() in open(os.path.join(MG, r["paf"]), "rb").read().splitlines()
    res = M.run_cli(r["args"] + [os.path.join(MG, r["genome"]), os.path.join(MG, r["reads"])], timeout=120)
    assert res.returncode == 0, res.stderr.decode()
    want = open(os.path.join(MG, r["paf"]), "rb").read()
    got = res.stdout
    if got != want:
        gl, wl = got.splitlines(), want.splitlines()
        diff = [(a[:160], b[:160]) for a, b in zip(gl, wl) if a != b][:3]
        raise AssertionError(f"{r['paf']}: {len(gl)} vs {len(wl)} lines; first diffs {diff}")


def test_mapper_slide17_published_lines():
    """pptx slide 16/17: `-a local -m 2 -n -1 -g 2 -k 3 -w 2 -c ref.fasta seq.fasta.txt`
    prints these two lines (team_mapper.cpp:685-698); team_mapper_amd prints them too."""
    r = [x for x in _runs() if x["genome"] == "demo_ref9.fasta"][0]
    res = M.run_cli(r["args"] + [os.path.join(MG, r["genome"]), os.path.join(MG, r["reads"])], timeout=120)
    assert res.returncode == 0, res.stderr.decode()
    got = res.stdout.splitlines()
    assert b"seq1\t6\t1\t6\t-\tref\t9\t0\t5\t18\t5\t60\tcg:Z:1M4D4I" in got
    assert b"seq2\t7\t0\t5\t+\tref\t9\t3\t8\t18\t5\t60\tcg:Z:1M4D4I" in got


def test_map_batch_api_matches_cli(mp):
    """The batched API (Index + map_batch) agrees with the CLI run on FASTQ rules."""
    r = _runs()[1]
    g = open(os.path.join(MG, r["genome"]), "rb").read().split(b"\n", 1)[1].replace(b"\n", b"")
    lines = open(os.path.join(MG, r["reads"]), "rb").read().split(b"\n")
    reads = [lines[i + 1] for i in range(0, len(lines) - 1, 4)]
    idx = M.Index(mp, "chr_syn60k", g, 15, 5, 0.001)
    st = idx.stats()
    assert st["banned_fwd"] == st["banned_rev"] > 0
    res = idx.map_batch(reads, M.Options.make(type=2, want_cigar=True, fastq_rules=True))
    paf = open(os.path.join(MG, r["paf"]), "rb").read().splitlines()
    assert int(res.mapped.sum()) == len(paf)
    j = 0
    for i in range(len(reads)):
        if not res.mapped[i]:
            continue
        cols = paf[j].split(b"\t")
        j += 1
        assert int(cols[2]) == res.q_begin[i] and int(cols[3]) == res.q_end[i] + 1
        assert int(cols[9]) == res.scores[i]
        assert cols[12] == b"cg:Z:" + res.cigar(i)
