#!/usr/bin/env python3
"""Generate the committed golden vectors for the team::Align path.

Every expected value in tests/golden/ comes from the UNMODIFIED reference
team_alignment.cpp (/root/reference/team_alignment/), compiled in place by
oracle/Makefile into oracle/_ref/libref_align.so and called through
oracle/ref_harness.cpp.  Run in the build container (where /root/reference
exists):

    make -C oracle && python tests/golden/make_golden.py [--skip-digests]

Outputs (all data: inputs + expected outputs, no reference source):
  kat.json           doc/slide known-answer tests, the reference's example
                     FASTA files in every mode, and edge cases
  random_pairs.json  ~300 seeded random pairs over several alphabets and
                     scoring schemes, every mode
  digest_*.npz/.json full-batch digests for seeded synthetic batches
                     (bioinfo1_amd.synth): per-pair score, target_begin,
                     cigar length and CRC32, plus a SHA-256 over all CIGARs
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from bioinfo1_amd import synth  # noqa: E402
from oracle.pyoracle import AlignError, Reference  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
REF_DIR = "/root/reference"
MODES = {0: "global", 1: "local", 2: "semiGlobal"}


def read_fasta(path):
    recs, name, seq = [], None, []
    with open(path, "rb") as f:
        for line in f.read().splitlines():
            line = line.strip()
            if line.startswith(b">"):
                if name is not None:
                    recs.append((name, b"".join(seq)))
                name, seq = line[1:].decode(), []
            elif line:
                seq.append(line)
    if name is not None:
        recs.append((name, b"".join(seq)))
    return recs


def case(ref, q, t, typ, m, n, g, source, doc=None):
    rec = {"source": source, "query": q.hex(), "target": t.hex(), "type": typ, "match": m, "mismatch": n,
           "gap": g}
    try:
        s, cig, tb = ref.align(q, t, typ, m, n, g, True)
        s2, _, tb2 = ref.align(q, t, typ, m, n, g, False)
        assert (s, tb) == (s2, tb2), "score-only mode disagrees with cigar mode"
        rec.update(score=s, target_begin=tb, cigar=cig.hex(), error=None)
    except AlignError as e:
        rec.update(score=None, target_begin=None, cigar=None, error=str(e))
    if doc is not None:
        rec["doc_expect"] = doc
        assert rec["score"] == doc["score"] and bytes.fromhex(rec["cigar"]) == doc["cigar"].encode(), (rec, doc)
        if "target_begin" in doc:
            assert rec["target_begin"] == doc["target_begin"]
    return rec


def kat_cases(ref):
    cases = []
    # printed matrices / CIGARs in the pptx and the .doc report
    doc = [
        (b"TACGATG", b"ACGTACGAC", 0, 2, -2, -2, "pptx slide 6 (image13)", {"score": 0, "cigar": "3I5M1D1M"}),
        (b"TTACAC", b"ACGTACGAC", 1, 2, -2, -2, "pptx slide 8 (image16)",
         {"score": 8, "cigar": "3M1I2M", "target_begin": 10}),
        (b"TCGTAAGA", b"ACGTACGAC", 2, 2, -2, -2, "pptx slide 10 (image18)", {"score": 8, "cigar": "8M1I"}),
        (b"TACGA", b"TACGA", 1, 2, -1, 2, "pptx slide 17 mapper seq2 fwd", {"score": 18, "cigar": "1M4D4I"}),
        (b"TACGT", b"TACGT", 1, 2, -1, 2, "pptx slide 17 mapper seq1 rev", {"score": 18, "cigar": "1M4D4I"}),
        (b"GTACC", b"GATACGTTA", 0, 1, -1, -1, "BASELINE config 1", {"score": -1, "cigar": "1M1I3M3I1M",
                                                                      "target_begin": 0}),
    ]
    for q, t, typ, m, n, g, src, d in doc:
        cases.append(case(ref, q, t, typ, m, n, g, src, d))
    # the reference's example FASTA files, every mode, both orientations
    for fn in ["1_primjer_globalno_poravnanje.fasta.txt", "1_primjer_globalno_poravnanje2.fasta.txt",
               "2_primjer_poluGlobalno_poravnanje.fasta.txt", "3_primjer_lokalno_poravnanje.fasta.txt",
               "dokumentacija_primjer.fasta.txt"]:
        recs = read_fasta(os.path.join(REF_DIR, fn))
        a, b = recs[0][1], recs[1][1]
        for typ in (0, 1, 2):
            for (m, n, g) in [(1, -1, -1), (2, -2, -2), (2, -1, 2)]:
                cases.append(case(ref, a, b, typ, m, n, g, f"{fn} seq1/seq2"))
                cases.append(case(ref, b, a, typ, m, n, g, f"{fn} seq2/seq1"))
    # mapper demo data: every read against the 9-bp reference
    refseq = read_fasta(os.path.join(REF_DIR, "ref.fasta"))[0][1]
    for name, s in read_fasta(os.path.join(REF_DIR, "seq.fasta.txt")):
        for typ in (0, 1, 2):
            cases.append(case(ref, s, refseq, typ, 2, -1, 2, f"seq.fasta.txt {name} vs ref.fasta"))
            cases.append(case(ref, s, refseq, typ, 1, -1, -1, f"seq.fasta.txt {name} vs ref.fasta"))
    # edge cases
    edges = [
        (b"", b""), (b"", b"ACGT"), (b"ACGT", b""), (b"A", b"A"), (b"A", b"C"), (b"AAAA", b"CCCC"),
        (b"acgt", b"ACGT"), (b"NNNN", b"NNNN"), (b"A-C", b"AGC"), (b"AGC", b"A-C"), (b"----", b"ACGT"),
        (b"ACGT", b"----"), (b"--", b"--"), (b"GATTACA", b"GATTACA"), (b"G", b"GATTACA"), (b"GATTACA", b"G"),
        (b"\x00\xff\x7f", b"\x00\x80\x7f"),
    ]
    for q, t in edges:
        for typ in (0, 1, 2):
            for (m, n, g) in [(1, -1, -1), (2, -1, 2), (0, 0, 0), (-1, 1, -1), (3, -2, 0)]:
                cases.append(case(ref, q, t, typ, m, n, g, "edge"))
    for bad in (3, -1, 7):
        cases.append(case(ref, b"ACGT", b"ACGT", bad, 1, -1, -1, "edge: bad AlignmentType"))
    return cases


def random_cases(ref):
    rng = np.random.default_rng(0x5EED)
    alphabets = [b"ACGT", b"ACGTN", b"ACGTacgt", b"AC-GT", b"AC"]
    schemes = [(1, -1, -1), (2, -2, -2), (2, -1, 2), (3, -2, -5), (5, -4, -1), (1, 1, -1), (-1, -2, -3),
               (0, 0, 0), (100000, -70000, -90000)]
    cases = []
    for k in range(300):
        big = k % 25 == 0
        hi = 1200 if big else 160
        n = int(rng.integers(0, hi + 1))
        m = int(rng.integers(0, hi + 1))
        alpha = alphabets[k % len(alphabets)]
        q = bytes(rng.choice(np.frombuffer(alpha, np.uint8), n)) if n else b""
        if k % 3 == 0 and n:  # related target
            t = bytearray()
            for c in q:
                u = rng.random()
                if u < 0.08:
                    t.append(int(rng.choice(np.frombuffer(alpha, np.uint8))))
                elif u < 0.14:
                    t.append(int(rng.choice(np.frombuffer(alpha, np.uint8))))
                    t.append(c)
                elif u < 0.2:
                    pass
                else:
                    t.append(c)
            t = bytes(t[:m]) if m else b""
        else:
            t = bytes(rng.choice(np.frombuffer(alpha, np.uint8), m)) if m else b""
        typ = k % 3
        sm = schemes[(k // 3) % len(schemes)]
        cases.append(case(ref, q, t, typ, *sm, f"random #{k}"))
    return cases


def cigar_digest(res, P):
    h = hashlib.sha256()
    crc = np.zeros(P, np.uint32)
    for p in range(P):
        c = res.cigar(p)
        h.update(len(c).to_bytes(4, "little"))
        h.update(c)
        crc[p] = zlib.crc32(c)
    return h.hexdigest(), crc


def make_digest(ref, name, batch, typ, m, n, g, desc, indices=None):
    t0 = time.time()
    res = ref.align_batch(batch, typ, m, n, g, True)
    dt = time.time() - t0
    assert not res.status.any()
    sha, crc = cigar_digest(res, batch.n_pairs)
    extra = {} if indices is None else {"indices": np.asarray(indices, np.int64)}
    np.savez_compressed(os.path.join(OUT, f"digest_{name}.npz"), scores=res.scores, target_begins=res.target_begins,
                        cigar_lens=res.cigar_lens, cigar_crc32=crc, **extra)
    meta = {"name": name, "desc": desc, "type": typ, "match": m, "mismatch": n, "gap": g,
            "n_pairs": batch.n_pairs, "cells": batch.cells, "cigar_sha256": sha,
            "score_sum": int(res.scores.astype(np.int64).sum()), "generated_by": "oracle/_ref (reference)",
            "cpu_seconds_8threads": round(dt, 2)}
    with open(os.path.join(OUT, f"digest_{name}.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"digest {name}: {batch.n_pairs} pairs, {dt:.1f}s, sha {sha[:16]}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-digests", action="store_true")
    ap.add_argument("--only", default="", help="comma-separated digest names: regenerate only these")
    a = ap.parse_args()
    ref = Reference()
    if a.only:
        for name in a.only.split(","):
            DIGEST_SPECS[name](ref)
        return
    kat = kat_cases(ref)
    with open(os.path.join(OUT, "kat.json"), "w") as f:
        json.dump({"generated_by": "oracle/_ref (reference team_alignment.cpp)", "cases": kat}, f, indent=0)
    print(f"kat.json: {len(kat)} cases")
    rnd = random_cases(ref)
    with open(os.path.join(OUT, "random_pairs.json"), "w") as f:
        json.dump({"generated_by": "oracle/_ref (reference team_alignment.cpp)", "cases": rnd}, f, indent=0)
    print(f"random_pairs.json: {len(rnd)} cases")
    if a.skip_digests:
        return
    seed = 0x5EED
    make_digest(ref, "cfg2_local", synth.uniform_batch(10000, 1000, 1000, seed), 1, 1, -1, -1,
                "BASELINE config 2: 10k uniform 1kx1k local 1/-1/-1, synth.uniform_batch(seed=0x5EED)")
    make_digest(ref, "cfg2_related_local", synth.related_batch(10000, 1000, 1000, seed), 1, 1, -1, -1,
                "config 2 related variant (5% sub/ins/del), synth.related_batch(seed=0x5EED)")
    make_digest(ref, "g1k_global", synth.related_batch(1000, 1000, 1000, 0xA11CE), 0, 1, -1, -1,
                "1000 related 1kx1k global, synth.related_batch(seed=0xA11CE)")
    make_digest(ref, "s1k_semi", synth.related_batch(1000, 1000, 1000, 0xB0B), 2, 1, -1, -1,
                "1000 related 1kx1k semiGlobal, synth.related_batch(seed=0xB0B)")
    make_digest(ref, "ragged_local", synth.ragged_batch(2000, 0, 3000, 0xC0FFEE), 1, 2, -3, -2,
                "2000 ragged 0..3000 local 2/-3/-2, synth.ragged_batch(seed=0xC0FFEE)")
    make_digest(ref, "ragged_semi", synth.ragged_batch(2000, 0, 3000, 0xD00D), 2, 1, -1, -1,
                "2000 ragged 0..3000 semiGlobal, synth.ragged_batch(seed=0xD00D)")
    make_digest(ref, "ragged_global", synth.ragged_batch(2000, 0, 3000, 0xF00D), 0, 1, -1, -1,
                "2000 ragged 0..3000 global, synth.ragged_batch(seed=0xF00D)")
    make_digest(ref, "cfg5_semi_sample", synth.related_batch(32, 10000, 10000, 0x5EED), 2, 1, -1, -1,
                "config 5 linear-gap sample: 32 related 10kx10k semiGlobal, synth.related_batch(seed=0x5EED)")
    for spec in DIGEST_SPECS.values():
        spec(ref)


def _cfg3_sample(ref):
    b, _, _ = synth.cfg3_batch(64)
    make_digest(ref, "cfg3_semi_sample", b, 2, 1, -1, -1,
                "config 3 stand-in sample: first 64 ONT-like reads (1-20 kb, 10% error, 50% reverse) of "
                "synth.cfg3_batch() vs their true-origin windows, semiGlobal 1/-1/-1")


def _cfg3_local_sample(ref):
    b, _, _ = synth.cfg3_batch(64)
    make_digest(ref, "cfg3_local_sample", b, 1, 1, -1, -1,
                "config 3 stand-in sample, local: first 64 ONT-like reads (1-20 kb, 10% error, 50% reverse) of "
                "synth.cfg3_batch() vs their true-origin windows, local 1/-1/-1")


def _cfg5_strided(ref):
    idx = synth.CFG5_STRIDED
    make_digest(ref, "cfg5_semi_strided", synth.related_pairs_at(idx, 10000, 10000, 0x5EED), 2, 1, -1, -1,
                "config 5 (linear gap) stratified sample: the 128 related 10kx10k pairs at stream positions "
                "781*k (k = 0..127) of the 100,000-pair stream, semiGlobal 1/-1/-1", indices=idx)


def _cfg3_strided(ref, mode, name):
    idx = synth.CFG3_STRIDED
    b, _, _ = synth.cfg3_batch(indices=idx)
    make_digest(ref, name, b, mode, 1, -1, -1,
                f"config 3 stand-in stratified sample: the 256 ONT-like reads at positions 39*k (k = 0..255) of the "
                f"10,000-read set vs their true-origin windows, {MODES[mode]} 1/-1/-1", indices=idx)


# digests added after the first set (regenerate one with --only NAME)
DIGEST_SPECS = {"cfg3_semi_sample": _cfg3_sample, "cfg3_local_sample": _cfg3_local_sample,
                "cfg5_semi_strided": _cfg5_strided,
                "cfg3_semi_strided": lambda ref: _cfg3_strided(ref, 2, "cfg3_semi_strided"),
                "cfg3_local_strided": lambda ref: _cfg3_strided(ref, 1, "cfg3_local_strided")}


if __name__ == "__main__":
    main()
