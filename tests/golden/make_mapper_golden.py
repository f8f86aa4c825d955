#!/usr/bin/env python3
"""Golden vectors for the mapper stages around team::Align.

Expected values come from oracle/_ref, built by oracle/Makefile from the
UNMODIFIED reference sources in /root/reference:
  * minimizers.json -- team::KMER::Minimize (team_minimizers.cpp, compiled in
    place) on the reference's own example sequences and seeded random ones;
  * *.paf           -- oracle/_ref/ref_mapper (reference Minimize + Align with
    the restated team_mapper.cpp glue, oracle/ref_mapper.cpp) on the committed
    synthetic inputs *.fasta / *.fastq below.
Run in the build container:  make -C oracle && python tests/golden/make_mapper_golden.py
"""
from __future__ import annotations

import json
import os
import random
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from bioinfo1_amd import synth  # noqa: E402
from oracle.pymapper import REF_MAPPER_BIN, RefMapper  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mapper")
REF_DIR = "/root/reference"

# (name, options) for every PAF fixture; inputs named <genome>.fasta / <reads>.{fasta,fastq}
RUNS = [
    ("g60k", "r60k.fasta", ["-a", "semiGlobal", "-c"]),
    ("g60k", "r60k.fastq", ["-a", "semiGlobal", "-c"]),
    ("g60k", "r60k.fasta", ["-a", "local", "-c"]),
    ("g60k", "r60k.fasta", ["-a", "global"]),
    ("g60k", "r60k.fasta", ["-a", "semiGlobal", "-c", "-k", "10", "-w", "8", "-f", "0.01"]),
    ("grep", "rrep.fasta", ["-a", "semiGlobal", "-c", "-f", "0.005"]),
    ("grep", "rrep.fastq", ["-a", "local", "-c", "-k", "12", "-w", "3", "-m", "2", "-n", "-3", "-g", "-2"]),
    ("demo", "demo_reads.fasta", ["-c", "-k", "3", "-w", "2"]),
    ("demo", "demo_reads.fasta", ["-a", "local", "-c", "-k", "4", "-w", "3"]),
    # pptx slide 16/17: the reference's published mapper run on its 9-bp ref.fasta
    ("demo_ref9", "demo_reads.fasta", ["-a", "local", "-m", "2", "-n", "-1", "-g", "2", "-k", "3", "-w", "2", "-c"]),
]
# the PAF lines the reference's slides publish for the last run (team_mapper.cpp:685-698)
SLIDE17_LINES = [b"seq1\t6\t1\t6\t-\tref\t9\t0\t5\t18\t5\t60\tcg:Z:1M4D4I",
                 b"seq2\t7\t0\t5\t+\tref\t9\t3\t8\t18\t5\t60\tcg:Z:1M4D4I"]


def write_fasta(path, recs, width=70):
    with open(path, "w") as f:
        for name, seq in recs:
            f.write(f">{name} synthetic\n")
            s = seq.decode()
            for i in range(0, len(s), width):
                f.write(s[i:i + width] + "\n")


def write_fastq(path, recs):
    with open(path, "w") as f:
        for name, seq in recs:
            f.write(f"@{name}\n{seq.decode()}\n+\n{'I' * len(seq)}\n")


def repeat_genome(seed):
    """60 kb with repeated blocks (multi-hit seeds, tied minimizer counts)."""
    rng = np.random.default_rng(seed)
    blocks = [synth.genome(3000, seed + i) for i in range(6)]
    order = [0, 1, 2, 1, 3, 4, 1, 5, 2, 0, 3, 5, 4, 2, 1, 0, 5, 3, 4, 1]
    g = np.concatenate([blocks[i] for i in order])
    mut = rng.random(g.shape[0]) < 0.02
    g[mut] = synth.ACGT[rng.integers(0, 4, int(mut.sum()))]
    return g


def reads_of(g, n, seed, median, lo, hi):
    rs = synth.ont_reads(n, g, seed, median=median, min_len=lo, max_len=hi)
    return [(f"read{r}", rs.read(r)) for r in range(rs.n_reads)]


def minimizer_cases(ref):
    cases = []
    ex = []
    for fn in ("primjer_minimizeri.txt", "dokumentacija_primjer.fasta.txt", "reference.fasta", "seq.fasta.txt",
               "ref.fasta"):
        p = os.path.join(REF_DIR, fn)
        if os.path.exists(p):
            name = None
            for line in open(p, "rb").read().splitlines():
                line = line.strip()
                if line.startswith(b">"):
                    name = line[1:].decode()
                elif line:
                    ex.append((f"{fn}:{name}", line))
    for src, s in ex:
        for k, w in ((3, 2), (3, 4), (5, 3), (2, 1), (4, 5)):
            if len(s) >= k and len(s) < w + k - 2:
                continue  # the reference reads past the end of the string there
            cases.append((src, s, k, w))
    rng = random.Random(20251016)
    for i in range(120):
        alpha = [b"ACGT", b"AC", b"ACGTN", b"acgtACGT", b"GGGT"][i % 5]
        L = rng.randint(0, 400)
        s = bytes(rng.choice(alpha) for _ in range(L))
        k, w = rng.randint(1, 15), rng.randint(1, 12)
        if L >= k and L < w + k - 2:
            continue
        cases.append((f"random #{i}", s, k, w))
    out = []
    for src, s, k, w in cases:
        for fwd in (True, False):
            m, u = ref.minimize(s, k, w, fwd)
            out.append({"source": src, "seq": s.decode("latin1"), "k": k, "w": w, "is_fwd": fwd,
                        "hash": [x[0] for x in m], "pos": [x[1] for x in m], "strand": [int(x[2]) for x in m],
                        "n_unique": u})
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    ref = RefMapper()
    mc = minimizer_cases(ref)
    with open(os.path.join(OUT, "minimizers.json"), "w") as f:
        json.dump({"generated_by": "oracle/_ref/libref_mapper.so (reference team_minimizers.cpp)", "cases": mc}, f)
    print(f"minimizers.json: {len(mc)} cases")
    g = synth.genome(60000, 0x6E0)
    write_fasta(os.path.join(OUT, "g60k.fasta"), [("chr_syn60k", g.tobytes())])
    rd = reads_of(g, 48, 0x0E7A, 1500, 300, 4000)
    write_fasta(os.path.join(OUT, "r60k.fasta"), rd)
    write_fastq(os.path.join(OUT, "r60k.fastq"), rd)
    gr = repeat_genome(0x5EB)
    write_fasta(os.path.join(OUT, "grep.fasta"), [("chr_rep", gr.tobytes())])
    rr = reads_of(gr, 40, 0x0E7B, 1200, 200, 3000)
    write_fasta(os.path.join(OUT, "rrep.fasta"), rr)
    write_fastq(os.path.join(OUT, "rrep.fastq"), rr)
    # the reference's own mapper demo inputs (copied as data)
    for src, dst in (("reference.fasta", "demo.fasta"), ("seq.fasta.txt", "demo_reads.fasta"),
                     ("ref.fasta", "demo_ref9.fasta")):
        with open(os.path.join(REF_DIR, src), "rb") as a, open(os.path.join(OUT, dst), "wb") as b:
            b.write(a.read())
    runs = []
    for i, (gname, rname, opts) in enumerate(RUNS):
        cmd = [REF_MAPPER_BIN] + opts + [os.path.join(OUT, gname + ".fasta"), os.path.join(OUT, rname)]
        res = subprocess.run(cmd, capture_output=True, check=True)
        paf = f"run{i}.paf"
        with open(os.path.join(OUT, paf), "wb") as f:
            f.write(res.stdout)
        runs.append({"genome": gname + ".fasta", "reads": rname, "args": opts, "paf": paf,
                     "lines": res.stdout.count(b"\n")})
        if gname == "demo_ref9":
            for line in SLIDE17_LINES:  # the reference build reproduces its own published lines
                assert line in res.stdout.splitlines(), (line, res.stdout)
            runs[-1]["published_lines"] = [x.decode() for x in SLIDE17_LINES]
        print(paf, gname, rname, " ".join(opts), res.stdout.count(b"\n"), "lines")
    with open(os.path.join(OUT, "runs.json"), "w") as f:
        json.dump({"generated_by": "oracle/_ref/ref_mapper (reference Minimize + Align, restated glue)",
                   "runs": runs}, f, indent=1)


if __name__ == "__main__":
    main()
