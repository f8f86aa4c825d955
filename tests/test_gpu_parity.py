"""GPU parity: the gfx950 kernels (through the C-ABI) against the committed
golden vectors (made by the reference itself) and against the CPU oracle on
seeded batches.  Bit-exact: scores, target_begin and CIGAR bytes."""
import os
import subprocess

import numpy as np
import pytest
from conftest import DIGESTS, ROOT, STRIDED, cigar_digest, digest_batch, load_digest, run_plan

from bioinfo1_amd import synth
from bioinfo1_amd.align import (TA_PLAN_CK, TA_PLAN_INT32_ONLY, TA_PLAN_NO_BLK, TA_PLAN_NO_CK, TA_PLAN_NO_FLEX, TA_PLAN_SERIAL_PASSES, TA_PLAN_UNFUSED, TA_PLAN_WALK1, TA_PLAN_WALK2, Aligner, DevicePlan,
                                align)
from oracle.pyoracle import Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def aligner():
    return Aligner(0)


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


def _run_cases(aligner, cases):
    groups = {}
    for c in cases:
        groups.setdefault((c["type"], c["match"], c["mismatch"], c["gap"]), []).append(c)
    n = 0
    for (typ, m, mm, g), cs in groups.items():
        if cs[0]["error"]:
            for c in cs:
                with pytest.raises(ValueError, match=r"Unknown AlignmentType provided\."):
                    align(bytes.fromhex(c["query"]), bytes.fromhex(c["target"]), typ, m, mm, g)
            continue
        b = synth.from_pairs([(bytes.fromhex(c["query"]), bytes.fromhex(c["target"])) for c in cs])
        r = aligner.align_batch(b, typ, m, mm, g, True)
        r0 = aligner.align_batch(b, typ, m, mm, g, False)
        for k, c in enumerate(cs):
            got = (int(r.scores[k]), r.cigar(k), int(r.target_begins[k]))
            assert got == (c["score"], bytes.fromhex(c["cigar"]), c["target_begin"]), (c["source"], c, got)
            assert (int(r0.scores[k]), int(r0.target_begins[k])) == (c["score"], c["target_begin"])
            n += 1
    return n


def test_kat(aligner, kat_cases):
    assert _run_cases(aligner, kat_cases) > 300


def test_random_pairs(aligner, random_cases):
    assert _run_cases(aligner, random_cases) == 300


def test_config1_single_call():
    # BASELINE config 1 through the single-pair mirror of team::Align
    assert align(b"GTACC", b"GATACGTTA", 0, 1, -1, -1) == (-1, b"1M1I3M3I1M", 0)


@pytest.mark.parametrize("name", DIGESTS + STRIDED)
def test_digest(aligner, name):
    meta, d = load_digest(name)
    batch = digest_batch(name)
    r = aligner.align_batch(batch, meta["type"], meta["match"], meta["mismatch"], meta["gap"], True)
    np.testing.assert_array_equal(r.scores, d["scores"])
    np.testing.assert_array_equal(r.target_begins, d["target_begins"])
    np.testing.assert_array_equal(r.cigar_lens, d["cigar_lens"])
    sha, crc = cigar_digest(r, batch.n_pairs)
    np.testing.assert_array_equal(crc, d["cigar_crc32"])
    assert sha == meta["cigar_sha256"]
    r0 = aligner.align_batch(batch, meta["type"], meta["match"], meta["mismatch"], meta["gap"], False)
    np.testing.assert_array_equal(r0.scores, d["scores"])
    np.testing.assert_array_equal(r0.target_begins, d["target_begins"])


@pytest.mark.parametrize("name", ["cfg2_local", "cfg2_related_local"])
def test_digest_walk_kinds(aligner, name):
    """The full config-2 digests (10,000 pairs: the default plan takes
    checkpoints and recomputing walks, test_digest) through the other walks of
    the same plans too: blocked codes and band walks, the [step][lane] layout
    and lane walks."""
    meta, d = load_digest(name)
    batch = digest_batch(name)
    plan = DevicePlan(aligner, batch, meta["type"], meta["match"], meta["mismatch"], meta["gap"], True)
    assert plan.ck, "config 2 plans take checkpoints by default"
    plan.close()
    for flags in (TA_PLAN_NO_CK, TA_PLAN_NO_BLK):
        r = run_plan(aligner, batch, meta["type"], (meta["match"], meta["mismatch"], meta["gap"]), True, flags)
        np.testing.assert_array_equal(r.scores, d["scores"])
        np.testing.assert_array_equal(r.cigar_lens, d["cigar_lens"])
        sha, crc = cigar_digest(r, batch.n_pairs)
        assert sha == meta["cigar_sha256"], flags


FUZZ = [
    # (mode, scoring, alphabet, min_len, max_len, n_pairs)
    (0, (1, -1, -1), b"ACGT", 0, 80, 400),
    (1, (1, -1, -1), b"ACGT", 0, 80, 400),
    (2, (1, -1, -1), b"ACGT", 0, 80, 400),
    (0, (2, -1, 2), b"AC-GT", 0, 300, 200),
    (1, (2, -1, 2), b"AC-GT", 0, 300, 200),
    (2, (3, -2, 0), b"acgtN-", 0, 300, 200),
    (1, (5, 4, -1), b"AC", 900, 1200, 40),
    (2, (1, -1, -1), b"ACGT", 1000, 1100, 40),
    (0, (1, 2, -3), b"ACGT", 1020, 1030, 40),
    (1, (1, -1, -1), b"ACGT", 2040, 2060, 16),
    (2, (2, -3, -1), b"ACGT-", 2040, 2060, 16),
    (0, (1, -1, -1), b"ACGT", 3000, 3100, 8),
    (1, (100000, -70000, -90000), b"ACGT", 0, 1500, 60),  # unpacked (WIDE) local argmax
    (1, (40000, -1, -1), b"AC", 1500, 2100, 12),           # WIDE + multi-pass
]


@pytest.mark.parametrize("case", range(len(FUZZ)))
def test_oracle_fuzz(aligner, oracle, case):
    mode, sc, alpha, lo, hi, P = FUZZ[case]
    b = synth.ragged_batch(P, lo, hi, seed=0xF022 + case, alphabet=alpha)
    want = oracle.align_batch(b, mode, *sc, True)
    got = aligner.align_batch(b, mode, *sc, True)
    for p in range(P):
        assert (int(got.scores[p]), got.cigar(p), int(got.target_begins[p])) == (
            int(want.scores[p]), want.cigar(p), int(want.target_begins[p])), (case, p, b.qlen[p], b.tlen[p])


# Batches whose pairs repeat a few (n, m) shapes, so most of them couple into
# the packed two-pair int16 fill (ta_dual.hip): (mode, scoring, alphabet, shapes, n_pairs)
DUAL_FUZZ = [
    (0, (1, -1, -1), b"ACGT", [(1, 1), (1, 5), (7, 3), (16, 16), (17, 200), (64, 64), (100, 37)], 300),
    (1, (1, -1, -1), b"ACGT", [(1, 1), (1, 5), (7, 3), (16, 16), (17, 200), (64, 64), (100, 37)], 300),
    (2, (1, -1, -1), b"ACGT", [(1, 1), (1, 5), (7, 3), (16, 16), (17, 200), (64, 64), (100, 37)], 300),
    (0, (2, -1, 2), b"AC-GT", [(33, 90), (250, 250), (5, 300)], 120),
    (1, (2, -1, 2), b"AC-GT", [(33, 90), (250, 250), (5, 300)], 120),
    (2, (2, -1, 2), b"AC-GT", [(33, 90), (250, 250), (5, 300)], 120),
    (1, (5, -4, -3), b"acgtN-", [(300, 280), (31, 31)], 80),
    (2, (3, -2, 0), b"ACGT-", [(300, 280), (31, 31)], 80),
    (0, (1, -1, -1), b"ACGT", [(1024, 1024), (1025, 700), (1500, 1500), (2100, 900)], 24),
    (1, (1, -1, -1), b"ACGT", [(1024, 1024), (1025, 700), (1500, 1500), (1900, 1900)], 24),
    (2, (1, -1, -1), b"AC", [(1024, 1024), (1025, 700), (1500, 1500), (2100, 900)], 24),
    (1, (1, 2, -3), b"AC", [(1017, 333), (2049, 64)], 12),
    # multi-pass couples run one wave per (couple, pass); couples with '-' are handed back
    (2, (2, -1, 2), b"AC-GT", [(2100, 1200), (1500, 800)], 16),
    (0, (1, -1, -1), b"ACGTTTTTTTTTTTTTTTTTTTTTTTTTTTTTTTTT-", [(3100, 700), (1030, 1030)], 16),
]


def _shaped_batch(P, shapes, alphabet, seed):
    rng = np.random.default_rng(seed)
    al = np.frombuffer(alphabet, np.uint8)
    pairs = []
    for k in range(P):
        n, m = shapes[rng.integers(len(shapes))]
        pairs.append((al[rng.integers(len(al), size=n)].tobytes(), al[rng.integers(len(al), size=m)].tobytes()))
    return synth.from_pairs(pairs)


@pytest.mark.parametrize("case", range(len(DUAL_FUZZ)))
def test_dual_fuzz(aligner, oracle, case):
    mode, sc, alpha, shapes, P = DUAL_FUZZ[case]
    b = _shaped_batch(P, shapes, alpha, 0xD0A1 + case)
    plan = DevicePlan(aligner, b, mode, *sc, True)
    assert plan.dual_pairs >= P // 2, plan.dual_pairs
    plan.close()
    want = oracle.align_batch(b, mode, *sc, True)
    # packed kernels (default), the int32 kernel alone (fused / separate walk)
    for flags in (0, TA_PLAN_WALK1, TA_PLAN_WALK2, TA_PLAN_INT32_ONLY, TA_PLAN_INT32_ONLY | TA_PLAN_UNFUSED,
                  TA_PLAN_INT32_ONLY | TA_PLAN_SERIAL_PASSES):
        for cig in (True, False):
            got = run_plan(aligner, b, mode, sc, cig, flags)
            np.testing.assert_array_equal(got.scores, want.scores)
            np.testing.assert_array_equal(got.target_begins, want.target_begins)
            if cig:
                for p in range(P):
                    assert got.cigar(p) == want.cigar(p), (case, flags, p, b.qlen[p], b.tlen[p])


def test_related_long_pairs(aligner, oracle):
    # long tracebacks across pass and tile boundaries
    for mode in (0, 1, 2):
        b = synth.related_batch(6, 2500, 2600, seed=77 + mode)
        want = oracle.align_batch(b, mode, 1, -1, -1, True)
        got = aligner.align_batch(b, mode, 1, -1, -1, True)
        assert want.cigars() == got.cigars()
        np.testing.assert_array_equal(want.scores, got.scores)


def test_device_plan_and_chunking(aligner):
    import torch

    b = synth.uniform_batch(300, 1000, 1000, seed=11)
    host = aligner.align_batch(b, 1, 1, -1, -1, True)
    for budget in (0, 3 * 1063 * 256):  # default, and ~3 pairs per chunk
        plan = DevicePlan(aligner, b, 1, 1, -1, -1, True, workspace_budget=budget)
        # couples of equal-shape pairs share a wave (dual fill): 2 pairs per chunk then
        per_chunk = 2 if plan.dual_pairs == b.n_pairs else 3
        assert plan.chunks == (1 if budget == 0 else -(-b.n_pairs // per_chunk))
        plan.run()
        torch.cuda.synchronize()
        r = plan.results()
        np.testing.assert_array_equal(r.scores, host.scores)
        np.testing.assert_array_equal(r.target_begins, host.target_begins)
        assert r.cigars() == host.cigars()
        plan.close()


def _shim_binary():
    out = os.path.join(ROOT, "build", "shim_caller")
    libdir = os.path.join(ROOT, "bioinfo1_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-pthread", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "shim_caller.cpp"), "-L", libdir,
                           "-lteam_alignment", f"-Wl,-rpath,{libdir}", "-o", out])
    return out


def test_team_align_dropin(kat_cases, random_cases):
    """An unmodified team::Align caller links and gets the reference's
    answers (incl. the exception message), single- and multi-threaded."""
    exe = _shim_binary()
    cases = kat_cases + random_cases
    lines = [f"{c['type']} {c['match']} {c['mismatch']} {c['gap']} {c['query'] or '-'} {c['target'] or '-'}"
             for c in cases]
    want = []
    for c in cases:
        if c["error"]:
            want.append(f"ERR {c['error']}")
        else:
            want.append(f"{c['score']} {c['target_begin']} {c['cigar'] or '-'}")
    for mode in ([], ["threads"], ["threads", "16"]):  # combined batches of mixed scorings and errors
        out = subprocess.run([exe] + mode, input="\n".join(lines) + "\n", capture_output=True, text=True,
                             timeout=600, check=True).stdout.splitlines()
        assert out == want


def test_team_align_dropin_mixed_sizes(oracle):
    """16 caller threads mixing pairs the resident server takes with pairs
    past its limits (query > 4,096: the batch path).  A batch pauses the
    device's servers around its launches, so no batch kernel queues behind
    the persistent kernel on a shared hardware queue; every call finishes,
    bounded in time, with the oracle's answers (shim stream /
    queue sharing)."""
    import time

    exe = _shim_binary()
    small = synth.ragged_batch(96, 1, 400, seed=0x31)
    big = synth.related_batch(6, 4400, 600, seed=0x32)  # n > kSrvQMax: never served
    pairs = [(small.query(p), small.target(p)) for p in range(small.n_pairs)]
    at = [3 + 16 * k for k in range(big.n_pairs)]  # spread over the threads' strides
    for k, p in enumerate(at):
        pairs.insert(p, (big.query(k), big.target(k)))
    b = synth.from_pairs(pairs)
    want = oracle.align_batch(b, 1, 1, -1, -1, True)
    lines = [f"1 1 -1 -1 {q.hex() or '-'} {t.hex() or '-'}" for q, t in pairs]
    exp = [f"{int(want.scores[p])} {int(want.target_begins[p])} {want.cigar(p).hex() or '-'}"
           for p in range(b.n_pairs)]
    t0 = time.time()
    out = subprocess.run([exe, "threads", "16"], input="\n".join(lines) + "\n", capture_output=True, text=True,
                         timeout=120, check=True).stdout.splitlines()
    assert out == exp
    assert time.time() - t0 < 60


def _check_full(aligner, batch, mode, sc):
    from oracle.pyoracle import cigar_check_batch

    r = aligner.align_batch(batch, mode, *sc, True)
    st = cigar_check_batch(batch, mode, *sc, r.scores, r.target_begins, r.arena, r.cigar_offsets, r.cigar_lens)
    assert not st.any(), (np.nonzero(st)[0][:8], st[np.nonzero(st)[0][:8]])
    r0 = aligner.align_batch(batch, mode, *sc, False)
    np.testing.assert_array_equal(r0.scores, r.scores)
    np.testing.assert_array_equal(r0.target_begins, r.target_begins)
    return r


def _check_strided(r, name, lo=0):
    """Pairs of the stratified reference digest `name` inside a full-size run
    (pair p of the run = stream position lo + p): bit-exact score,
    target_begin, CIGAR length, CRC32 and, all of them present, the SHA-256."""
    import zlib

    meta, d = load_digest(name)
    idx = d["indices"] - lo
    np.testing.assert_array_equal(r.scores[idx], d["scores"])
    np.testing.assert_array_equal(r.target_begins[idx], d["target_begins"])
    np.testing.assert_array_equal(r.cigar_lens[idx], d["cigar_lens"])
    cig = [r.cigar(int(p)) for p in idx]
    assert [zlib.crc32(c) for c in cig] == [int(x) for x in d["cigar_crc32"]]
    sha, _ = cigar_digest(type("R", (), {"cigar": lambda self, k: cig[k]})(), len(cig))
    assert sha == meta["cigar_sha256"]


def test_config3_full_batch_properties(aligner):
    """BASELINE config 3 stand-in at full size (10k ONT-like reads, 1-20 kb,
    1.18e12 cells): every CIGAR is a full semi-global path whose score is the
    reported score, and score-only mode agrees.  The first 64 reads and 256
    reads spread over the whole set (every 39th) are bit-exact against the
    reference digests."""
    b, _, _ = synth.cfg3_batch(10000)
    r = _check_full(aligner, b, 2, (1, -1, -1))
    meta, d = load_digest("cfg3_semi_sample")
    np.testing.assert_array_equal(r.scores[:64], d["scores"])
    np.testing.assert_array_equal(r.cigar_lens[:64], d["cigar_lens"])
    _check_strided(r, "cfg3_semi_strided")


def test_config3_local_full_batch_properties(aligner):
    """The config 3 stand-in in local mode (the flexible packed fill's local
    path): every CIGAR is a local path scoring the reported score, score-only
    agrees, and the first 64 reads and 256 reads spread over the set are
    bit-exact against the reference digests."""
    b, _, _ = synth.cfg3_batch(10000)
    r = _check_full(aligner, b, 1, (1, -1, -1))
    meta, d = load_digest("cfg3_local_sample")
    np.testing.assert_array_equal(r.scores[:64], d["scores"])
    np.testing.assert_array_equal(r.target_begins[:64], d["target_begins"])
    np.testing.assert_array_equal(r.cigar_lens[:64], d["cigar_lens"])
    _check_strided(r, "cfg3_local_strided")


def test_config5_shape_properties(aligner):
    """Config 5 shape (10 kb x 10 kb semi-global, linear gap) on 512 pairs:
    path/score properties; the first 32 pairs bit-exact vs the reference digest."""
    b = synth.related_batch(512, 10000, 10000, 0x5EED)
    r = _check_full(aligner, b, 2, (1, -1, -1))
    meta, d = load_digest("cfg5_semi_sample")
    np.testing.assert_array_equal(r.scores[:32], d["scores"])
    np.testing.assert_array_equal(r.cigar_lens[:32], d["cigar_lens"])


def _flex_batch(P, lo, hi, alphabet, seed, tdash=False, qdash=False):
    """Ragged related pairs in groups that couple for the flexible dual fill
    (same query pass count and length mod 16, different target lengths)."""
    rng = np.random.default_rng(seed)
    al = np.frombuffer(alphabet, np.uint8)
    pairs = []
    while len(pairs) < P:
        n0 = int(rng.integers(lo, hi + 1))
        for _ in range(2):
            n = max(1, n0 - 16 * int(rng.integers(0, 4)))
            if (n - 1) // 1024 != (n0 - 1) // 1024:
                n = n0
            m = max(1, int(n0 * rng.uniform(0.8, 1.2)))
            q = al[rng.integers(len(al), size=n)]
            t = q[: min(n, m)].copy()
            flip = rng.random(t.shape[0]) < 0.1
            t[flip] = al[rng.integers(len(al), size=int(flip.sum()))]
            if m > t.shape[0]:
                t = np.concatenate([t, al[rng.integers(len(al), size=m - t.shape[0])]])
            if tdash and len(pairs) % 3 == 0:
                t[rng.integers(m, size=max(1, m // 50))] = ord("-")
            if qdash and len(pairs) % 5 == 0:
                q = q.copy()
                q[rng.integers(n, size=1)] = ord("-")
            pairs.append((q.tobytes(), t.tobytes()))
    return synth.from_pairs(pairs[:P])


FLEX_FUZZ = [
    # (mode, scoring, alphabet, lo, hi, n_pairs, tdash, qdash)
    (0, (1, -1, -1), b"ACGT", 1, 300, 120, False, False),
    (2, (1, -1, -1), b"ACGT", 1, 300, 120, False, False),
    (0, (2, -3, -2), b"ACGT", 900, 2200, 24, True, False),
    (2, (2, -3, -2), b"ACGT", 900, 2200, 24, True, True),
    (2, (3, -2, 0), b"ACGTN", 1000, 1100, 16, False, False),
    (0, (2, -1, 2), b"AC", 500, 1500, 20, False, False),
    (2, (1, -1, -1), b"ACGT", 10700, 12500, 6, False, False),   # beyond absolute int16: rebasing
    (0, (1, -1, -1), b"ACGT", 10700, 11200, 4, False, False),
    (2, (1, -1, -1), b"ACGT", 4100, 6000, 3, False, False),     # odd groups: long singles coupled with themselves
    (0, (2, -3, -2), b"ACGT", 4100, 6000, 5, True, True),
    # local mode (clamp, row-major first-max argmax, cost-tracking walk)
    (1, (1, -1, -1), b"ACGT", 1, 300, 120, False, False),
    (1, (2, -3, -2), b"ACGT", 900, 2200, 24, True, False),
    (1, (2, -3, -2), b"ACGT", 900, 2200, 24, True, True),      # '-' in queries: handed to the int32 fill
    (1, (3, -2, 0), b"ACGTN", 1000, 1100, 16, False, False),   # gap 0
    (1, (2, -1, 2), b"AC", 500, 1500, 20, False, False),       # positive gap
    (1, (1, -1, -1), b"ACGT", 10700, 12500, 6, False, False),  # long: rebasing, 11+ passes
    (1, (1, -1, -1), b"ACGT", 4100, 6000, 3, False, False),    # odd group: long singles coupled with themselves
    (1, (5, -4, -3), b"ACGT", 1000, 3000, 12, False, False),
]


@pytest.mark.parametrize("case", range(len(FLEX_FUZZ)))
def test_flex_fuzz(aligner, oracle, case):
    mode, sc, alpha, lo, hi, P, td, qd = FLEX_FUZZ[case]
    b = _flex_batch(P, lo, hi, alpha, 0xF1E0 + case, td, qd)
    plan = DevicePlan(aligner, b, mode, *sc, True)
    assert plan.flex_pairs >= P // 3, (plan.flex_pairs, plan.dual_pairs)
    plan.close()
    want = oracle.align_batch(b, mode, *sc, True)
    for flex in (0, TA_PLAN_NO_FLEX):
        for cig in (True, False):
            got = run_plan(aligner, b, mode, sc, cig, flex)
            np.testing.assert_array_equal(got.scores, want.scores)
            np.testing.assert_array_equal(got.target_begins, want.target_begins)
            if cig:
                for p in range(P):
                    assert got.cigar(p) == want.cigar(p), (case, flex, p, b.qlen[p], b.tlen[p])


def test_flex_records_ignore_stale_workspace():
    """Regression: on a fresh context, this digest sequence once left traceback
    codes in freed memory that the next ws_bnd allocation reused, and two
    stale dwords carried the flexible fill's small hand-off tags (epoch 3):
    ragged_global's first run read them as pass-0 records (2/2000 scores
    wrong).  The host now zeroes the record buffers before each flex launch."""
    al = Aligner(0)
    try:
        for name in ("cfg2_local", "cfg2_related_local", "g1k_global", "s1k_semi", "ragged_local", "ragged_semi"):
            meta, _ = load_digest(name)
            for cig in (True, False):
                al.align_batch(digest_batch(name), meta["type"], meta["match"], meta["mismatch"], meta["gap"], cig)
        meta, d = load_digest("ragged_global")
        batch = digest_batch("ragged_global")
        for cig in (True, False):
            r = al.align_batch(batch, meta["type"], meta["match"], meta["mismatch"], meta["gap"], cig)
            np.testing.assert_array_equal(r.scores, d["scores"])
            if cig:
                np.testing.assert_array_equal(r.cigar_lens, d["cigar_lens"])
    finally:
        al.close()


@pytest.mark.parametrize("sc", [(2, -1, 1), (1, -1, -1), (3, -2, 0), (1, 2, -3)])
def test_local_walk_cost_tracking(aligner, oracle, sc):
    """Packed local fill (raw codes, no STOP) + the cost-tracking walk: '-'
    only in targets (the couples stay packed), gap > 0 / = 0 / < 0, mismatch
    above match: every stop rule of the walk (closed-form gap runs, byte
    windows, prefix-sum stop inside a run) against the oracle."""
    rng = np.random.default_rng(0x10CA1 + sc[0] * 7 + sc[2])
    qa, ta = np.frombuffer(b"ACGT", np.uint8), np.frombuffer(b"ACGT-", np.uint8)
    shapes = [(300, 280), (64, 64), (1030, 900), (17, 130)]
    pairs = []
    for k in range(64):
        n, m = shapes[k % len(shapes)]
        pairs.append((qa[rng.integers(4, size=n)].tobytes(), ta[rng.integers(5, size=m)].tobytes()))
    b = synth.from_pairs(pairs)
    plan = DevicePlan(aligner, b, 1, *sc, True)
    # 1030 x 900 leaves int16 for gap > 0 or match 3 (fits_int16): those couples run int32
    assert plan.dual_pairs >= 48, plan.dual_pairs
    plan.close()
    want = oracle.align_batch(b, 1, *sc, True)
    got = aligner.align_batch(b, 1, *sc, True)
    np.testing.assert_array_equal(got.scores, want.scores)
    np.testing.assert_array_equal(got.target_begins, want.target_begins)
    for p in range(b.n_pairs):
        assert got.cigar(p) == want.cigar(p), (sc, p)


@pytest.mark.parametrize("sc", [(1, -1, -1), (2, -3, -1), (1, -2, -3)])
def test_local_group_walk_dual_and_fallback(aligner, oracle, sc):
    """Local plans of equal-shape couples only, walked two pairs per wave
    (ta_walk2.h); couples with a '-' query go to the int32 fill.  Against the
    oracle, with the one-pair walk too."""
    rng = np.random.default_rng(0xF05E + sc[0])
    al, ald = np.frombuffer(b"ACGT", np.uint8), np.frombuffer(b"ACGT-N", np.uint8)
    pairs = []
    for k in range(96):
        n, m = [(200, 180), (700, 650), (33, 900)][k % 3]
        qa = ald if k % 17 == 0 else al
        ta = ald if k % 5 == 0 else al
        pairs.append((qa[rng.integers(len(qa), size=n)].tobytes(), ta[rng.integers(len(ta), size=m)].tobytes()))
    b = synth.from_pairs(pairs)
    plan = DevicePlan(aligner, b, 1, *sc, True)
    assert plan.dual_pairs == 96 and not plan.fused, (plan.dual_pairs, plan.fused)
    plan.close()
    want = oracle.align_batch(b, 1, *sc, True)
    for flags in (0, TA_PLAN_WALK1, TA_PLAN_WALK2):
        got = run_plan(aligner, b, 1, sc, True, flags)
        np.testing.assert_array_equal(got.scores, want.scores)
        np.testing.assert_array_equal(got.target_begins, want.target_begins)
        for p in range(b.n_pairs):
            assert got.cigar(p) == want.cigar(p), (sc, flags, p)


# Band walks (ta_walk_band.h) over the blocked code layout: local plans of
# equal-shape couples only.  (scoring, query alphabet, target alphabet, shapes
# -- each taken an even number of times, so every pair couples --, walk kind)
BAND_CASES = [
    ((1, -1, -1), b"ACGT", b"ACGT", [(1000, 1000)] * 16, 64),           # config 2's shape
    ((1, -1, -1), b"ACGT", b"ACGT", [(1, 1), (5, 9), (16, 16), (17, 3), (64, 300), (15, 1), (1, 200), (300, 1)], 64),
    ((2, -3, -1), b"ACGTN", b"acgtN", [(1030, 900), (2100, 700), (1500, 600)], 64),  # across passes; N, lowercase
    ((3, 4, 0), b"ACGT", b"ACGT", [(300, 280), (64, 64)], 64),          # mismatch above match, free gaps
    ((5, -4, -3), b"AC", b"ACGT", [(257, 255), (300, 280)], 64),        # (16 x 5 x min(n, m) within int16)
    ((1, -1, -1), b"AC-GT", b"ACGT-", [(200, 180), (700, 650)], 64),     # '-': handed back, the fallback walk
    ((2, -1, 2), b"ACGT", b"ACGT", [(300, 280), (64, 64)], 0),           # gap > 0: one-pair walk, blocked layout
]


@pytest.mark.parametrize("case", range(len(BAND_CASES)))
def test_band_walk(aligner, oracle, case):
    sc, qa, ta, shapes, walk = BAND_CASES[case]
    rng = np.random.default_rng(0xBA4D + case)
    qa, ta = np.frombuffer(qa, np.uint8), np.frombuffer(ta, np.uint8)
    pairs = []
    for k in range(2 * len(shapes) * 4):
        n, m = shapes[(k // 2) % len(shapes)]
        pairs.append((qa[rng.integers(len(qa), size=n)].tobytes(), ta[rng.integers(len(ta), size=m)].tobytes()))
    if case == 0:  # plus related pairs: long match runs, long walks
        rb = synth.related_batch(32, 1000, 1000, seed=0xBA4E)
        pairs += [(rb.query(p), rb.target(p)) for p in range(rb.n_pairs)]
    b = synth.from_pairs(pairs)
    plan = DevicePlan(aligner, b, 1, *sc, True)
    assert not plan.blk and plan.walk == 16, (plan.blk, plan.walk, plan.ck)  # (small: codes and lane walks)
    plan.close()
    # TA_PLAN_NO_CK: blocked codes and band walks
    plan = DevicePlan(aligner, b, 1, *sc, True, flags=TA_PLAN_NO_CK)
    assert plan.blk and plan.walk == walk and not plan.ck, (plan.blk, plan.walk, plan.ck)
    plan.close()
    # TA_PLAN_CK: checkpoints + recomputing walks (ta_walk_ck.hip) when walked with gap <= 0
    # (gap > 0: no checkpoints, so the codes and lane walks)
    plan = DevicePlan(aligner, b, 1, *sc, True, flags=TA_PLAN_CK)
    if walk == 64:
        assert plan.blk and plan.walk == 64 and plan.ck, (plan.blk, plan.walk, plan.ck)
    else:
        assert not plan.blk and plan.walk == 16 and not plan.ck, (plan.blk, plan.walk, plan.ck)
    plan.close()
    want = oracle.align_batch(b, 1, *sc, True)
    for flags in (0, TA_PLAN_NO_CK, TA_PLAN_CK, TA_PLAN_NO_BLK):
        got = run_plan(aligner, b, 1, sc, True, flags)
        np.testing.assert_array_equal(got.scores, want.scores)
        np.testing.assert_array_equal(got.target_begins, want.target_begins)
        for p in range(b.n_pairs):
            assert got.cigar(p) == want.cigar(p), (case, flags, p, b.qlen[p], b.tlen[p])


CK_SCORES = [(1, -1, -1), (2, -3, -1), (1, -2, -3), (3, 4, 0), (5, -4, -3), (1, 0, -1), (4, -1, -2)]


@pytest.mark.parametrize("sc", CK_SCORES)
def test_ck_walk(aligner, oracle, sc):
    """Recomputing walks over checkpoints (ta_walk_ck.hip) against the oracle:
    an odd number of couples of each shape (a pair coupled with itself), one
    to three query passes, and paths with long I runs (more than a window of
    32 columns) and long D runs (across stripes and a pass edge) -- inserted
    blocks that match nothing -- beside random and related pairs."""
    rng = np.random.default_rng(0xC4EC + 7 * sc[0] - sc[1])
    al = np.frombuffer(b"ACGT", np.uint8)
    rnd = lambda k: al[rng.integers(4, size=k)].tobytes()  # noqa: E731
    pairs = []
    # shapes within the dual fill's int16 frame for these scores (ta_planner.cpp fits_int16)
    hs, mag = max(sc[0], sc[1], 1), max(abs(sc[0]), abs(sc[1]), abs(sc[2]), 1)
    mcap, scap = (28900 - 32 * mag) // (16 * sc[0] - 1), (31000 - 32 * mag) // (16 * hs)
    for n, m, cnt in ((300, 280, 9), (1030, 990, 5), (2100, 700, 3), (40, 1200, 3), (1500, 64, 3)):
        m = min(m, mcap)
        if min(n, m) > scap:
            m = scap
        for k in range(cnt):
            core = rnd(min(n, m) - 200 if min(n, m) > 400 else min(n, m) // 2)
            gapb = b"N" * (40 + 23 * k)
            if k % 3 == 0:  # an insertion in the target: an I run
                q, t = core, core[: len(core) // 2] + gapb + core[len(core) // 2:]
            elif k % 3 == 1:  # a deletion: a D run
                q, t = core[: len(core) // 3] + gapb + core[len(core) // 3:], core
            else:
                q, t = rnd(n), rnd(m)
            q, t = (q + rnd(max(0, n - len(q))))[:n], (t + rnd(max(0, m - len(t))))[:m]
            pairs.append((q, t))
    L = min(1000, mcap, scap)
    rb = synth.related_batch(9, L, L, seed=0xC4ED)
    pairs += [(rb.query(p), rb.target(p)) for p in range(rb.n_pairs)]
    b = synth.from_pairs(pairs)
    plan = DevicePlan(aligner, b, 1, *sc, True, flags=TA_PLAN_CK)
    assert plan.blk and plan.ck and plan.walk == 64, (plan.blk, plan.ck, plan.walk)
    plan.close()
    want = oracle.align_batch(b, 1, *sc, True)
    got = run_plan(aligner, b, 1, sc, True, TA_PLAN_CK)
    np.testing.assert_array_equal(got.scores, want.scores)
    np.testing.assert_array_equal(got.target_begins, want.target_begins)
    for p in range(b.n_pairs):
        assert got.cigar(p) == want.cigar(p), (sc, p, b.qlen[p], b.tlen[p])


@pytest.mark.parametrize("name", ["g1k_global", "s1k_semi", "cfg5_semi_sample"])
def test_digest_ck_edge(aligner, name):
    """Global and semi-global digests of the reference through checkpoint plans
    (TA_PLAN_CK: the dual fill stores checkpoints, the global / semi-global
    recomputing walk of ta_walk_ck.hip walks to row 0 / column 0): bit-exact."""
    meta, d = load_digest(name)
    batch = digest_batch(name)
    sc = (meta["match"], meta["mismatch"], meta["gap"])
    plan = DevicePlan(aligner, batch, meta["type"], *sc, True, flags=TA_PLAN_CK)
    assert plan.ck and plan.blk and plan.walk == 64, (plan.ck, plan.blk, plan.walk)
    plan.close()
    r = run_plan(aligner, batch, meta["type"], sc, True, TA_PLAN_CK)
    np.testing.assert_array_equal(r.scores, d["scores"])
    np.testing.assert_array_equal(r.target_begins, d["target_begins"])
    np.testing.assert_array_equal(r.cigar_lens, d["cigar_lens"])
    sha, crc = cigar_digest(r, batch.n_pairs)
    np.testing.assert_array_equal(crc, d["cigar_crc32"])
    assert sha == meta["cigar_sha256"]


@pytest.mark.parametrize("mode", [0, 2])
def test_ck_walk_edge_kats(aligner, kat_cases, random_cases, mode):
    """Every known-answer case and random pair of the reference in global /
    semi-global mode through checkpoint plans (TA_PLAN_CK; lone pairs run
    coupled with themselves): the worked examples, the semi trailing runs
    (5I1M1I2M2D, 7I1M8D), goals on row 0 / column 0, '-' bytes (handed back to
    the one-pair walk), lowercase and N."""
    groups = {}
    for c in kat_cases + random_cases:
        if c["type"] == mode and not c["error"] and c["query"] and c["target"]:
            groups.setdefault((c["match"], c["mismatch"], c["gap"]), []).append(c)
    ck = n = 0
    for sc, cs in groups.items():
        b = synth.from_pairs([(bytes.fromhex(c["query"]), bytes.fromhex(c["target"])) for c in cs])
        flags = TA_PLAN_CK | TA_PLAN_NO_FLEX  # (every pair a dual couple, coupled with itself)
        plan = DevicePlan(aligner, b, mode, *sc, True, flags=flags)
        ck += plan.ck
        plan.close()
        r = run_plan(aligner, b, mode, sc, True, flags)
        for k, c in enumerate(cs):
            got = (int(r.scores[k]), r.cigar(k), int(r.target_begins[k]))
            assert got == (c["score"], bytes.fromhex(c["cigar"]), c["target_begin"]), (c["source"], c, got)
            n += 1
    assert ck >= 3 and n > 50, (ck, n)


@pytest.mark.parametrize("mode,sc", [(m, s) for m in (0, 2) for s in ((1, -1, -1), (2, -3, -1), (3, 4, 0), (2, -1, 2))])
def test_ck_walk_edge(aligner, oracle, mode, sc):
    """Global / semi-global recomputing walks over checkpoints against the
    oracle: odd numbers of couples per shape (self-coupled pairs), one to three
    query passes, long I runs and D runs (inserted blocks that match nothing)
    that cross windows, stripes and a pass edge, semi goals in the last row and
    the last column, and related pairs."""
    rng = np.random.default_rng(0xED6E + 11 * mode + 7 * sc[0] - sc[1])
    al = np.frombuffer(b"ACGT", np.uint8)
    rnd = lambda k: al[rng.integers(4, size=k)].tobytes()  # noqa: E731
    pairs = []
    for n, m, cnt in ((300, 280, 9), (1030, 990, 5), (2100, 700, 3), (40, 600, 3), (700, 64, 3)):
        for k in range(cnt):
            core = rnd(min(n, m) - 100 if min(n, m) > 200 else min(n, m) // 2)
            gapb = b"N" * (40 + 23 * k)
            if k % 3 == 0:  # an insertion in the target: an I run
                q, t = core, core[: len(core) // 2] + gapb + core[len(core) // 2:]
            elif k % 3 == 1:  # a deletion: a D run
                q, t = core[: len(core) // 3] + gapb + core[len(core) // 3:], core
            else:
                q, t = rnd(n), rnd(m)
            q, t = (q + rnd(max(0, n - len(q))))[:n], (t + rnd(max(0, m - len(t))))[:m]
            pairs.append((q, t))
    rb = synth.related_batch(9, 900, 900, seed=0xED6F)
    pairs += [(rb.query(p), rb.target(p)) for p in range(rb.n_pairs)]
    b = synth.from_pairs(pairs)
    plan = DevicePlan(aligner, b, mode, *sc, True, flags=TA_PLAN_CK)
    assert plan.ck and plan.walk == 64, (plan.blk, plan.ck, plan.walk)
    plan.close()
    want = oracle.align_batch(b, mode, *sc, True)
    got = run_plan(aligner, b, mode, sc, True, TA_PLAN_CK)
    np.testing.assert_array_equal(got.scores, want.scores)
    np.testing.assert_array_equal(got.target_begins, want.target_begins)
    for p in range(b.n_pairs):
        assert got.cigar(p) == want.cigar(p), (mode, sc, p, b.qlen[p], b.tlen[p])


@pytest.mark.parametrize("mode,sc", [(m, s) for m in (0, 1, 2) for s in ((1, -1, -1), (2, -3, -1), (3, 4, 0))])
def test_ck_walk_flex(aligner, oracle, mode, sc):
    """Checkpoints of the flexible fill (couples of different shapes, H itself in the
    checkpoints) walked by the recomputing walk, against the oracle: every mode, ragged
    couples of one to three passes, pairs coupled with themselves, long I and D runs,
    queries with other letters than A, C, G, T (the fill's non-table path) and a '-' in a
    target (the couple handed back to the int32 fill and the one-pair walk)."""
    if mode == 1 and sc[2] > 0:
        pytest.skip("local checkpoint walks need gap <= 0")
    rng = np.random.default_rng(0xF1E + 13 * mode + 5 * sc[0] - sc[1])
    al = np.frombuffer(b"ACGT", np.uint8)
    rnd = lambda k: al[rng.integers(4, size=k)].tobytes()  # noqa: E731
    pairs = []
    # (n, m of each couple's pairs): same pass count and n mod 16 within a group, so the
    # planner couples them; m within 25 % of waste
    for n, ms in ((517, (600, 520, 480, 555, 610)), (1030, (990, 1100, 940)), (2100, (700, 640, 690)),
                  (300, (260, 280, 300, 240))):
        for k, m in enumerate(ms):
            core = rnd(min(n, m) - 60)
            gapb = b"N" * (30 + 17 * k)
            if k % 3 == 0:  # an insertion in the target: an I run
                q, t = core, core[: len(core) // 2] + gapb + core[len(core) // 2:]
            elif k % 3 == 1:  # a deletion: a D run
                q, t = core[: len(core) // 3] + gapb + core[len(core) // 3:], core
            else:
                q, t = rnd(n), rnd(m)
            q, t = (q + rnd(max(0, n - len(q))))[:n], (t + rnd(max(0, m - len(t))))[:m]
            pairs.append((q, t))
    pairs.append((b"ACGTN" * 103 + b"AC", rnd(530)))  # a query letter past A, C, G, T (n = 517)
    pairs.append((rnd(517), rnd(200) + b"-" + rnd(300)))  # a free gap step in a target
    b = synth.from_pairs(pairs)
    plan = DevicePlan(aligner, b, mode, *sc, True, flags=TA_PLAN_CK)
    assert plan.ck and plan.walk == 64 and plan.flex_pairs > 0, (plan.blk, plan.ck, plan.walk, plan.flex_pairs)
    plan.close()
    want = oracle.align_batch(b, mode, *sc, True)
    got = run_plan(aligner, b, mode, sc, True, TA_PLAN_CK)
    np.testing.assert_array_equal(got.scores, want.scores)
    np.testing.assert_array_equal(got.target_begins, want.target_begins)
    for p in range(b.n_pairs):
        assert got.cigar(p) == want.cigar(p), (mode, sc, p, b.qlen[p], b.tlen[p])


def test_ck_walk_long_free_run(aligner, oracle):
    """gap = 0 (local walks over checkpoints allow it): a free insertion of 9,000 target
    columns inside the local path, an I run that crosses ~560 windows and passes the
    event's 14-bit count (8,192: the walk splits it), plus a long free
    deletion in a second pair; against the oracle."""
    rng = np.random.default_rng(0x8192)
    al = np.frombuffer(b"ACGT", np.uint8)
    core = al[rng.integers(4, size=240)].tobytes()
    pairs = [(core, core[:120] + b"N" * 9000 + core[120:]),   # I run of 9,000
             (core[:90] + b"N" * 8500 + core[90:], core)]     # D run of 8,500
    b = synth.from_pairs(pairs)
    sc = (2, -3, 0)
    plan = DevicePlan(aligner, b, 1, *sc, True, flags=TA_PLAN_CK)
    assert plan.ck and plan.walk == 64, (plan.blk, plan.ck, plan.walk)
    plan.close()
    want = oracle.align_batch(b, 1, *sc, True)
    got = run_plan(aligner, b, 1, sc, True, TA_PLAN_CK)
    np.testing.assert_array_equal(got.scores, want.scores)
    np.testing.assert_array_equal(got.target_begins, want.target_begins)
    for p in range(b.n_pairs):
        assert got.cigar(p) == want.cigar(p), (p, got.cigar(p)[:60], want.cigar(p)[:60])


def test_local_walk_long_runs(aligner, oracle):
    """Local paths with long gap and match runs (past the group walk's 32-cell
    clip and the one-pair walk's 64-cell windows) across pass and tile edges
    (1,100 x 1,100 pairs: two query passes); equal shapes so the couples run packed."""
    rng = np.random.default_rng(0x1046)
    al = np.frombuffer(b"ACGT", np.uint8)
    pairs = []
    for k in range(64):
        core = al[rng.integers(4, size=300)].tobytes()
        ins = b"N" * (40 + (k % 7) * 11)  # matches nothing: one contiguous gap run
        if k % 2:  # a long insertion in the target (I run), then a long deletion (D runs)
            q = core[:150] + core[150:]
            t = core[:150] + ins + core[150:]
        else:
            q = core[:120] + ins + core[120:]
            t = core
        pad = 1100 - len(q), 1100 - len(t)
        pairs.append((q + al[rng.integers(4, size=pad[0])].tobytes(), t + al[rng.integers(4, size=pad[1])].tobytes()))
    b = synth.from_pairs(pairs)
    for sc in ((5, -4, -1), (2, -3, -1)):
        want = oracle.align_batch(b, 1, *sc, True)
        for flags in (0, TA_PLAN_WALK1, TA_PLAN_WALK2):
            got = run_plan(aligner, b, 1, sc, True, flags)
            np.testing.assert_array_equal(got.scores, want.scores)
            np.testing.assert_array_equal(got.target_begins, want.target_begins)
            for p in range(b.n_pairs):
                assert got.cigar(p) == want.cigar(p), (sc, flags, p)
    import re

    runs = [(int(c), op) for p in range(b.n_pairs) for c, op in re.findall(rb"(\d+)([MID])", want.cigar(p))]
    assert max(c for c, op in runs if op == b"I") > 32 and max(c for c, op in runs if op == b"D") > 32
    assert max(c for c, op in runs if op == b"M") > 64


def test_config5_shape_multichunk(aligner):
    """Config 5 shape forced through >= 4 chunks (small workspace budget):
    every chunk reuses the code workspace; the first 32 pairs bit-exact vs the
    reference digest, all 64 equal to the one-chunk plan and path-checked."""
    from oracle.pyoracle import cigar_check_batch

    b = synth.related_batch(64, 10000, 10000, 0x5EED)
    per_pair = 10 * (10000 + 63) * 64 * 4  # 2-bit code dwords of one 10 kb x 10 kb pair
    plan = DevicePlan(aligner, b, 2, 1, -1, -1, True, workspace_budget=16 * per_pair)
    assert plan.chunks >= 4, plan.chunks
    plan.run()
    r = plan.results()
    plan.close()
    meta, d = load_digest("cfg5_semi_sample")
    np.testing.assert_array_equal(r.scores[:32], d["scores"])
    np.testing.assert_array_equal(r.cigar_lens[:32], d["cigar_lens"])
    sha, _ = cigar_digest(r, 32)
    assert sha == meta["cigar_sha256"]
    one = run_plan(aligner, b, 2, (1, -1, -1), True)
    np.testing.assert_array_equal(one.scores, r.scores)
    assert one.cigars() == r.cigars()
    st = cigar_check_batch(b, 2, 1, -1, -1, r.scores, r.target_begins, r.arena, r.cigar_offsets, r.cigar_lens)
    assert not st.any()


def test_config5_stated_size_strided(aligner):
    """Config 5 at its stated size: 100,000 related 10 kb x 10 kb pairs
    generated in HBM (as bench.py does), semi-global, CIGAR on, one plan of
    >= 4 chunks; the 128 pairs at stream positions 781*k, which fall in every
    chunk, are bit-exact against the reference's stratified digest."""
    import torch

    P, L = 100000, 10000
    q, t = synth.related_batch_torch(P, L, L, 0x5EED, device="cuda")
    off = torch.arange(P, dtype=torch.int64, device="cuda") * L
    ln = np.full(P, L, np.uint32)
    shapes = synth.PairBatch(np.zeros(0, np.uint8), np.zeros(P, np.uint64), ln, np.zeros(0, np.uint8),
                             np.zeros(P, np.uint64), ln)
    plan = DevicePlan(aligner, shapes, 2, 1, -1, -1, True, workspace_budget=200 << 30, inputs=(q, off, t, off))
    try:
        assert plan.chunks >= 4, plan.chunks
        plan.run()
        meta, d = load_digest("cfg5_semi_strided")
        idx = d["indices"]
        chunks = plan.pair_chunks()[idx]
        assert len(np.unique(chunks)) == plan.chunks, (np.unique(chunks), plan.chunks)
        r = plan.results_at(idx)
        np.testing.assert_array_equal(r.scores, d["scores"])
        np.testing.assert_array_equal(r.target_begins, d["target_begins"])
        np.testing.assert_array_equal(r.cigar_lens, d["cigar_lens"])
        sha, _ = cigar_digest(r, len(idx))
        assert sha == meta["cigar_sha256"]
    finally:
        plan.close()
        aligner.release()  # the module's context: give the ~200 GB code workspace back
        del q, t
        torch.cuda.empty_cache()


def test_related_batch_generated_in_hbm():
    """bench.py's config-5 inputs are generated on the GPU: same bytes as the
    host generator (int64 wrap-around arithmetic on the device)."""
    import torch

    want = synth.related_batch(40, 1000, 1000, 0x5EED, first_pair=7)
    q, t = synth.related_batch_torch(40, 1000, 1000, 0x5EED, first_pair=7, device="cuda", block=16)
    assert q.cpu().numpy().tobytes() == want.qbytes.tobytes()
    assert t.cpu().numpy().tobytes() == want.tbytes.tobytes()


def test_host_batch_paths(aligner, oracle):
    """ta_align_batch's two download paths (whole output block when the
    CIGAR slots are small; records first and device compaction when large),
    sequences packed into the pinned upload or sent on their own, and
    HostBatchRunner (pinned caller buffers) -- all identical to the oracle."""
    from bioinfo1_amd.align import HostBatchRunner

    small = synth.related_batch(50, 300, 280, seed=3)          # < 4 MB of slots, packed sequences
    big = synth.related_batch(1200, 1000, 1000, seed=4)       # 4.8 MB of slots: device compaction
    large_in = synth.uniform_batch(2100, 1000, 1000, seed=5)  # 4.2 MB of sequences: separate upload
    for b, mode in ((small, 0), (big, 1), (large_in, 2)):
        want = oracle.align_batch(b, mode, 1, -1, -1, True)
        got = aligner.align_batch(b, mode, 1, -1, -1, True)
        np.testing.assert_array_equal(got.scores, want.scores)
        np.testing.assert_array_equal(got.target_begins, want.target_begins)
        assert got.cigars() == want.cigars()
        hr = HostBatchRunner(aligner, b, mode, 1, -1, -1, True)
        for _ in range(2):
            hr.run()
            h = hr.results()
            np.testing.assert_array_equal(h.scores, want.scores)
            assert h.cigars() == want.cigars()


def test_plans_on_two_streams(aligner, oracle):
    """Two plans of one context executed on two torch streams back to back:
    the second waits for the first (shared workspace), results intact."""
    import torch

    b1 = synth.related_batch(200, 700, 650, seed=31)
    b2 = synth.related_batch(200, 900, 800, seed=32)
    p1 = DevicePlan(aligner, b1, 1, 1, -1, -1, True)
    p2 = DevicePlan(aligner, b2, 2, 1, -1, -1, True)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        with torch.cuda.stream(s1):
            p1.run()
        with torch.cuda.stream(s2):
            p2.run()
    torch.cuda.synchronize()
    for p, b, mode in ((p1, b1, 1), (p2, b2, 2)):
        want = oracle.align_batch(b, mode, 1, -1, -1, True)
        r = p.results()
        np.testing.assert_array_equal(r.scores, want.scores)
        assert r.cigars() == want.cigars()
        p.close()


def test_flex_local_no_positive_cell(aligner, oracle):
    """Local mode where no cell is positive (all mismatches): score 0, CIGAR
    "1\0", target_begin 2 -- the first cell in row-major order -- through the
    flexible fill's argmax (ragged shapes, several passes)."""
    rng = np.random.default_rng(0x0C)
    qa, ta = np.frombuffer(b"AC", np.uint8), np.frombuffer(b"GT", np.uint8)
    pairs = []
    for k in range(12):  # couples: same pass count and n mod 16, different m
        n0 = int(rng.integers(40, 2600))
        for h in range(2):
            n = n0 - 16 * h
            m = int(rng.integers(max(1, n0 * 8 // 10), n0 * 12 // 10 + 1))
            pairs.append((qa[rng.integers(2, size=n)].tobytes(), ta[rng.integers(2, size=m)].tobytes()))
    b = synth.from_pairs(pairs)
    plan = DevicePlan(aligner, b, 1, 1, -1, -1, True)
    assert plan.flex_pairs >= 12, plan.flex_pairs
    plan.close()
    want = oracle.align_batch(b, 1, 1, -1, -1, True)
    got = run_plan(aligner, b, 1, (1, -1, -1), True)
    np.testing.assert_array_equal(got.scores, want.scores)
    np.testing.assert_array_equal(got.target_begins, want.target_begins)
    assert got.cigars() == want.cigars()


def test_local_walk_choices(aligner, oracle):
    """Local walks of every kind on the same batches: lane walks (default for
    short pairs with an int8 gap), two-pair run walks (TA_PLAN_WALK2, and the
    default when |gap| > 127), one-pair run walks (TA_PLAN_WALK1); '-' bytes
    make indel steps free (the lane walk's per-byte indel costs)."""
    rng = np.random.default_rng(0x1A2E)
    for alpha, sc in ((b"ACGT", (1, -1, -1)), (b"AC-GT", (2, -1, 3)), (b"ACGT", (300, -200, -150)),
                      (b"ACGTN-", (4, -3, -2))):
        al = np.frombuffer(alpha, np.uint8)
        pairs = [(al[rng.integers(len(al), size=int(rng.integers(1, 700)))].tobytes(),
                  al[rng.integers(len(al), size=int(rng.integers(1, 700)))].tobytes()) for _ in range(150)]
        b = synth.from_pairs(pairs)
        want = oracle.align_batch(b, 1, *sc, True)
        for flags in (0, TA_PLAN_WALK1, TA_PLAN_WALK2):
            got = run_plan(aligner, b, 1, sc, True, flags)
            np.testing.assert_array_equal(got.scores, want.scores)
            for p in range(b.n_pairs):
                assert got.cigar(p) == want.cigar(p), (alpha, sc, flags, p)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_self_coupled_single_pair_with_dash(aligner, oracle, mode):
    """A one-pair batch of >= 4,096 cells runs coupled with itself in the packed
    fill (ta_planner.cpp); a '-' sends it back to the int32 fill, which must
    take it ONCE (two waves on one pair of > 1,024 rows would share its
    in-place pass boundary row).  '-' in the query, then in the target."""
    rng = np.random.default_rng(0x5E1F + mode)
    al = np.frombuffer(b"ACGT", np.uint8)
    for where in ("query", "target"):
        q = al[rng.integers(4, size=1500)].copy()
        t = q.copy()
        flip = rng.random(1500) < 0.1
        t[flip] = al[rng.integers(4, size=int(flip.sum()))]
        (q if where == "query" else t)[[100, 700, 1400]] = ord("-")
        b = synth.from_pairs([(q.tobytes(), t.tobytes())])
        want = oracle.align_batch(b, mode, 1, -1, -1, True)
        for _ in range(3):
            got = aligner.align_batch(b, mode, 1, -1, -1, True)
            assert (int(got.scores[0]), int(got.target_begins[0]), got.cigar(0)) == (
                int(want.scores[0]), int(want.target_begins[0]), want.cigar(0)), where


def test_single_pair_server(kat_cases, random_cases, oracle):
    """The resident single-pair server (ta_server_*, the drop-in's path for
    pairs that fit): every KAT and random case of its mode, score-only too;
    multi-pass pairs (n > 1024); calls from 8 threads at once; a pause past
    the idle stop, after which the next call relaunches the kernel."""
    import threading
    import time

    from bioinfo1_amd.align import Server

    cases = [c for c in kat_cases + random_cases if not c["error"]]
    for mode in (0, 1, 2):
        srv = Server(0, mode)
        try:
            for c in (c for c in cases if c["type"] == mode):
                q, t = bytes.fromhex(c["query"]), bytes.fromhex(c["target"])
                args = (c["match"], c["mismatch"], c["gap"])
                if not srv.fits(len(q), len(t), *args):
                    continue
                got = srv.align(q, t, *args)
                assert got == (c["score"], bytes.fromhex(c["cigar"]), c["target_begin"]), (c["source"], got)
                assert srv.align(q, t, *args, want_cigar=False) == (c["score"], None, c["target_begin"])
            b = synth.related_batch(6, 2500, 2300, seed=91 + mode)  # 3 passes
            want = oracle.align_batch(b, mode, 1, -1, -1, True)
            for p in range(b.n_pairs):
                assert srv.align(b.query(p), b.target(p), 1, -1, -1) == (
                    int(want.scores[p]), want.cigar(p), int(want.target_begins[p]))
            rb = synth.ragged_batch(160, 0, 600, seed=0x7E + mode, alphabet=b"ACGT-N")
            rw = oracle.align_batch(rb, mode, 2, -1, -1, True)
            errs = []

            def worker(k):
                for p in range(k, rb.n_pairs, 8):
                    got = srv.align(rb.query(p), rb.target(p), 2, -1, -1)
                    if got != (int(rw.scores[p]), rw.cigar(p), int(rw.target_begins[p])):
                        errs.append(p)

            th = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            assert not errs, errs[:5]
            time.sleep(0.5)  # past the idle stop (200 ms): the kernel has ended
            assert not srv.running()
            assert srv.align(b"GTACC", b"GATACGTTA", 1, -1, -1)[0] == want_score_cfg1(mode)
            assert srv.running()
            assert not srv.fits(5000, 10, 1, -1, -1) and not srv.fits(10, 20000, 1, -1, -1)
        finally:
            srv.close()


def test_single_pair_server_small(oracle):
    """The server's small-pair path (one, two or four query rows per lane up to
    n = 256, codes in LDS, serve_small): random pairs at its edges (n = 1 / 64 /
    128 / 256, m up to 1,024 / 481 / 209, ragged in between) over A C G T - N, several scoring schemes
    (positive gaps and matches below mismatches included), every mode, CIGAR
    and score-only, against the oracle."""
    from bioinfo1_amd import synth as S
    from bioinfo1_amd.align import Server

    rng = np.random.default_rng(0x5A11)
    shapes = [(1, 1), (1, 1024), (64, 1), (64, 1024), (64, 64), (2, 3), (63, 1023), (17, 200)]
    shapes += [(int(rng.integers(1, 65)), int(rng.integers(1, 1025))) for _ in range(40)]
    # two and four rows per lane (n up to 128 / 256, m as the LDS code budget allows)
    shapes += [(65, 480), (128, 481), (100, 300), (129, 200), (200, 200), (256, 209), (256, 1), (255, 33)]
    shapes += [(int(rng.integers(65, 129)), int(rng.integers(1, 482))) for _ in range(12)]
    shapes += [(int(rng.integers(129, 257)), int(rng.integers(1, 210))) for _ in range(12)]
    pairs = []
    for k, (n, m) in enumerate(shapes):
        a = b"ACGT-N" if k % 3 == 0 else b"ACGT"
        q = bytes(rng.choice(np.frombuffer(a, np.uint8), n))
        t = bytes(rng.choice(np.frombuffer(a, np.uint8), m))
        if k % 2:  # related: the query drawn from the target
            st = int(rng.integers(0, max(1, m - n + 1)))
            q = (t[st:st + n] + q)[:n]
        pairs.append((q, t))
    batch = S.from_pairs(pairs)
    for mode in (0, 1, 2):
        srv = Server(0, mode)
        try:
            for sc in ((1, -1, -1), (2, -3, -2), (-1, 1, 1), (3, 0, 2)):
                want = oracle.align_batch(batch, mode, *sc, True)
                for p, (q, t) in enumerate(pairs):
                    assert srv.fits(len(q), len(t), *sc)
                    got = srv.align(q, t, *sc)
                    assert got == (int(want.scores[p]), want.cigar(p), int(want.target_begins[p])), (mode, sc, p)
                    assert srv.align(q, t, *sc, want_cigar=False) == (int(want.scores[p]), None,
                                                                     int(want.target_begins[p]))
        finally:
            srv.close()


def want_score_cfg1(mode):
    return {0: -1, 1: 3, 2: 2}[mode]  # SURVEY §4 table 2, GTACC / GATACGTTA


def test_host_pipeline(aligner, oracle):
    """align.HostPipeline (host inputs -> host results, transfers overlapped with
    the kernels, two plans alternating): after several steps the last results
    equal the oracle's, in all modes and score-only."""
    from bioinfo1_amd.align import HostPipeline

    b = synth.related_batch(300, 700, 650, seed=41)
    for mode in (0, 1, 2):
        want = oracle.align_batch(b, mode, 1, -1, -1, True)
        for cig in (True, False):
            hp = HostPipeline(aligner, b, mode, 1, -1, -1, cig)
            for _ in range(5):
                hp.step()
            hp.drain()
            r = hp.results()
            hp.close()
            np.testing.assert_array_equal(r.scores, want.scores)
            np.testing.assert_array_equal(r.target_begins, want.target_begins)
            if cig:
                assert r.cigars() == want.cigars()


def test_device_pipeline(aligner, oracle):
    """align.DevicePipeline (batch k's traceback beside batch k+1's fill, one
    context per slot) over THREE different batches of one shape in turn, so each
    slot gets a different batch at every use (depth 2): every step's results --
    snapshotted on the caller's stream right after the step, with no sync in
    between -- equal the oracle's for its own batch.  A walk reading a workspace
    its slot's next fill already overwrote, or a fill starting before its own
    batch's inputs, shows up as another batch's results.  Checkpoint walks, the
    int32 path, and plans split into chunks (a small workspace budget), whose
    fills and walks interleave per chunk."""
    import torch

    from bioinfo1_amd.align import DevicePipeline, DevicePlan

    bs = [synth.related_batch(200, 900, 800, seed=43 + v) for v in range(3)]
    dev = torch.device("cuda", 0)
    ins = [tuple(torch.from_numpy(np.ascontiguousarray(a)).to(dev)
                 for a in (b.qbytes, b.qoff.view(np.int64), b.tbytes, b.toff.view(np.int64))) for b in bs]
    torch.cuda.synchronize()
    for mode, flags, budget in ((1, TA_PLAN_CK, 0), (1, 0, 0), (0, 0, 0), (1, TA_PLAN_CK, 12 << 20),
                                (2, 0, 10 << 20)):
        wants = [oracle.align_batch(b, mode, 1, -1, -1, True) for b in bs]
        first = DevicePlan(Aligner(0), bs[0], mode, 1, -1, -1, True, workspace_budget=budget, flags=flags)
        pipe = DevicePipeline(0, bs[0], mode, 1, -1, -1, True, workspace_budget=budget, flags=flags, first=first)
        assert budget == 0 or pipe.chunks > 1
        snaps = []
        for k in range(7):
            plan = pipe.step(inputs=ins[k % 3])
            dst, off = plan.compact_cigars()
            snaps.append((k % 3, plan.score.clone(), plan.target_begin.clone(), plan.cigar_len.clone(), dst, off))
        pipe.check()
        for v, sc, tb, cl, dst, off in snaps:
            want = wants[v]
            np.testing.assert_array_equal(sc.cpu().numpy(), want.scores)
            np.testing.assert_array_equal(tb.cpu().numpy().view(np.uint32), want.target_begins)
            np.testing.assert_array_equal(cl.cpu().numpy().view(np.uint32), want.cigar_lens)
            assert dst[:int(off[-1])].cpu().numpy().tobytes() == b"".join(want.cigars()), (mode, flags, budget, v)
        pipe.close()
        first.close()
        first.aligner.close()


@pytest.mark.gpu
def test_int32_pass_pipeline(aligner, oracle):
    """Multi-pass int32 pairs run one wave per (pair, pass) (fill_pipe_kernel,
    fill_combine_kernel): local pairs past flex_local_fits (scores beyond the
    int16 range, the natural int32 case), a 69-pass query, empty and one-pass
    pairs in the same chunk, several chunks; against the oracle and against the
    serial-pass fill (TA_PLAN_SERIAL_PASSES)."""
    rel = synth.related_batch(3, 6500, 6400, seed=0x1F7)
    rng = np.random.default_rng(0x1F8)
    al = np.frombuffer(b"ACGT", np.uint8)

    def rnd(k):
        return al[rng.integers(4, size=k)].tobytes()

    pairs = [(rel.query(p), rel.target(p)) for p in range(3)]
    pairs += [(rnd(70000), rnd(200)), (b"", rnd(50)), (rnd(40), b""), (rnd(900), rnd(1200)), (rnd(3000), rnd(2500)),
              (rnd(2049), rnd(64))]
    b = synth.from_pairs(pairs)
    for mode, sc in ((1, (5, -4, -4)), (0, (1, -1, -1)), (2, (2, -1, -1)), (1, (1, -1, -1))):
        want = oracle.align_batch(b, mode, *sc, True)
        if sc[0] == 5:  # the long local pairs leave the packed kernels: pipelined, walk in its own kernel
            plan = DevicePlan(aligner, b, mode, *sc, True)
            assert not plan.fused and plan.dual_pairs < b.n_pairs
            plan.close()
        for flags, budget in ((0, 0), (TA_PLAN_INT32_ONLY, 0), (TA_PLAN_INT32_ONLY, 1 << 20),
                              (TA_PLAN_INT32_ONLY | TA_PLAN_SERIAL_PASSES, 0)):
            for cig in (True, False):
                got = run_plan(aligner, b, mode, sc, cig, flags, budget=budget)
                np.testing.assert_array_equal(got.scores, want.scores)
                np.testing.assert_array_equal(got.target_begins, want.target_begins)
                if cig:
                    for p in range(b.n_pairs):
                        assert got.cigar(p) == want.cigar(p), (mode, sc, flags, budget, p)
        got = aligner.align_batch(b, mode, *sc, True)  # host-memory batch (ta_align_batch)
        np.testing.assert_array_equal(got.scores, want.scores)
        for p in range(b.n_pairs):
            assert got.cigar(p) == want.cigar(p), (mode, sc, "host", p)
        # one pair per call (the drop-in's path for pairs the server does not take)
        assert align(b.query(0), b.target(0), mode, *sc) == (int(want.scores[0]), want.cigar(0),
                                                              int(want.target_begins[0]))
