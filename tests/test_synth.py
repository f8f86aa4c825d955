import numpy as np

from bioinfo1_amd import synth


def test_splitmix64_known_values():
    # splitmix64 from state 0: first outputs (published reference values)
    st = np.zeros(1, np.uint64)
    out = [int(synth.splitmix64_next(st)[0]) for _ in range(3)]
    assert out == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, 0x06C45D188009454F]


def test_uniform_batch_shape_and_determinism():
    b = synth.uniform_batch(8, 100, 120, seed=7)
    assert b.n_pairs == 8 and b.cells == 8 * 100 * 120
    assert set(b.qbytes.tobytes()) <= set(b"ACGT")
    b2 = synth.uniform_batch(8, 100, 120, seed=7)
    assert b.qbytes.tobytes() == b2.qbytes.tobytes() and b.tbytes.tobytes() == b2.tbytes.tobytes()
    # pair p depends only on seed ^ p: a range slice regenerates identically
    b3 = synth.uniform_batch(3, 100, 120, seed=7, first_pair=5)
    assert all(b3.query(k) == b.query(5 + k) and b3.target(k) == b.target(5 + k) for k in range(3))


def test_related_batch_is_related():
    b = synth.related_batch(4, 500, 500, seed=3)
    for p in range(4):
        q, t = b.query(p), b.target(p)
        assert len(q) == 500 and len(t) == 500
        same = sum(x == y for x, y in zip(q[:50], t[:50]))
        assert same > 10


def test_ragged_and_from_pairs():
    b = synth.ragged_batch(20, 0, 30, seed=1, alphabet=b"AC-")
    assert b.n_pairs == 20
    assert all(0 <= int(x) <= 30 for x in b.qlen)
    s = b.slice(3, 7)
    assert [s.query(k) for k in range(4)] == [b.query(3 + k) for k in range(4)]


def test_related_batch_blocked_is_prefix_stable():
    # the blocked generator gives the same pairs as one block
    a = synth.related_batch(5, 300, 280, seed=11)
    b = synth.related_batch(3, 300, 280, seed=11, first_pair=2)
    assert [a.target(2 + k) for k in range(3)] == [b.target(k) for k in range(3)]


def test_related_batch_torch_matches_numpy():
    import torch

    for (P, n, m, first) in ((7, 300, 280, 0), (5, 200, 450, 3), (3, 64, 64, 11)):
        want = synth.related_batch(P, n, m, seed=0x5EED, first_pair=first)
        q, t = synth.related_batch_torch(P, n, m, seed=0x5EED, first_pair=first, device="cpu", block=2)
        assert q.numpy().tobytes() == want.qbytes.tobytes()
        assert t.numpy().tobytes() == want.tbytes.tobytes()
