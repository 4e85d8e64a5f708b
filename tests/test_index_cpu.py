"""Feature index oracle (oracle/ivf.py): faiss IndexIVFFlat byte layout, search semantics and the
pipeline's retrieval blend (rvc/infer/pipeline.py:378-388). CPU only.

Parity against faiss itself is unpinned (faiss-cpu 1.7.4 is not installed and the reference holds no
.index fixture); these tests pin the restatement to its own invariants: exhaustive search equals a
brute-force scan, the writer and reader are inverse, numpy's rounding order is the one restated."""
import struct

import numpy as np
import pytest


def _data(n=600, d=64, seed=0):
    rng = np.random.default_rng(seed)
    centers = rng.standard_normal((12, d)).astype(np.float32) * 3
    x = centers[rng.integers(0, 12, n)] + rng.standard_normal((n, d)).astype(np.float32)
    return x.astype(np.float32)


@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("direct_map", [0, 1])
def test_write_read_roundtrip(sparse, direct_map):
    from oracle import ivf

    x = _data()
    idx = ivf.build_ivfflat(x, nlist=10, nprobe=2)
    buf = ivf.write_ivfflat(idx, sparse=sparse, direct_map=direct_map)
    assert buf[:4] == b"IwFl" and buf[0x35:0x39] == b"IxF2"  # layout the reference's Swift reader relies on
    assert struct.unpack("<i", buf[4:8])[0] == 64 and struct.unpack("<q", buf[8:16])[0] == 600
    back = ivf.read_ivfflat(buf)
    assert (back.d, back.nlist, back.nprobe, back.ntotal) == (64, 10, 2, 600)
    np.testing.assert_array_equal(back.centroids, idx.centroids)
    for a, b in zip(back.list_vecs, idx.list_vecs):
        np.testing.assert_array_equal(a, b)
    for a, b in zip(back.list_ids, idx.list_ids):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(ivf.reconstruct_n(back, 0, 600), x)


def test_reader_rejects_other_index_types():
    from oracle import ivf

    idx = ivf.build_ivfflat(_data(), nlist=4)
    buf = bytearray(ivf.write_ivfflat(idx))
    with pytest.raises(ValueError):
        ivf.read_ivfflat(b"IxF2" + bytes(buf[4:]))
    with pytest.raises(ValueError):
        ivf.read_ivfflat(bytes(buf[:-10]))


def test_exhaustive_search_is_brute_force():
    from oracle import ivf

    x = _data()
    idx = ivf.build_ivfflat(x, nlist=8, nprobe=8)
    q = _data(40, seed=3)
    D, I = ivf.search(idx, q, 8)
    full = ((q[:, None, :].astype(np.float64) - x[None].astype(np.float64)) ** 2).sum(-1)
    order = np.lexsort((np.broadcast_to(np.arange(len(x)), full.shape), full), axis=1)[:, :8]
    np.testing.assert_array_equal(I, order)
    np.testing.assert_allclose(D, np.take_along_axis(full, order, 1).astype(np.float32), rtol=1e-6)
    assert np.all(np.diff(D, axis=1) >= 0)


def test_short_lists_are_padded():
    from oracle import ivf

    x = _data(30)
    idx = ivf.build_ivfflat(x, nlist=10, nprobe=1)
    D, I = ivf.search(idx, x[:5], 8)
    for q in range(5):
        n = len(idx.list_ids[int(np.argmin(((idx.centroids - x[q]) ** 2).sum(1)))])
        if n < 8:
            assert np.all(I[q, n:] == -1) and np.all(np.isinf(D[q, n:]))


def test_numpy_rounding_order_of_the_blend():
    """The device kernel restates these float32 orders: pairwise row sum of 8, sequential axis-1 sum."""
    rng = np.random.default_rng(1)
    a = (rng.standard_normal((2000, 8)) * 10.0 ** rng.integers(-3, 4, (2000, 8))).astype(np.float32)
    s = a.sum(axis=1, keepdims=True)[:, 0]
    tree = ((a[:, 0] + a[:, 1]) + (a[:, 2] + a[:, 3])) + ((a[:, 4] + a[:, 5]) + (a[:, 6] + a[:, 7]))
    np.testing.assert_array_equal(s, tree)
    b = rng.standard_normal((50, 8, 768)).astype(np.float32)
    seq = b[:, 0].copy()
    for j in range(1, 8):
        seq = seq + b[:, j]
    np.testing.assert_array_equal(np.sum(b, axis=1), seq)


def test_retrieve_semantics():
    from oracle import ivf

    x = _data(200)
    idx = ivf.build_ivfflat(x, nlist=4, nprobe=1)
    big = ivf.reconstruct_n(idx, 0, idx.ntotal)
    q = _data(16, seed=9)
    D, I = ivf.search(idx, q, 8)
    out = ivf.retrieve_speaker_embeddings(q, D, I, big, 0.75)
    w = (1 / D.astype(np.float64)) ** 2
    w /= w.sum(1, keepdims=True)
    ref = 0.75 * (big[I] * w[:, :, None]).sum(1) + 0.25 * q
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-5)
    # an exact hit (distance 0) gives inf/inf = nan weights, as in the reference
    D2, I2 = ivf.search(idx, x[:1], 8)
    assert D2[0, 0] == 0
    assert np.isnan(ivf.retrieve_speaker_embeddings(x[:1], D2, I2, big, 0.5)).all()
