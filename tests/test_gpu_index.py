"""Feature index on device (csrc/ivf.hip through the C-ABI) vs the faiss restatement in oracle/ivf.py,
and the pipeline with index_rate > 0 vs the oracle pipeline (rvc/infer/pipeline.py:338-342, :378-388,
:430-434). Bar: identical ids, distances within float32 summation-order rounding (rel 1e-5), the blend
bit-exact given the same search result (numpy/torch float32 order), big_npy rows exact."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def _clustered(n, d, seed, ncl=24):
    rng = np.random.default_rng(seed)
    centers = rng.standard_normal((ncl, d)).astype(np.float32) * 2
    return (centers[rng.integers(0, ncl, n)] + rng.standard_normal((n, d)).astype(np.float32)).astype(np.float32)


@pytest.fixture(scope="module")
def ix_engine():
    from rvcx.engine import Engine

    e = Engine(0)
    yield e
    e.close()


def _load(eng, idx):
    from oracle import ivf
    from rvcx.infer.index import IndexIVFFlat

    return IndexIVFFlat(eng, data=ivf.write_ivfflat(idx))


@pytest.mark.parametrize("nprobe", [1, 3])
def test_search_matches_oracle(ix_engine, nprobe):
    from oracle import ivf

    x = _clustered(3000, 768, 1)
    idx = ivf.build_ivfflat(x, nlist=48, nprobe=nprobe)
    h = _load(ix_engine, idx)
    assert (h.d, h.ntotal, h.nlist, h.nprobe) == (768, 3000, 48, nprobe)
    q = _clustered(400, 768, 2)
    D, I = h.search(q, 8)
    Do, Io = ivf.search(idx, q, 8)
    np.testing.assert_array_equal(I, Io)
    np.testing.assert_allclose(D, Do, rtol=1e-5)
    np.testing.assert_array_equal(h.reconstruct_n(0, h.ntotal), x)
    np.testing.assert_array_equal(h.reconstruct_n(100, 7), x[100:107])


def test_search_k_and_padding(ix_engine):
    from oracle import ivf

    x = _clustered(60, 256, 3, ncl=6)
    idx = ivf.build_ivfflat(x, nlist=20, nprobe=1)  # many lists shorter than k
    h = _load(ix_engine, idx)
    q = _clustered(64, 256, 4, ncl=6)
    for k in (1, 5, 8, 16):
        D, I = h.search(q, k)
        Do, Io = ivf.search(idx, q, k)
        np.testing.assert_array_equal(I, Io)
        np.testing.assert_allclose(D, Do, rtol=1e-5)
    assert (Io == -1).any()  # the padding path was exercised


def test_empty_lists_sparse_file(ix_engine):
    from oracle import ivf

    x = _clustered(40, 64, 5, ncl=2)
    idx = ivf.build_ivfflat(x, nlist=16, nprobe=2)
    idx.list_vecs[3] = idx.list_vecs[3][:0]
    idx.list_ids[3] = idx.list_ids[3][:0]
    keep = np.concatenate(idx.list_ids)
    # renumber ids 0..n-1 (RVC indexes hold a permutation of 0..ntotal-1)
    remap = {int(i): j for j, i in enumerate(np.sort(keep))}
    idx.list_ids = [np.array([remap[int(i)] for i in ids], dtype=np.int64) for ids in idx.list_ids]
    from rvcx.infer.index import IndexIVFFlat

    h = IndexIVFFlat(ix_engine, data=ivf.write_ivfflat(idx, sparse=True))
    q = _clustered(32, 64, 6, ncl=2)
    D, I = h.search(q, 8)
    Do, Io = ivf.search(idx, q, 8)
    np.testing.assert_array_equal(I, Io)
    np.testing.assert_allclose(D, Do, rtol=1e-5)


def test_retrieve_blend_bit_exact(ix_engine):
    from oracle import ivf

    x = _clustered(2000, 768, 7)
    idx = ivf.build_ivfflat(x, nlist=32, nprobe=1)
    h = _load(ix_engine, idx)
    q = _clustered(300, 768, 8)
    q[5] = x[17]  # an exact hit: distance 0 -> nan row, as in the reference
    D, I = h.search(q, 8)
    big = h.reconstruct_n(0, h.ntotal)
    for rate in (0.75, 0.3, 1.0):
        got = h.retrieve(q, rate)
        ref = ivf.retrieve_speaker_embeddings(q, D, I, big, rate)
        np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
        ok = ~np.isnan(ref)
        assert np.array_equal(got[ok], ref[ok]), float(np.abs(got[ok] - ref[ok]).max())
    assert np.isnan(got[5]).all()


def test_bad_files_raise(ix_engine):
    from oracle import ivf
    from rvcx._lib import RvcxError
    from rvcx.infer.index import IndexIVFFlat

    x = _clustered(100, 64, 9)
    buf = ivf.write_ivfflat(ivf.build_ivfflat(x, nlist=4))
    for bad in (buf[:-8], b"IxF2" + buf[4:], buf[:40]):
        with pytest.raises(RvcxError):
            IndexIVFFlat(ix_engine, data=bad)


def test_pipeline_with_index_matches_oracle(engine, synth_w, hubert_w, rmvpe_w, tmp_path):
    """PipelineMLX.pipeline(file_index=..., index_rate=0.75) vs the oracle pipeline with the same index."""
    from oracle import hubert as ohubert
    from oracle import ivf
    from oracle.metrics import spectrogram_correlation
    from rvcx import synthetic
    from rvcx.config import HUBERT_BASE
    from rvcx.infer import Config, HubertModel, PipelineMLX, RMVPE0Predictor, Synthesizer

    from test_gpu_pipeline_api import NoiseRecorder, oracle_pipeline

    # index over the oracle's HuBERT features of other speech (what extract_index.py builds from)
    train = synthetic.speech_like(16000 * 4, seed=31).astype(np.float32)
    with torch.no_grad():
        feats = ohubert.hubert_forward(hubert_w, HUBERT_BASE, torch.from_numpy(train).view(1, -1), "v2")[0].numpy()
    idx = ivf.build_ivfflat(feats, nlist=6, nprobe=1)
    path = tmp_path / "added_IVF6_Flat_nprobe_1_v2.index"
    path.write_bytes(ivf.write_ivfflat(idx))

    g = golden("pipeline_2p5s.npz")
    noise = NoiseRecorder(44)
    orc = oracle_pipeline(synth_w, hubert_w, rmvpe_w, noise)
    ref = orc.pipeline(0, g["audio"].copy(), protect=0.33, index=ivf.read_ivfflat(path.read_bytes()), index_rate=0.75)
    ez, es = noise.cat()
    hub, rm, net_g = HubertModel(engine), RMVPE0Predictor(engine), Synthesizer(engine)
    pipe = PipelineMLX(48000, Config(), hub, rm)
    out = pipe.pipeline(hub, net_g, 0, g["audio"], 0, "rmvpe", str(path), 0.75, True, 1.0, "v2", 0.33, False, 1.0,
                        False, 155.0, eps_z=ez, eps_src=es)
    assert out.shape == ref.shape
    assert spectrogram_correlation(out, ref) > 0.99
    # the retrieval changed the output (index_rate 0 gives a different conversion)
    out0 = pipe.pipeline(hub, net_g, 0, g["audio"], 0, "rmvpe", str(path), 0.0, True, 1.0, "v2", 0.33, False, 1.0,
                         False, 155.0, eps_z=ez, eps_src=es)
    assert spectrogram_correlation(out0, ref) < spectrogram_correlation(out, ref)
    # a missing index file means no retrieval (pipeline.py:430), not an error
    out_missing = pipe.pipeline(hub, net_g, 0, g["audio"], 0, "rmvpe", str(tmp_path / "none.index"), 0.75, True,
                                1.0, "v2", 0.33, False, 1.0, False, 155.0, eps_z=ez, eps_src=es)
    np.testing.assert_array_equal(out_missing, out0)
