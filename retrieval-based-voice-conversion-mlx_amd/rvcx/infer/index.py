"""FAISS-compatible feature index handle on MI355X.

Replaces the reference's use of faiss in the pipeline (rvc/infer/pipeline.py:430-434 and :378-388;
rvc_mlx/infer/pipeline_mlx.py:267-278 and :183-201):

    index = read_index(path, engine)          # faiss.read_index(path)
    big_npy = index.reconstruct_n(0, index.ntotal)
    D, I = index.search(feats, k=8)

The file is parsed by librvcx.so (faiss 1.7.4 IndexIVFFlat layout) and kept in HBM; search and the
retrieval blend run as HIP kernels (csrc/ivf.hip). Outputs are numpy at this API edge, like faiss.
"""
from __future__ import annotations

import numpy as np

from ..engine import Engine


class IndexIVFFlat:
    """Device-resident IndexIVFFlat bound to one Engine (one rvcx context holds one index)."""

    def __init__(self, engine: Engine, path: str = None, data: bytes = None):
        if data is None:
            with open(path, "rb") as f:
                data = f.read()
        engine.index_load(data)
        self.engine = engine
        self.path = path
        info = engine.index_info()
        self.d, self.ntotal, self.nlist = info["d"], info["ntotal"], info["nlist"]
        self._nprobe = info["nprobe"]
        self.is_trained = True

    @property
    def nprobe(self) -> int:
        return self._nprobe

    @nprobe.setter
    def nprobe(self, v: int):
        self.engine.index_set_nprobe(int(v))
        self._nprobe = self.engine.index_info()["nprobe"]

    def _bound(self):
        info = self.engine.index_info()
        if info is None or info["ntotal"] != self.ntotal or info["d"] != self.d:
            raise RuntimeError("this index is no longer the one loaded in its engine")

    def search(self, x, k: int):
        """-> (D float32 [n, k], I int64 [n, k]) like faiss Index.search."""
        self._bound()
        d, i = self.engine.index_search(np.ascontiguousarray(x, dtype=np.float32), int(k))
        return self.engine.host(d), self.engine.host(i)

    def reconstruct_n(self, i0: int, ni: int) -> np.ndarray:
        self._bound()
        return self.engine.host(self.engine.index_reconstruct_n(i0, ni))

    def retrieve(self, feats, index_rate: float) -> np.ndarray:
        """Pipeline._retrieve_speaker_embeddings (pipeline.py:378-388) for feats [L, d] (or [1, L, d])."""
        self._bound()
        f = np.asarray(feats, dtype=np.float32)
        out = self.engine.host(self.engine.index_retrieve(f.reshape(-1, f.shape[-1]), index_rate))
        return out.reshape(f.shape)


def read_index(path: str, engine: Engine) -> IndexIVFFlat:
    return IndexIVFFlat(engine, path=path)
