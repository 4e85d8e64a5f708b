"""Oracle: FAISS IndexIVFFlat file format, search and the speaker-embedding retrieval of the pipeline.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference calls faiss (``faiss-cpu==1.7.4``, requirements.txt:15), a third-party library that is
not installed here and not vendored in the reference, so its published algorithm is restated:

* file format -- faiss 1.7.4 ``impl/index_write.cpp`` / ``index_read.cpp`` for ``IndexIVFFlat``
  (fourcc ``IwFl``): index header (d int32, ntotal int64, two int64 dummies 1<<20, is_trained u8,
  metric int32 [+ metric_arg f32 when metric > 1]), nlist u64, nprobe u64, the coarse quantizer
  ``IndexFlatL2`` (``IxF2`` + header + u64 count + nlist*d f32), the direct map (type u8 + u64 count +
  int64s [+ hashtable pairs]), then ``ArrayInvertedLists`` (``ilar``, nlist u64, code_size u64, ``full``
  + u64 count + sizes, or ``sprs`` + u64 count + (list, size) pairs, then per non-empty list its codes
  (size*code_size bytes) followed by its ids (size int64)).  The reference's own reader of this format,
  Demos/iOS/.../FAISSIndexReader.swift:50-121, agrees on the header, the ``ilar`` block and the
  sizes; it reads ids before codes, which is the opposite of faiss's writer (codes first) -- faiss wins.
* search (``IndexIVF::search`` with ``nprobe`` lists, L2): coarse top-``nprobe`` centroids, then an exact
  L2 scan of the probed lists keeping the k best in a max-heap that admits a candidate only when it
  is strictly closer than the current worst (``CMax::cmp``), ties in the output ordered by id
  (``CMax::cmp2``); missing results are (+inf, -1) (``CMax::neutral``).  Distances here are computed
  in float64 and rounded to float32 (faiss accumulates in float32 with SIMD order -- unpinned).
* ``reconstruct_n(0, ntotal)`` (``IndexIVF::reconstruct_n``): row ``id`` of the result is the stored
  vector whose id is ``id``.
* ``retrieve_speaker_embeddings`` restates rvc/infer/pipeline.py:378-388 (= rvc_mlx/infer/
  pipeline_mlx.py:183-201) with the exact numpy float32 operations.

Parity status: **unpinned against faiss itself** (no faiss, no .index fixture in the reference);
anchored on the reference's call sites and on faiss's published format and heap semantics.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

METRIC_L2 = 1


@dataclass
class IvfFlat:
    d: int
    nlist: int
    nprobe: int
    centroids: np.ndarray                      # [nlist, d] float32
    list_vecs: List[np.ndarray] = field(default_factory=list)   # per list [n_i, d] float32
    list_ids: List[np.ndarray] = field(default_factory=list)    # per list [n_i] int64
    metric: int = METRIC_L2

    @property
    def ntotal(self) -> int:
        return int(sum(len(i) for i in self.list_ids))


# ------------------------------------------------------------------------------------ format
def _hdr(d: int, ntotal: int, metric: int) -> bytes:
    return struct.pack("<iqqqBi", d, ntotal, 1 << 20, 1 << 20, 1, metric)


def write_ivfflat(idx: IvfFlat, sparse: Optional[bool] = None, direct_map: int = 0) -> bytes:
    """Serialise like faiss.write_index(IndexIVFFlat) (faiss 1.7.4 index_write.cpp)."""
    d, nlist = idx.d, idx.nlist
    out = [b"IwFl", _hdr(d, idx.ntotal, idx.metric), struct.pack("<QQ", nlist, idx.nprobe)]
    out += [b"IxF2", _hdr(d, nlist, METRIC_L2), struct.pack("<Q", nlist * d),
            np.ascontiguousarray(idx.centroids, dtype="<f4").tobytes()]
    if direct_map == 0:
        out += [struct.pack("<BQ", 0, 0)]
    else:  # array direct map: id -> (list << 32 | offset)
        dm = np.zeros(idx.ntotal, dtype="<i8")
        for l, ids in enumerate(idx.list_ids):
            for o, i in enumerate(ids):
                dm[i] = (l << 32) | o
        out += [struct.pack("<BQ", 1, len(dm)), dm.tobytes()]
    sizes = [len(i) for i in idx.list_ids]
    out += [b"ilar", struct.pack("<QQ", nlist, 4 * d)]
    n_non0 = sum(1 for s in sizes if s > 0)
    if sparse is None:
        sparse = not (n_non0 > nlist // 2)
    if not sparse:
        out += [b"full", struct.pack("<Q", nlist), np.asarray(sizes, dtype="<u8").tobytes()]
    else:
        pairs = [v for l, s in enumerate(sizes) if s > 0 for v in (l, s)]
        out += [b"sprs", struct.pack("<Q", len(pairs)), np.asarray(pairs, dtype="<u8").tobytes()]
    for vecs, ids in zip(idx.list_vecs, idx.list_ids):
        if len(ids):
            out += [np.ascontiguousarray(vecs, dtype="<f4").tobytes(), np.asarray(ids, dtype="<i8").tobytes()]
    return b"".join(out)


def read_ivfflat(buf: bytes) -> IvfFlat:
    """Parse an IndexIVFFlat written by faiss (faiss 1.7.4 index_read.cpp)."""
    p = 0

    def take(n):
        nonlocal p
        if p + n > len(buf):
            raise ValueError("truncated faiss index")
        b = buf[p:p + n]
        p += n
        return b

    if take(4) != b"IwFl":
        raise ValueError("not an IndexIVFFlat (fourcc != IwFl)")
    d, ntotal, _, _, _, metric = struct.unpack("<iqqqBi", take(33))
    if metric > 1:
        take(4)
    nlist, nprobe = struct.unpack("<QQ", take(16))
    if take(4) != b"IxF2":
        raise ValueError("coarse quantizer is not IndexFlatL2")
    qd, qn, _, _, _, qm = struct.unpack("<iqqqBi", take(33))
    if qm > 1:
        take(4)
    (nc,) = struct.unpack("<Q", take(8))
    if qd != d or qn != nlist or nc != nlist * d:
        raise ValueError("quantizer shape mismatch")
    cent = np.frombuffer(take(4 * nc), dtype="<f4").reshape(nlist, d).copy()
    (dm_type,) = struct.unpack("<B", take(1))
    (dm_n,) = struct.unpack("<Q", take(8))
    take(8 * dm_n)
    if dm_type == 2:
        (hn,) = struct.unpack("<Q", take(8))
        take(16 * hn)
    if take(4) != b"ilar":
        raise ValueError("inverted lists are not ArrayInvertedLists")
    il_n, code_size = struct.unpack("<QQ", take(16))
    if il_n != nlist or code_size != 4 * d:
        raise ValueError("inverted list header mismatch")
    kind = take(4)
    (cnt,) = struct.unpack("<Q", take(8))
    raw = np.frombuffer(take(8 * cnt), dtype="<u8")
    sizes = np.zeros(nlist, dtype=np.int64)
    if kind == b"full":
        sizes[:] = raw
    elif kind == b"sprs":
        sizes[raw[0::2].astype(np.int64)] = raw[1::2].astype(np.int64)
    else:
        raise ValueError("unknown inverted list type")
    vecs, ids = [], []
    for s in sizes:
        s = int(s)
        if s:
            vecs.append(np.frombuffer(take(s * code_size), dtype="<f4").reshape(s, d).copy())
            ids.append(np.frombuffer(take(8 * s), dtype="<i8").copy())
        else:
            vecs.append(np.zeros((0, d), np.float32))
            ids.append(np.zeros(0, np.int64))
    idx = IvfFlat(d, int(nlist), int(nprobe), cent, vecs, ids, metric)
    if idx.ntotal != ntotal:
        raise ValueError("ntotal does not match the inverted lists")
    return idx


# ------------------------------------------------------------------------------------ build
def build_ivfflat(x: np.ndarray, nlist: int, nprobe: int = 1, iters: int = 8, seed: int = 0) -> IvfFlat:
    """A small IVF-Flat over x (Lloyd k-means in float64, ids 0..n-1 in insertion order), for tests.
    The reference builds with index_factory(768, f"IVF{n},Flat"), nprobe 1 (extract_index.py:58-64)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    rng = np.random.Generator(np.random.PCG64(seed))
    c = x[rng.choice(len(x), nlist, replace=False)].astype(np.float64)
    x64 = x.astype(np.float64)
    for _ in range(iters):
        a = _sqdist(x64, c).argmin(1)
        for l in range(nlist):
            m = a == l
            if m.any():
                c[l] = x64[m].mean(0)
    cent = c.astype(np.float32)
    a = _sqdist(x64, cent.astype(np.float64)).argmin(1)
    vecs = [x[a == l] for l in range(nlist)]
    ids = [np.nonzero(a == l)[0].astype(np.int64) for l in range(nlist)]
    return IvfFlat(x.shape[1], nlist, nprobe, cent, vecs, ids)


def _sqdist(x64: np.ndarray, y64: np.ndarray) -> np.ndarray:
    return ((x64[:, None, :] - y64[None, :, :]) ** 2).sum(-1)


# ------------------------------------------------------------------------------------ search
def search(idx: IvfFlat, x: np.ndarray, k: int):
    """IndexIVFFlat.search(x, k) -> (D float32 [n, k], I int64 [n, k])."""
    x64 = np.asarray(x, dtype=np.float32).astype(np.float64)
    n = x64.shape[0]
    D = np.full((n, k), np.inf, dtype=np.float32)
    I = np.full((n, k), -1, dtype=np.int64)
    cd = _sqdist(x64, idx.centroids.astype(np.float64))
    for q in range(n):
        probes = sorted(range(idx.nlist), key=lambda l: (cd[q, l], l))[: idx.nprobe]
        cand = []  # (dist, scan position, id)
        pos = 0
        for l in probes:
            v = idx.list_vecs[l].astype(np.float64)
            if len(v):
                dl = np.float32(((v - x64[q]) ** 2).sum(-1))
                for j in range(len(v)):
                    cand.append((float(dl[j]), pos, int(idx.list_ids[l][j])))
                    pos += 1
        best = sorted(cand, key=lambda c: (c[0], c[1]))[:k]      # strict-less admission, scan order
        best.sort(key=lambda c: (c[0], c[2]))                     # output ordered by (dist, id)
        for j, (dd, _, i) in enumerate(best):
            D[q, j], I[q, j] = dd, i
    return D, I


def reconstruct_n(idx: IvfFlat, i0: int, ni: int) -> np.ndarray:
    out = np.zeros((ni, idx.d), dtype=np.float32)
    for vecs, ids in zip(idx.list_vecs, idx.list_ids):
        for v, i in zip(vecs, ids):
            if i0 <= i < i0 + ni:
                out[i - i0] = v
    return out


def retrieve_speaker_embeddings(feats: np.ndarray, score: np.ndarray, ix: np.ndarray, big_npy: np.ndarray,
                                index_rate: float) -> np.ndarray:
    """rvc/infer/pipeline.py:378-388 on feats [L, D] float32 given the search result (score, ix)."""
    import torch

    with np.errstate(divide="ignore", invalid="ignore"):
        weight = np.square(1 / score)
        weight /= weight.sum(axis=1, keepdims=True)
        npy = np.sum(big_npy[ix] * np.expand_dims(weight, axis=2), axis=1)
    out = torch.from_numpy(npy).unsqueeze(0) * index_rate + (1 - index_rate) * torch.from_numpy(feats).unsqueeze(0)
    return out[0].numpy()
