// FAISS IndexIVFFlat ingestion and the device-side search/retrieval entry points.
//
// Replaces faiss.read_index + index.reconstruct_n(0, ntotal) (rvc/infer/pipeline.py:430-434;
// rvc_mlx/infer/pipeline_mlx.py:267-278) and index.search / _retrieve_speaker_embeddings
// (pipeline.py:378-388). The byte layout follows faiss 1.7.4 (faiss-cpu==1.7.4, requirements.txt:15)
// impl/index_write.cpp for IndexIVFFlat; the reference's own parser of the format is
// Demos/iOS/.../FAISSIndexReader.swift:50-121. Parsing happens once on the host, then the
// centroids, the lists (vectors in list order), their ids and an id -> slot map go to HBM.
#include <cstring>

#include "runtime.h"

namespace rvcx {

namespace {

struct Reader {
  const uint8_t* p;
  int64_t n, at = 0;
  void need(int64_t k) {
    if (k < 0 || at + k > n) throw Error(RVCX_E_INVALID, "faiss index: truncated at byte " + std::to_string(at));
  }
  template <class T>
  T get() {
    need(sizeof(T));
    T v;
    std::memcpy(&v, p + at, sizeof(T));
    at += sizeof(T);
    return v;
  }
  std::string fourcc() {
    need(4);
    std::string s(reinterpret_cast<const char*>(p + at), 4);
    at += 4;
    return s;
  }
  const uint8_t* take(int64_t k) {
    need(k);
    const uint8_t* r = p + at;
    at += k;
    return r;
  }
  // `count` elements of `elem` bytes, with the byte count checked against the bytes left (no wrap-around:
  // counts come from the file and are untrusted)
  const uint8_t* take_n(uint64_t count, uint64_t elem) {
    const uint64_t left = (uint64_t)(n - at);
    if (elem == 0 || count > left / elem)
      throw Error(RVCX_E_INVALID, "faiss index: truncated at byte " + std::to_string(at) + " (count " +
                                      std::to_string(count) + " x " + std::to_string(elem) + " B)");
    return take((int64_t)(count * elem));
  }
};

struct Header {
  int32_t d;
  int64_t ntotal;
  int32_t metric;
};

// write_index_header: d i32, ntotal i64, dummy i64 x2, is_trained u8, metric i32 [, metric_arg f32]
Header read_header(Reader& r) {
  Header h;
  h.d = r.get<int32_t>();
  h.ntotal = r.get<int64_t>();
  (void)r.get<int64_t>();
  (void)r.get<int64_t>();
  (void)r.get<uint8_t>();
  h.metric = r.get<int32_t>();
  if (h.metric > 1) (void)r.get<float>();
  return h;
}

template <class T>
void upload(DevBuf& b, const T* host, size_t count) {
  const size_t bytes = std::max<size_t>(count * sizeof(T), 16);
  if (hipMalloc(&b.p, bytes) != hipSuccess) {
    (void)hipGetLastError();
    throw Error(RVCX_E_OOM, "faiss index: device allocation failed");
  }
  b.bytes = bytes;
  if (count) RVCX_HIP(hipMemcpy(b.p, host, count * sizeof(T), hipMemcpyHostToDevice));
}

}  // namespace

ParsedIvf parse_ivf(const uint8_t* bytes, int64_t nbytes) {
  ParsedIvf P;
  Reader r{bytes, nbytes};
  const std::string magic = r.fourcc();
  if (magic != "IwFl") throw Error(RVCX_E_INVALID, "faiss index: fourcc '" + magic + "' is not IndexIVFFlat (IwFl)");
  const Header h = read_header(r);
  if (h.metric != 1) throw Error(RVCX_E_INVALID, "faiss index: only METRIC_L2 is supported");
  if (h.d <= 0 || h.d % 64 != 0 || h.d > 4096)
    throw Error(RVCX_E_INVALID, "faiss index: dimension must be a positive multiple of 64 (got " +
                                    std::to_string(h.d) + ")");
  const uint64_t nlist = r.get<uint64_t>();
  const uint64_t nprobe = r.get<uint64_t>();
  if (nlist == 0 || nlist > (1u << 24)) throw Error(RVCX_E_INVALID, "faiss index: bad nlist");
  // coarse quantizer: IndexFlatL2
  const std::string qmagic = r.fourcc();
  if (qmagic != "IxF2") throw Error(RVCX_E_INVALID, "faiss index: coarse quantizer '" + qmagic + "' is not IndexFlatL2");
  const Header qh = read_header(r);
  const uint64_t ncent = r.get<uint64_t>();
  if (qh.d != h.d || (uint64_t)qh.ntotal != nlist || ncent != nlist * (uint64_t)h.d)
    throw Error(RVCX_E_INVALID, "faiss index: quantizer shape does not match the IVF header");
  const float* cent = reinterpret_cast<const float*>(r.take_n(ncent, 4));
  P.cent.assign(cent, cent + ncent);
  // direct map: type u8, array (u64 count + i64s), [hashtable pairs]
  const uint8_t dm_type = r.get<uint8_t>();
  const uint64_t dm_n = r.get<uint64_t>();
  r.take_n(dm_n, 8);
  if (dm_type == 2) r.take_n(r.get<uint64_t>(), 16);
  // inverted lists: ArrayInvertedLists
  const std::string il = r.fourcc();
  if (il != "ilar") throw Error(RVCX_E_INVALID, "faiss index: inverted lists '" + il + "' are not ArrayInvertedLists");
  const uint64_t il_n = r.get<uint64_t>();
  const uint64_t code_size = r.get<uint64_t>();
  if (il_n != nlist || code_size != 4 * (uint64_t)h.d)
    throw Error(RVCX_E_INVALID, "faiss index: inverted list header does not match the IVF header");
  if (h.ntotal <= 0 || h.ntotal >= (int64_t(1) << 31))
    throw Error(RVCX_E_INVALID, "faiss index: ntotal " + std::to_string(h.ntotal) + " out of range");
  const std::string kind = r.fourcc();
  const uint64_t cnt = r.get<uint64_t>();
  const uint8_t* raw_bytes = r.take_n(cnt, 8);  // checked before anything is allocated from cnt
  std::vector<uint64_t> raw(cnt);
  if (cnt) std::memcpy(raw.data(), raw_bytes, cnt * 8);
  std::vector<uint64_t> sizes(nlist, 0);
  if (kind == "full") {
    if (cnt != nlist) throw Error(RVCX_E_INVALID, "faiss index: list size count mismatch");
    sizes = raw;
  } else if (kind == "sprs") {
    if (cnt % 2) throw Error(RVCX_E_INVALID, "faiss index: odd sparse size vector");
    for (uint64_t i = 0; i < cnt; i += 2) {
      if (raw[i] >= nlist) throw Error(RVCX_E_INVALID, "faiss index: sparse list id out of range");
      sizes[raw[i]] = raw[i + 1];
    }
  } else {
    throw Error(RVCX_E_INVALID, "faiss index: unknown list size encoding '" + kind + "'");
  }
  // list sizes are untrusted: bound each by ntotal and the running sum step by step (no wrap-around)
  std::vector<long long>& off = P.off;
  off.assign(nlist + 1, 0);
  const uint64_t ntot_u = (uint64_t)h.ntotal;
  uint64_t acc = 0;
  for (uint64_t l = 0; l < nlist; ++l) {
    if (sizes[l] > ntot_u || acc + sizes[l] > ntot_u)
      throw Error(RVCX_E_INVALID, "faiss index: inverted list " + std::to_string(l) + " size exceeds ntotal");
    acc += sizes[l];
    off[l + 1] = (long long)acc;
  }
  const long long ntotal = off[nlist];
  if (ntotal != h.ntotal) throw Error(RVCX_E_INVALID, "faiss index: ntotal does not match the inverted lists");
  std::vector<float>& vecs = P.vecs;
  std::vector<long long>& ids = P.ids;
  vecs.resize((size_t)ntotal * h.d);
  ids.resize((size_t)ntotal);
  for (uint64_t l = 0; l < nlist; ++l) {
    const uint64_t s = sizes[l];
    if (!s) continue;
    std::memcpy(vecs.data() + (size_t)off[l] * h.d, r.take_n(s, code_size), s * code_size);
    std::memcpy(ids.data() + off[l], r.take_n(s, 8), s * 8);
  }
  // reconstruct_n(0, ntotal) semantics: row id <- the stored vector with that id. RVC indexes hold ids
  // 0..ntotal-1 (sequential add, extract_index.py:66-68); anything else is refused.
  std::vector<int>& slot = P.slot;
  slot.assign((size_t)ntotal, -1);
  for (long long i = 0; i < ntotal; ++i) {
    const long long id = ids[i];
    if (id < 0 || id >= ntotal || slot[id] >= 0)
      throw Error(RVCX_E_INVALID, "faiss index: ids are not a permutation of 0..ntotal-1");
    slot[id] = (int)i;
  }
  P.d = h.d;
  P.nlist = (long long)nlist;
  P.ntotal = ntotal;
  P.nprobe = (int)std::max<uint64_t>(1, std::min<uint64_t>(nprobe, nlist));
  return P;
}

void index_load(Ctx& c, const uint8_t* bytes, int64_t nbytes) {
  const ParsedIvf P = parse_ivf(bytes, nbytes);
  auto ix = std::make_unique<IvfIndex>();
  RVCX_HIP(hipSetDevice(c.device));
  upload(ix->cent, P.cent.data(), P.cent.size());
  upload(ix->vecs, P.vecs.data(), P.vecs.size());
  upload(ix->off, P.off.data(), P.off.size());
  upload(ix->ids, P.ids.data(), P.ids.size());
  upload(ix->slot_of_id, P.slot.data(), P.slot.size());
  IvfView& v = ix->view;
  v.d = P.d;
  v.nlist = P.nlist;
  v.ntotal = P.ntotal;
  v.nprobe = P.nprobe;
  v.cent = static_cast<const float*>(ix->cent.p);
  v.vecs = static_cast<const float*>(ix->vecs.p);
  v.off = static_cast<const long long*>(ix->off.p);
  v.ids = static_cast<const long long*>(ix->ids.p);
  v.slot_of_id = static_cast<const int*>(ix->slot_of_id.p);
  c.ivf = std::move(ix);
}

static const IvfView& loaded(Ctx& c) {
  if (!c.ivf) throw Error(RVCX_E_STATE, "no feature index loaded");
  return c.ivf->view;
}

void index_search(Ctx& c, const float* x, int64_t n, int k, float* dist, int64_t* ids, hipStream_t s) {
  const IvfView& v = loaded(c);
  if (k < 1 || k > IVF_MAX_K) throw Error(RVCX_E_INVALID, "index search: k must be in 1..16");
  if (n <= 0) return;
  float* ws = c.buf<float>("ivf.ws", ivf_ws_floats(n, v.nlist, v.nprobe), s);
  check(ivf_search(v, x, n, k, dist, reinterpret_cast<long long*>(ids), 0.f, 0.f, nullptr, ws, s), "ivf_search");
}

void index_retrieve(Ctx& c, const float* feats, int64_t L, int d, double index_rate, float* out, hipStream_t s) {
  const IvfView& v = loaded(c);
  if (d != v.d)
    throw Error(RVCX_E_SHAPE, "index dimension " + std::to_string(v.d) + " != feature width " + std::to_string(d));
  if (L <= 0) return;
  float* ws = c.buf<float>("ivf.ws", ivf_ws_floats(L, v.nlist, v.nprobe), s);
  // torch: npy * index_rate + (1 - index_rate) * feats, python scalars cast to float32 (1 - r in double)
  check(ivf_search(v, feats, L, 8, nullptr, nullptr, (float)index_rate, (float)(1.0 - index_rate), out, ws, s),
        "ivf_retrieve");
}

void index_reconstruct_n(Ctx& c, int64_t i0, int64_t ni, float* out, hipStream_t s) {
  const IvfView& v = loaded(c);
  if (i0 < 0 || ni < 0 || i0 + ni > v.ntotal) throw Error(RVCX_E_INVALID, "reconstruct_n: range out of bounds");
  // ids are a permutation of 0..ntotal-1: row r is the stored vector at slot_of_id[i0 + r]
  if (ni == 0) return;
  check(gather_rows(v.vecs, v.d, v.slot_of_id + i0, out, (int)ni, v.d, s), "reconstruct_n");
}

}  // namespace rvcx
