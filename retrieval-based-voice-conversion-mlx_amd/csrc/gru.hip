// RMVPE BiGRU recurrence (RMVPE.py:543-564: nn.GRU(384, 256, bidirectional, batch_first)).
//
// The input projection gi = x W_ih^T + b_ih (both directions, [T][1536]) is one MFMA GEMM
// launched before this kernel. What is left is 2 x T dependent steps of h' = GRUCell(gi_t, h)
// with W_hh = 768 x 256 fp32 (786 KB per direction: more than one CU's VGPRs + LDS can hold).
//
// Design: 4 working workgroups per sequence = 2 directions x 2 halves of the hidden units (partners on one XCD). A workgroup
// owns 128 hidden units = 384 rows of W_hh (its units' r, z, n rows) and keeps ALL of them in VGPRs (768 threads, 128
// weights each, as packed pairs for v_pk_fma_f32; layout below). Per step every wave first takes the dot with its own
// half of h (local), then waits for the partner values it needs and takes the second dot, so the partner-dependent
// work after the hand-off is spread over all 12 waves (3 per SIMD).
// Hand-off: 8-byte {tag = step + 1, value} granules stored with agent-scope relaxed atomics (the
// data IS the flag; MI355X_MICROARCH.md, hand-off "R2"), double-buffered by step parity; each
// wave polls the 64 granules its lanes need (one per lane) with agent-scope relaxed loads (sc1,
// L1-bypassing). Spins are bounded: on timeout *status is set and the kernel exits (no hang); the
// runtime reports it as an error (RVCX_E_HIP, "gru: partner hand-off timed out") at its next check.
// Tags continue across launches (gru_bidir), so the granule buffer needs no zeroing between them.
//
// Cell arithmetic follows ATen GRUCell: r = sig(hg_r + ig_r), z = sig(hg_z + ig_z),
// n = tanh(ig_n + hg_n * r), h' = (h - n) * z + n, with hg = W_hh h + b_hh.
#include <cstdlib>

#include "rvcx_kernels.h"

namespace rvcx {

namespace {
constexpr int H = 256;
constexpr int UNITS = 128;  // hidden units per workgroup
constexpr int ROWS = 3 * UNITS;
constexpr int NT = 2 * ROWS;  // 768 threads
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr unsigned SPIN_LIMIT = 1u << 22;  // default bound on the polls of one hand-off (RVCX_GRU_SPIN_LIMIT overrides)

// gate activations on the hardware exp/rcp (v_exp_f32, v_rcp_f32): the libm expf/tanhf and IEEE divisions
// were 0.14 us of every 1.5 us step (and __frcp_rn, used until round 6, is still the IEEE division sequence: three
// dependent 10-instruction chains per step on the hand-off path); error <= ~2e-6 relative on sigmoid, ~1e-7 absolute
// on tanh
__device__ __forceinline__ float rcp_hw(float v) { return __builtin_amdgcn_rcpf(v); }
__device__ __forceinline__ float sigm(float v) { return rcp_hw(1.f + __expf(-v)); }
__device__ __forceinline__ float tanh_g(float v) { return 1.f - 2.f * rcp_hw(1.f + __expf(2.f * v)); }
}  // namespace

// Gate-major layout (round 5): a wave owns ONE gate of all 128 units of its workgroup and a 32-column group of each
// half of h: wave w = (gate g = w / 4, column group cg = w % 4), lane l holds rows (g, unit l) and (g, unit 64 + l)
// over own columns [32 cg, 32 cg + 32) and the same 32 partner columns (128 weights per thread). Every h value a wave
// reads feeds two rows, so the per-step LDS broadcast reads of h are 16 ds_read_b128 per wave (32 in rounds 2-4's
// row-major waves, which were the larger part of the math phase: 1.405 -> 1.24 us per step), the partner work after
// the hand-off is 32 packed FMAs on every wave, and the gate threads sum four column-group partials.
// MODE (measurement aid, RVCX_GRU_MODE; bench_gru): 0 the recurrence; 1 the hand-off alone (no W_hh dots: the partner
// poll, the gates and the publish of every step); 2 the math alone (the dots and gates, no poll: partner values read
// as published by nobody)
template <int MODE>
__global__ __launch_bounds__(NT, 1) void k_gru_bidir_g(const float* __restrict__ gi, const float* whh_f,
                                                       const float* bhh_f, const float* whh_b, const float* bhh_b,
                                                       int T, float* out, unsigned long long* xchg,
                                                       unsigned* status, unsigned spin_limit, unsigned tag0) {
  constexpr int CG = 32;  // columns of each half per wave
  __shared__ __attribute__((aligned(16))) float h_own[UNITS];
  __shared__ __attribute__((aligned(16))) float h_pw[NT / 64][CG];  // per-wave copy of its partner columns
  __shared__ float part[4][ROWS];
  __shared__ float bias_h[ROWS];
  __shared__ float igl[3][UNITS];  // this step's input gates (staged from registers after the poll)
  __shared__ int abort_flag;

  const int w = blockIdx.x & 15;
  if ((w & 7) > 1) return;  // partners w and w + 8 share an XCD under round-robin placement (speed only)
  const int d = w & 1;       // direction
  const int q = w >> 3;      // half
  const int seq = blockIdx.x >> 4;
  gi += (long long)seq * T * 6 * H;
  out += (long long)seq * T * 2 * H;
  xchg += (long long)seq * 4 * 2 * UNITS;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = wave >> 2, cg = wave & 3;  // gate, column group (wave-uniform)
  const float* whh = d ? whh_b : whh_f;
  const float* bhh = d ? bhh_b : bhh_f;
  unsigned long long* mine = xchg + ((long long)(d * 2 + q) * 2) * UNITS;
  unsigned long long* theirs = xchg + ((long long)(d * 2 + (1 - q)) * 2) * UNITS;

  // rows (g, unit lane) and (g, unit 64 + lane) of W_hh (global row g * H + q * UNITS + unit)
  const int grow0 = g * H + q * UNITS + lane, grow1 = grow0 + 64;
  const int own0 = q * UNITS + cg * CG, par0 = (1 - q) * UNITS + cg * CG;
  f32x2 wo0[CG / 2], wo1[CG / 2], wp0[CG / 2], wp1[CG / 2];
#pragma unroll
  for (int k = 0; k < CG; k += 4) {
    float4 v = *reinterpret_cast<const float4*>(&whh[(long long)grow0 * H + own0 + k]);
    wo0[k / 2] = f32x2{v.x, v.y};
    wo0[k / 2 + 1] = f32x2{v.z, v.w};
    v = *reinterpret_cast<const float4*>(&whh[(long long)grow1 * H + own0 + k]);
    wo1[k / 2] = f32x2{v.x, v.y};
    wo1[k / 2 + 1] = f32x2{v.z, v.w};
    v = *reinterpret_cast<const float4*>(&whh[(long long)grow0 * H + par0 + k]);
    wp0[k / 2] = f32x2{v.x, v.y};
    wp0[k / 2 + 1] = f32x2{v.z, v.w};
    v = *reinterpret_cast<const float4*>(&whh[(long long)grow1 * H + par0 + k]);
    wp1[k / 2] = f32x2{v.x, v.y};
    wp1[k / 2 + 1] = f32x2{v.z, v.w};
  }
  if (tid < UNITS) h_own[tid] = 0.f;
  if (tid == 0) abort_flag = 0;
  const int gunit = q * UNITS + tid;
  if (tid < ROWS) bias_h[tid] = bhh[(tid / UNITS) * H + q * UNITS + tid % UNITS];
  __syncthreads();

  // two rows' dots over CG columns of h (broadcast float4 reads: each value feeds both rows)
#define RVCX_GRU_DOT2(W0, W1, HV, O0, O1)                                            \
  do {                                                                               \
    f32x2 a0_ = {0.f, 0.f}, a1_ = {0.f, 0.f}, b0_ = {0.f, 0.f}, b1_ = {0.f, 0.f};    \
    _Pragma("unroll") for (int k = 0; k < CG; k += 4) {                              \
      const float4 x_ = *reinterpret_cast<const float4*>(&(HV)[k]);                  \
      const f32x2 xl_ = f32x2{x_.x, x_.y}, xh_ = f32x2{x_.z, x_.w};                  \
      a0_ = __builtin_elementwise_fma(W0[k / 2], xl_, a0_);                          \
      a1_ = __builtin_elementwise_fma(W0[k / 2 + 1], xh_, a1_);                      \
      b0_ = __builtin_elementwise_fma(W1[k / 2], xl_, b0_);                          \
      b1_ = __builtin_elementwise_fma(W1[k / 2 + 1], xh_, b1_);                      \
    }                                                                                \
    O0 = (a0_.x + a1_.x) + (a0_.y + a1_.y);                                          \
    O1 = (b0_.x + b1_.x) + (b0_.y + b1_.y);                                          \
  } while (0)

  auto load_ig = [&](int s, float (&ig)[3]) {
    const int t = d ? (T - 1 - s) : s;
    const int o = t * (6 * H) + d * 3 * H + gunit;
    ig[0] = gi[o];
    ig[1] = gi[o + H];
    ig[2] = gi[o + 2 * H];
  };
  // The input gates of step s + 1 are loaded right after step s's poll into `ig` (the gate threads), and staged to
  // LDS right after step s + 1's poll, whose wait (vmcnt(0): the poll load is the newest) has retired them a whole step
  // after their issue. Loaded at the top of their own step (round 5), their latency sat on the hand-off path: the
  // poll's wait retires them in order, a few hundred ns after the issue.
  float ig[3] = {0.f, 0.f, 0.f};
  if (tid < UNITS) load_ig(0, ig);
  const int oofs = d * H + gunit;
  // retire every load issued so far (the W_hh registers) before the loop: otherwise the wait-count pass, merging the
  // loop's entry with its back edge, keeps the weights "pending" and waits for them inside the loop with counts that
  // also retire the input-gate loads just issued (vmcnt(0) in the partner dots)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt / lgkmcnt untouched (gfx9 encoding)
  for (int s = 0; s < T; ++s) {
    const int t = d ? (T - 1 - s) : s;
    float own0 = 0.f, own1 = 0.f, par0v = 0.f, par1v = 0.f;
    if constexpr (MODE != 1) RVCX_GRU_DOT2(wo0, wo1, h_own + cg * CG, own0, own1);
    asm volatile("" : "+v"(own0), "+v"(own1));  // finish the own-column dots before polling
    {
      float* hp = h_pw[wave];
      if (MODE != 2 && s > 0) {
        const unsigned epoch = tag0 + (unsigned)s;
        // lanes l and l + 32 poll the same granule (32 partner values per wave)
        const unsigned long long* slot = theirs + ((s - 1) & 1) * UNITS + cg * CG + (lane & (CG - 1));
        unsigned long long gv = 0;
#pragma nounroll
        for (unsigned spins = 0;; ++spins) {
          if (spins >= spin_limit) {
            abort_flag = 1;
            break;
          }
          gv = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((unsigned)(gv >> 32) == epoch) break;
          __builtin_amdgcn_s_sleep(1);
        }
        if (lane < CG) hp[lane] = __uint_as_float((unsigned)gv);
      } else if (lane < CG) {
        hp[lane] = 0.f;
      }
      if (tid < UNITS) {
        igl[0][tid] = ig[0];
        igl[1][tid] = ig[1];
        igl[2][tid] = ig[2];
        if (s + 1 < T) load_ig(s + 1, ig);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if constexpr (MODE != 1) RVCX_GRU_DOT2(wp0, wp1, hp, par0v, par1v);
    }
    part[cg][g * UNITS + lane] = own0 + par0v;
    part[cg][g * UNITS + 64 + lane] = own1 + par1v;
    __syncthreads();
    if (abort_flag) {
      if (tid == 0) __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    if (tid < UNITS) {
      const float hr = ((part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid])) + bias_h[tid];
      const float hz = ((part[0][UNITS + tid] + part[1][UNITS + tid]) + (part[2][UNITS + tid] + part[3][UNITS + tid])) +
                       bias_h[UNITS + tid];
      const float hn = ((part[0][2 * UNITS + tid] + part[1][2 * UNITS + tid]) +
                        (part[2][2 * UNITS + tid] + part[3][2 * UNITS + tid])) +
                       bias_h[2 * UNITS + tid];
      const float rr = sigm(hr + igl[0][tid]);
      const float zz = sigm(hz + igl[1][tid]);
      const float nn = tanh_g(igl[2][tid] + hn * rr);
      const float hprev = h_own[tid];
      const float hnew = (hprev - nn) * zz + nn;
      h_own[tid] = hnew;
      out[t * (2 * H) + oofs] = hnew;  // 32-bit offset on the scalar base (a 64-bit lane pointer spilled)
      const unsigned long long gg =
          ((unsigned long long)(tag0 + (unsigned)(s + 1)) << 32) | (unsigned long long)__float_as_uint(hnew);
      __hip_atomic_store(&mine[(s & 1) * UNITS + tid], gg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
#undef RVCX_GRU_DOT2
}

hipError_t gru_bidir(const float* gi, const float* whh_f, const float* bhh_f, const float* whh_b,
                     const float* bhh_b, int T, float* out, unsigned long long* xchg, unsigned* status,
                     unsigned* next_tag, hipStream_t s, int B) {
  // the two halves of a direction spin on each other: all 4B working workgroups (1 per CU) must be co-resident;
  // the 12B idle ones exit at once
  if (B < 1 || B > 16 || !next_tag) return hipErrorInvalidValue;
  // granule tags run on across launches on the same buffer (tag0 advances by T + 1 per launch; *next_tag is the
  // caller's counter OF THIS BUFFER, starting at 0 for a zeroed one), so whatever the buffer holds from an earlier
  // launch never matches a tag this launch waits for and no per-launch zeroing is needed. When the 32-bit tag space
  // would wrap, the buffer is zeroed and the count restarts at 1: no stale tag can equal a new one.
  unsigned tag0 = *next_tag;
  if ((unsigned long long)tag0 + (unsigned)T + 1 >= (1ull << 32) || tag0 == 0) {
    hipError_t e = hipMemsetAsync(xchg, 0, sizeof(unsigned long long) * gru_xchg_words(B), s);
    if (e != hipSuccess) return e;
    tag0 = 1;
  }
  *next_tag = tag0 + (unsigned)T + 1;
  // fault-injection hook (RVCX_EXPERIMENTAL=1 RVCX_GRU_SPIN_LIMIT=0 forces the loud timeout path; read per call so a
  // test can set and clear it)
  unsigned spin = SPIN_LIMIT;
  if (const char* e = rvcx_knob("RVCX_GRU_SPIN_LIMIT")) spin = (unsigned)std::strtoul(e, nullptr, 10);
  static const int mode = [] {
    const char* e = rvcx_knob("RVCX_GRU_MODE");
    return e ? std::atoi(e) : 0;
  }();
  auto kern = mode == 1 ? k_gru_bidir_g<1> : (mode == 2 ? k_gru_bidir_g<2> : k_gru_bidir_g<0>);
  hipLaunchKernelGGL(kern, dim3(16 * B), dim3(NT), 0, s, gi, whh_f, bhh_f, whh_b, bhh_b, T, out, xchg, status, spin,
                     tag0);
  return hipGetLastError();
}

}  // namespace rvcx
