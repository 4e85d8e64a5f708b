// fp32 operands as three exact bf16 planes (x = x0 + x1 + x2) for the MFMA conv kernels (conv_emu.hip: B staged
// through LDS; conv_wsb.hip: B pre-split in HBM). Shared row layout of one 32-channel chunk:
// [hi | mid | lo] x 32 channels + 16 B pad = ERS bytes (16 consecutive rows hit 16 distinct 4-bank groups).
#pragma once
#include "conv_common.h"

namespace rvcx {
namespace splitbf16 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int EK = 32;               // contraction channels per chunk = two K16 MFMA steps
constexpr int EC4 = EK / 4;          // float4 groups per row
constexpr int PLANE = EK * 2;        // bytes of one bf16 plane of one row
constexpr int ERS = 3 * PLANE + 16;  // LDS row stride in bytes

__device__ __forceinline__ unsigned pk_bf16(float x, float y) {
  const bf16x2 h = __builtin_convertvector((f32x2){x, y}, bf16x2);  // v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(unsigned, h);
}
__device__ __forceinline__ float lo_f(unsigned p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float hi_f(unsigned p) { return __uint_as_float(p & 0xffff0000u); }

// 4 consecutive channels (c4..c4+3) of one LDS row, split into the three planes
__device__ __forceinline__ void put_split4(char* row, int c4, f32x4 v) {
  uint2 h, m, l;
  h.x = pk_bf16(v[0], v[1]);
  h.y = pk_bf16(v[2], v[3]);
  float r0 = v[0] - lo_f(h.x), r1 = v[1] - hi_f(h.x), r2 = v[2] - lo_f(h.y), r3 = v[3] - hi_f(h.y);
  m.x = pk_bf16(r0, r1);
  m.y = pk_bf16(r2, r3);
  r0 -= lo_f(m.x);
  r1 -= hi_f(m.x);
  r2 -= lo_f(m.y);
  r3 -= hi_f(m.y);
  l.x = pk_bf16(r0, r1);
  l.y = pk_bf16(r2, r3);
  *reinterpret_cast<uint2*>(row + c4 * 2) = h;
  *reinterpret_cast<uint2*>(row + PLANE + c4 * 2) = m;
  *reinterpret_cast<uint2*>(row + 2 * PLANE + c4 * 2) = l;
}

// one channel (KN-layout operands are transposed on their way into LDS)
__device__ __forceinline__ void put_split1(char* row, int c, float v) {
  const unsigned h = pk_bf16(v, 0.f);
  const float r = v - lo_f(h);
  const unsigned m = pk_bf16(r, 0.f);
  const unsigned l = pk_bf16(r - lo_f(m), 0.f);
  *reinterpret_cast<unsigned short*>(row + c * 2) = (unsigned short)h;
  *reinterpret_cast<unsigned short*>(row + PLANE + c * 2) = (unsigned short)m;
  *reinterpret_cast<unsigned short*>(row + 2 * PLANE + c * 2) = (unsigned short)l;
}

// ---- fp32 operands as two fp16 planes (x = h + 2^-11 l): h = f16(x), l = f16((x - h) * 2^11). Each plane carries 11
// significand bits, so x is held to 2^-22 |x| (the residual scaled by 2^11 stays a normal fp16 wherever h is one); the
// MFMA sums h*h' in one accumulator and h*l' + l*h' in a second, combined as acc + 2^-11 acc2 (the dropped l*l' term is
// below 2^-22 |x y|). Three MFMA products per step instead of the bf16 split's six.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
constexpr int ERS_H = 2 * PLANE + 16;  // LDS row stride of the two-plane image: 36 dwords, 16 rows -> 16 bank groups
constexpr float H16_LO = 2048.f, H16_LO_INV = 1.f / 2048.f;
// activations are split at this scale (weights at a power of two chosen per tensor, conv_wsb.hip k_wmax_scale):
// inputs up to 2^20 stay finite fp16
constexpr float H16_XS = 1.f / 16.f;

__device__ __forceinline__ unsigned pk_f16(float x, float y) {
  const f16x2 h = __builtin_convertvector((f32x2){x, y}, f16x2);  // RNE
  return __builtin_bit_cast(unsigned, h);
}
__device__ __forceinline__ float f16lo_f(unsigned p) { return (float)__builtin_bit_cast(f16x2, p)[0]; }
__device__ __forceinline__ float f16hi_f(unsigned p) { return (float)__builtin_bit_cast(f16x2, p)[1]; }

// Per-tensor weight scale of the fp16 images: max |w| is gathered by every workgroup of the build grid into one word
// (non-negative floats order as their bit patterns: atomicMax on the bits, one per wave), then the split kernel turns
// it into the power of two sc with max |w| sc in [128, 256) (small weights stay normal fp16).
__device__ __forceinline__ void absmax_wave_publish(float m, unsigned* dst) {
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) atomicMax(dst, __float_as_uint(m));
}
__device__ __forceinline__ float h16_weight_scale(unsigned mbits) {
  const float m = __uint_as_float(mbits);
  int e = 0;
  (void)frexpf(m, &e);  // m = f 2^e, f in [0.5, 1)
  return m > 0.f ? ldexpf(1.f, 8 - e) : 1.f;
}

// 4 consecutive channels of one LDS row as the two fp16 planes (NPL = 1: the hi plane alone, the reduced-precision mode)
template <int NPL>
__device__ __forceinline__ void put_h16x4(char* row, int c4, f32x4 v) {
  uint2 h;
  h.x = pk_f16(v[0], v[1]);
  h.y = pk_f16(v[2], v[3]);
  *reinterpret_cast<uint2*>(row + c4 * 2) = h;
  if constexpr (NPL > 1) {
    uint2 l;
    l.x = pk_f16((v[0] - f16lo_f(h.x)) * H16_LO, (v[1] - f16hi_f(h.x)) * H16_LO);
    l.y = pk_f16((v[2] - f16lo_f(h.y)) * H16_LO, (v[3] - f16hi_f(h.y)) * H16_LO);
    *reinterpret_cast<uint2*>(row + PLANE + c4 * 2) = l;
  }
}

// row order of a store: the 8 rows written by one 64-lane store instruction (8 lanes per 32-channel row) go as
// 0,4,1,5,2,6,3,7 so each 16-lane group writes two rows 4 apart: 4 x 52 dwords = 16 mod 32 banks, disjoint halves
__device__ __forceinline__ int store_row(int w) { return (w & ~7) | (((w & 7) >> 1) + 4 * (w & 1)); }


}  // namespace splitbf16
}  // namespace rvcx
