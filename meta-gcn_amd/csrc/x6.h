// bf16x6 product arithmetic and LDS image helpers shared by gemm.hip and
// fused.hip (internal, device code only).
//
// Every fp32 operand is split exactly-rounded into three bf16 terms
// x = hi + mid + lo (RNE at each step; x - hi and r - mid are exact,
// |mid| <= 2^-9 |x|, |lo| <= 2^-18 |x|, |x - (hi + mid + lo)| <= 2^-27 |x|)
// and the six products whose magnitude reaches 2^-18 (hh, hm, mh, mm, hl, lh)
// are summed on bf16 MFMA into one fp32 accumulator.  Dropped terms (ml, lm,
// ll) are below 2^-27 of |a b|.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mgcn {
namespace x6 {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16_t;

// bf16 pair (one VGPR) -> the two floats it holds (exact)
__device__ __forceinline__ f32x2 widen_bf16x2(uint32_t p) {
  return f32x2{__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u)};
}

// one pair of floats -> its hi / mid / lo bf16 pairs (v_cvt_pk_bf16_f32, RNE)
// Range edge: |x| >= ~3.396e38 rounds to bf16 inf, and x - inf = -inf, so
// the terms would sum to NaN where fp32 gives a finite or infinite product.
// hi and mid therefore come from x and r clamped to +-kSplitMax (the largest
// float whose RNE bf16 is finite, v_med3_f32): for finite x the split stays
// exact (hi = 0x7f7f.. then r = x - hi exactly), for x = +-inf it is
// (+-M, +-M, +-inf) -- a product with w is +-inf (NaN for w = 0), as in fp32.
constexpr float kSplitMax = 0x1.fefffep+127f;  // 0x7f7f7fff = 3.3961514e38
__device__ __forceinline__ float split_clamp(float v) {
  return __builtin_amdgcn_fmed3f(v, -kSplitMax, kSplitMax);
}
__device__ __forceinline__ void split3_pair(f32x2 x, uint32_t &hi, uint32_t &mid, uint32_t &lo) {
  const f32x2 xc = {split_clamp(x.x), split_clamp(x.y)};
  hi = __builtin_bit_cast(uint32_t, __builtin_convertvector(xc, bf16x2));
  const f32x2 r = x - widen_bf16x2(hi);  // exact (Sterbenz)
  const f32x2 rc = {split_clamp(r.x), split_clamp(r.y)};
  mid = __builtin_bit_cast(uint32_t, __builtin_convertvector(rc, bf16x2));
  lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(r - widen_bf16x2(mid), bf16x2));
}

__device__ __forceinline__ void split3_bf16(const float (&x)[8], bf16x8 &hi, bf16x8 &mid,
                                            bf16x8 &lo) {
  uint32_t h[4], m[4], l[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) split3_pair(f32x2{x[2 * p], x[2 * p + 1]}, h[p], m[p], l[p]);
  hi = __builtin_bit_cast(bf16x8, h);
  mid = __builtin_bit_cast(bf16x8, m);
  lo = __builtin_bit_cast(bf16x8, l);
}

// six-product bf16 MFMA chain on one accumulator, smallest terms first
__device__ __forceinline__ f32x16 mfma_x6(const bf16x8 &ah, const bf16x8 &am, const bf16x8 &al,
                                          const bf16x8 &bh, const bf16x8 &bm, const bf16x8 &bl,
                                          f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4_t mfma16_x6(const bf16x8 &ah, const bf16x8 &am, const bf16x8 &al,
                                            const bf16x8 &bh, const bf16x8 &bm, const bf16x8 &bl,
                                            f32x4_t c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}

// Row-major bf16 image of a [rows][128] operand term (256-B rows), 16-B chunk
// ch of row r stored at ch ^ ((r & 3) << 2 | G[(r >> 2) & 3]), G = {0, 2, 3, 1}:
// conflict-free both for ds_read_b64_tr_b16 transposed reads (the four rows
// of a read differ in bits 2-3) and for the 16x16x32 row reads (the lane
// groups of ds_read_b128 land on 16 distinct chunks).
__device__ __forceinline__ int img_swz(int row) {
  return ((row & 3) << 2) | ((0x78 >> (2 * ((row >> 2) & 3))) & 3);
}
__device__ __forceinline__ int img_off(int row, int ch) { return 256 * row + 16 * (ch ^ img_swz(row)); }

// Buffer resource over [base, base + bytes): loads past it return 0 and
// stores past it are dropped, so tails and prefetches past the end need no
// branches (a branch around a load makes hipcc wait vmcnt(0) for every load
// in flight).  Inputs are wave-uniform; readfirstlane makes that provable.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void *base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void *p = reinterpret_cast<void *>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)__builtin_amdgcn_readfirstlane(bytes),
                                           0x00020000);
}

// Packed-table rows (pack.hip's layout): the lane's four words of a row from
// the 4-bit slice `nib` of its header mask word and the 16 B read at its value
// position (its own nonzero words first): each word back where its mask bit
// says, +0.0 elsewhere -- exactly the dense row's bits
__device__ __forceinline__ float4 pk_expand(uint32_t nib, const u32x4 v) {
  const uint32_t r2 = (nib & 1u) + ((nib >> 1) & 1u);  // values below word 2
  const uint32_t r3 = r2 + ((nib >> 2) & 1u);          // ... below word 3
  const uint32_t w0 = (nib & 1u) ? v[0] : 0u;
  const uint32_t w1 = (nib & 2u) ? ((nib & 1u) ? v[1] : v[0]) : 0u;
  const uint32_t w2 = (nib & 4u) ? (r2 == 0 ? v[0] : r2 == 1 ? v[1] : v[2]) : 0u;
  const uint32_t w3 = (nib & 8u) ? (r3 == 0 ? v[0] : r3 == 1 ? v[1] : r3 == 2 ? v[2] : v[3]) : 0u;
  return make_float4(__uint_as_float(w0), __uint_as_float(w1), __uint_as_float(w2),
                     __uint_as_float(w3));
}

}  // namespace x6
}  // namespace mgcn
