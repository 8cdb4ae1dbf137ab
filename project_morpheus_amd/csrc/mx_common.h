// Shared device helpers for the MI355X (gfx950) Orpheus hot path.
// Wave64 everywhere: lane = threadIdx.x & 63; reductions are 64-lane butterflies.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MX_WAVE 64

namespace mx {

__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

// fp32 -> bf16 round-to-nearest-even (matches torch .bfloat16() for finite values).
// A plain cast lowers to the hardware v_cvt_pk_bf16_f32 on gfx950 (MI355X_MICROARCH.md
// "Correctness boundaries": it also keeps NaNs NaN, unlike the integer-rounding trick).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
// two fp32 -> packed bf16x2 (lo in bits 0-15), one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack2_bf16(float lo, float hi) {
  const bf16x2_t v = __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t);
  return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, MX_WAVE);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, MX_WAVE));
  return v;
}
// reduce within aligned groups of G lanes (G power of two <= 64)
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int m = G / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, MX_WAVE);
  return v;
}

// dot of 8 bf16 weights (one 16-byte load) with 8 fp32 activations
__device__ __forceinline__ float dot8(const uint4 w, const float4 a, const float4 b, float acc) {
  acc = fmaf(bf16_lo(w.x), a.x, acc);
  acc = fmaf(bf16_hi(w.x), a.y, acc);
  acc = fmaf(bf16_lo(w.y), a.z, acc);
  acc = fmaf(bf16_hi(w.y), a.w, acc);
  acc = fmaf(bf16_lo(w.z), b.x, acc);
  acc = fmaf(bf16_hi(w.z), b.y, acc);
  acc = fmaf(bf16_lo(w.w), b.z, acc);
  acc = fmaf(bf16_hi(w.w), b.w, acc);
  return acc;
}

// Order-preserving float key for a 64-bit atomicMax argmax: high word = value,
// low word = ~index so that equal values resolve to the SMALLEST index (torch.argmax).
__device__ __forceinline__ unsigned long long argmax_key(float v, uint32_t idx) {
  uint32_t b = __float_as_uint(v);
  b = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  return ((unsigned long long)b << 32) | (unsigned long long)(~idx);
}
__device__ __forceinline__ uint32_t argmax_index(unsigned long long key) {
  return ~(uint32_t)(key & 0xffffffffull);
}

// Streaming (read-once) 16-byte load of weights: non-temporal hint.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 load_nt(const uint4* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// KV cache layout.  One (slot, kv head) holds max_pos x 128 bf16 of K and the
// same of V, stored in chunks of 32 positions (4,096 elements), each chunk in the order the
// attention MFMAs consume it, so that every wave load instruction reads 1 KB contiguous
// (lane-linear 16-byte pieces) instead of 16 rows x 64 B:
//   K chunk [T 2][st 4][g 4][rr 16][8 dims]: MFMA row rr of tile T is position
//     8 (rr >> 2) + 4 T + (rr & 3) of the chunk, k-step st / group g hold dims 32 st + 8 g + j;
//   V chunk [t 8][g 4][c 16][8 positions]: dim 16 t + c, positions 8 g .. 8 g + 7.
__device__ __forceinline__ size_t kv_k_off(int p, int d) {
  const int q = p & 31;
  const int rr = 4 * (q >> 3) + (q & 3), T = (q >> 2) & 1;
  return (size_t)(p >> 5) * 4096 + (size_t)((((T * 4 + (d >> 5)) * 64 + ((d >> 3) & 3) * 16 + rr) << 3) + (d & 7));
}
__device__ __forceinline__ size_t kv_v_off(int p, int d) {
  const int q = p & 31;
  return (size_t)(p >> 5) * 4096 + (size_t)(((((d >> 4) * 4 + (q >> 3)) * 16 + (d & 15)) << 3) + (q & 7));
}

}  // namespace mx
