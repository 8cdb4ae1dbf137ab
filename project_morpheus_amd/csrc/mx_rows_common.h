// Shared pieces of the multi-row (R >= 2) decode GEMMs: activation part split, the MFMA-tile
// epilogues (RoPE + KV append, residual, SiLU*up, penalty + argmax), write-through partials.
#pragma once
#include "mx_common.h"
#include "mx_llm_kernels.h"

namespace mx {
namespace rows {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// x[0..7] -> NPART bf16x8 fragments with x = sum of parts (to fp32 rounding for NPART 3)
template <int NPART>
__device__ __forceinline__ void split_parts(float* x, bf16x8* f) {
#pragma unroll
  for (int p = 0; p < NPART; ++p) {
    uint32_t wv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t pk = pack2_bf16(x[2 * j], x[2 * j + 1]);
      wv[j] = pk;
      if (p + 1 < NPART) {  // residual for the next part (exact in fp32)
        x[2 * j] -= bf16_lo(pk);
        x[2 * j + 1] -= bf16_hi(pk);
      }
    }
    f[p] = __builtin_bit_cast(bf16x8, make_uint4(wv[0], wv[1], wv[2], wv[3]));
  }
}

// Operands of the epilogue that do not depend on the GEMM result, loaded BEFORE the split-K
// hand-off (drain, ticket, merge loads) so that their round trips -- two dependent ones for
// RoPE (row position, then the table) -- overlap it instead of following it.
template <int MT, int NT, int EPI>
struct EpiPre {
  float y[EPI == EPI_RESID ? MT : 1][EPI == EPI_RESID ? NT : 1][4];    // RESID: Y before the add
  float cs[EPI == EPI_QKV ? MT : 1][EPI == EPI_QKV ? NT : 1][2];       // QKV: RoPE per pair
  float sn[EPI == EPI_QKV ? MT : 1][EPI == EPI_QKV ? NT : 1][2];
  int slot[EPI == EPI_QKV ? NT : 1], pos[EPI == EPI_QKV ? NT : 1];
  float ws[MT][4];                                                      // fp8 row scales
  // ARGMAX: the rows' slots, penalties, logits flags and `seen` bytes (4 per lane and tile),
  // loaded inside the last two sub-chunks of the main loop (argmax_slots / argmax_operands)
  int aslot[EPI == EPI_ARGMAX ? NT : 1];
  float apen[EPI == EPI_ARGMAX ? NT : 1];
  int akeep[EPI == EPI_ARGMAX ? NT : 1];
  uint32_t aseen[EPI == EPI_ARGMAX ? MT : 1][EPI == EPI_ARGMAX ? NT : 1];
};

// The lm_head epilogue's operands hang off the row's slot (row_slot -> seen / penalty): two
// dependent round trips that a block used to pay after its main loop (p50 9.4 us of a 41 us
// block at 8 rows, profiles/r05_rows_block_trace.log).  The slot loads go out at the top of
// sub-chunk SUB - 2, the dependent loads at the top of SUB - 1 (behind every weight load, so
// vmcnt stays exact), both under the last sub-chunks' weight latency.
template <int MT, int NT, int EPI>
__device__ __forceinline__ void argmax_slots(const GemvArgs& a, EpiPre<MT, NT, EPI>& P, int r0, int c) {
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
    P.aslot[nt % (EPI == EPI_ARGMAX ? NT : 1)] = a.row_slot[min(r0 + 16 * nt + c, a.R - 1)];
}
template <int MT, int NT, int EPI>
__device__ __forceinline__ void argmax_operands(const GemvArgs& a, EpiPre<MT, NT, EPI>& P, int n0, int g) {
  constexpr int ANT = EPI == EPI_ARGMAX ? NT : 1, AMT = EPI == EPI_ARGMAX ? MT : 1;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int slot = P.aslot[nt % ANT];
    P.apen[nt % ANT] = a.penalty[slot];
    P.akeep[nt % ANT] = a.logits && (a.logits_all || a.samp_temp[slot] > 0.f);
    const uint8_t* seen = a.seen + (size_t)slot * a.N;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int nb = n0 + 16 * mt + 4 * g;
      uint32_t v = 0;
      if ((a.N & 3) == 0) {
        v = *reinterpret_cast<const uint32_t*>(seen + min(nb, a.N - 4));
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (nb + i < a.N) v |= (uint32_t)seen[nb + i] << (8 * i);
      }
      P.aseen[mt % AMT][nt % ANT] = v;
    }
  }
}

template <int MT, int NT, int EPI>
__device__ __forceinline__ void rows_epilogue_pre(const GemvArgs& a, EpiPre<MT, NT, EPI>& P,
                                                  int n0, int r0, int c, int g) {
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int nb = n0 + 16 * mt + 4 * g;
#pragma unroll
    for (int i = 0; i < 4; ++i) P.ws[mt][i] = a.wdtype == WT_FP8 ? a.wscale[min(nb + i, a.N - 1)] : 1.f;
  }
  if (EPI == EPI_RESID) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int b = min(r0 + 16 * nt + c, a.R - 1);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int nb = min(n0 + 16 * mt + 4 * g, a.N - 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) P.y[mt % (EPI == EPI_RESID ? MT : 1)][nt % (EPI == EPI_RESID ? NT : 1)][i] =
            a.Y[(size_t)b * a.ystride + nb + i];
      }
    }
  } else if (EPI == EPI_QKV) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int b = min(r0 + 16 * nt + c, a.R - 1);
      P.slot[nt % (EPI == EPI_QKV ? NT : 1)] = a.row_slot[b];
      P.pos[nt % (EPI == EPI_QKV ? NT : 1)] = a.row_pos[b];
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          const int n = n0 + 16 * mt + 4 * g + i;
          const int p = (n & 127) >> 1;
          const size_t ix = (size_t)P.pos[nt % (EPI == EPI_QKV ? NT : 1)] * 64 + p;
          P.cs[mt % (EPI == EPI_QKV ? MT : 1)][nt % (EPI == EPI_QKV ? NT : 1)][i >> 1] = a.rope_cos[ix];
          P.sn[mt % (EPI == EPI_QKV ? MT : 1)][nt % (EPI == EPI_QKV ? NT : 1)][i >> 1] = a.rope_sin[ix];
        }
  }
}

// Epilogue of one wave's tile: lane (batch col c, group g) holds weight rows
// n0 + 16 mt + 4 g + i for batch rows r0 + 16 nt + c (MFMA C/D layout).
template <int MT, int NT, int EPI>
__device__ __forceinline__ void rows_epilogue(const GemvArgs& a, f32x4 (&acc)[MT][NT],
                                              const float (&scale)[NT], int n0, int r0, int c,
                                              int g, const EpiPre<MT, NT, EPI>& P) {
  unsigned long long best[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) best[nt] = 0ull;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int b = r0 + 16 * nt + c;
    const bool bok = b < a.R;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int nb = n0 + 16 * mt + 4 * g;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = acc[mt][nt][i] * scale[nt];
      if (a.wdtype == WT_FP8) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] *= P.ws[mt][i];
      }
      if (!bok || nb >= a.N) continue;
      if (EPI == EPI_STORE) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a.Y[(size_t)b * a.ystride + nb + i] = v[i];
      } else if (EPI == EPI_RESID) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          a.Y[(size_t)b * a.ystride + nb + i] =
              P.y[mt % (EPI == EPI_RESID ? MT : 1)][nt % (EPI == EPI_RESID ? NT : 1)][i] + v[i];
      } else if (EPI == EPI_SILU) {
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          const float gt = v[i], up = v[i + 1];
          a.Y[(size_t)b * (a.N >> 1) + ((nb + i) >> 1)] = gt / (1.0f + expf(-gt)) * up;
        }
      } else if (EPI == EPI_QKV) {
        const int slot = P.slot[nt % (EPI == EPI_QKV ? NT : 1)];
        const int pos = P.pos[nt % (EPI == EPI_QKV ? NT : 1)];
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          const int n = nb + i;
          const int hh = n >> 7, within = n & 127, p = within >> 1;
          const float x1 = v[i], x2 = v[i + 1];
          if (hh < a.heads + a.kv_heads) {
            const float cs = P.cs[mt % (EPI == EPI_QKV ? MT : 1)][nt % (EPI == EPI_QKV ? NT : 1)][i >> 1];
            const float sn = P.sn[mt % (EPI == EPI_QKV ? MT : 1)][nt % (EPI == EPI_QKV ? NT : 1)][i >> 1];
            const float o1 = x1 * cs - x2 * sn;
            const float o2 = x2 * cs + x1 * sn;
            if (hh < a.heads) {
              float* q = a.Q + ((size_t)b * a.heads + hh) * 128;
              q[p] = o1;
              q[p + 64] = o2;
            } else {
              uint16_t* kc = a.kcache +
                  ((size_t)slot * a.kv_heads + (hh - a.heads)) * a.max_pos * 128;
              kc[kv_k_off(pos, p)] = f32_to_bf16(o1);
              kc[kv_k_off(pos, p + 64)] = f32_to_bf16(o2);
            }
          } else {
            uint16_t* vc = a.vcache +
                ((size_t)slot * a.kv_heads + (hh - a.heads - a.kv_heads)) * 128 * a.max_pos;
            vc[kv_v_off(pos, within)] = f32_to_bf16(x1);
            vc[kv_v_off(pos, within + 1)] = f32_to_bf16(x2);
          }
        }
      } else if (EPI == EPI_ARGMAX) {
        constexpr int ANT = EPI == EPI_ARGMAX ? NT : 1, AMT = EPI == EPI_ARGMAX ? MT : 1;
        const float pen = P.apen[nt % ANT];
        const bool keep = P.akeep[nt % ANT];
        const uint32_t sn = P.aseen[mt % AMT][nt % ANT];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = nb + i;
          if (n >= a.N) continue;
          float x = v[i];
          if ((sn >> (8 * i)) & 0xffu) x = x > 0.f ? x / pen : x * pen;
          if (keep) a.logits[(size_t)b * a.N + n] = x;
          const unsigned long long key = argmax_key(x, (uint32_t)n);
          best[nt] = key > best[nt] ? key : best[nt];
        }
      }
    }
  }
  if (EPI == EPI_ARGMAX) {
    // one atomic per (block, batch row): the 8 waves' keys meet in LDS first (a per-wave
    // atomic put 8x the same-address device atomics on each row's key)
    __shared__ unsigned long long bred[8][16 * NT];
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      unsigned long long k = best[nt];
#pragma unroll
      for (int m = 16; m <= 32; m <<= 1) {
        const unsigned long long o = __shfl_xor(k, m, 64);
        k = o > k ? o : k;
      }
      if (g == 0) bred[w][16 * nt + c] = k;
    }
    __syncthreads();
    const int t = threadIdx.x;
    if (t < 16 * NT) {
      unsigned long long k = bred[0][t];
#pragma unroll
      for (int i = 1; i < 8; ++i) k = bred[i][t] > k ? bred[i][t] : k;
      const int b = r0 + t;
      if (b < a.R && k) atomicMax(a.best + b, k);
    }
  }
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// 16-byte write-through (sc1) store / load of a partial-tile quad (MI355X_MICROARCH.md
// "Valid forms" row 1 with 16-B accesses)
__device__ __forceinline__ void st4_wt(float* base, size_t idx, const f32x4& v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)(idx * 4), 0, 16);
}
__device__ __forceinline__ f32x4 ld4_wt(const float* base, size_t idx) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff, 0x00020000);
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(idx * 4), 0, 16));
}
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace rows
}  // namespace mx
