// Multi-row decode / prefill projections on bf16 MFMA (gfx950) — the B = 2..64 path.
//
// Replaces the batched decode GEMMs of vLLM's engine (continuous batching of concurrent
// requests, Orpheus-TTS/orpheus_tts_pypi/orpheus_tts/engine_class.py:117) for BASELINE
// configs 3 and 5 (B = 32 / 8 streams per GPU).  Every weight byte is still streamed ONCE
// per step (the step stays HBM-bound up to B ~ 300), so the kernel is a weight-streaming
// skinny GEMM:
//   * D[16 weight rows][16 batch rows] tiles of v_mfma_f32_16x16x32_bf16; A = weights
//     straight from HBM (16 B per lane, non-temporal), B = activation rows.
//   * Precision contract: activations are fp32.  They enter the MFMA as
//     NPART bf16 parts x = x0 + x1 (+ x2) split in registers, so products are the fp32
//     products of the oracle (bf16 weights are exact) up to summation order.
//   * RMSNorm is folded: y = (W (x . nw)) * rsqrt(mean(x^2) + eps); the sum of squares is
//     accumulated from the same activation loads.
//   * A block of WK waves splits K; partial tiles are summed in LDS in a fixed order
//     (deterministic), then wave 0 runs the epilogue (RoPE + KV append, SiLU*up, residual,
//     penalty + argmax) with the same lane layout as the MFMA result.
#include "mx_common.h"
#include "mx_llm_kernels.h"

namespace mx {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

// x[0..7] -> NPART bf16x8 fragments with x = sum of parts (to fp32 rounding for NPART 3)
template <int NPART>
__device__ __forceinline__ void split_parts(float* x, bf16x8* f) {
#pragma unroll
  for (int p = 0; p < NPART; ++p) {
    uint32_t wv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = x[2 * j], b = x[2 * j + 1];
      const uint16_t ha = f32_to_bf16(a), hb = f32_to_bf16(b);
      wv[j] = (uint32_t)ha | ((uint32_t)hb << 16);
      x[2 * j] = a - bf16_to_f32(ha);
      x[2 * j + 1] = b - bf16_to_f32(hb);
    }
    f[p] = __builtin_bit_cast(bf16x8, make_uint4(wv[0], wv[1], wv[2], wv[3]));
  }
}

template <int MT, int NT, int NPART, int EPI, bool NORM, int WK>
__global__ __launch_bounds__(WK * 64) void gemm_rows_kernel(GemvArgs a) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * (16 * MT);
  const int r0 = blockIdx.y * (16 * NT);
  const int Kw = a.K / WK;
  const int kbeg = w * Kw;

  const uint4* wp[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int n = min(n0 + 16 * mt + c, a.N - 1);
    wp[mt] = reinterpret_cast<const uint4*>(a.W + (size_t)n * a.K) + g;
  }
  const float* xp[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int b = min(r0 + 16 * nt + c, a.R - 1);
    xp[nt] = a.X + (size_t)b * a.xstride + 8 * g;
  }
  const float* nwp = a.norm_w + 8 * g;

  f32x4 acc[MT][NT];
  float ss[NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) ss[nt] = 0.f;

#pragma unroll 2
  for (int k = kbeg; k < kbeg + Kw; k += 32) {
    uint4 wv[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) wv[mt] = load_nt(wp[mt] + (k >> 3));
    float4 xl[NT], xh[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      xl[nt] = *reinterpret_cast<const float4*>(xp[nt] + k);
      xh[nt] = *reinterpret_cast<const float4*>(xp[nt] + k + 4);
    }
    float4 nl, nh;
    if (NORM) {
      nl = *reinterpret_cast<const float4*>(nwp + k);
      nh = *reinterpret_cast<const float4*>(nwp + k + 4);
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      float x[8] = {xl[nt].x, xl[nt].y, xl[nt].z, xl[nt].w, xh[nt].x, xh[nt].y, xh[nt].z, xh[nt].w};
      if (NORM) {
#pragma unroll
        for (int j = 0; j < 8; ++j) ss[nt] = fmaf(x[j], x[j], ss[nt]);
        x[0] *= nl.x; x[1] *= nl.y; x[2] *= nl.z; x[3] *= nl.w;
        x[4] *= nh.x; x[5] *= nh.y; x[6] *= nh.z; x[7] *= nh.w;
      }
      bf16x8 pf[NPART];
      split_parts<NPART>(x, pf);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16x8 wb = __builtin_bit_cast(bf16x8, wv[mt]);
#pragma unroll
        for (int p = 0; p < NPART; ++p)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb, pf[p], acc[mt][nt], 0, 0, 0);
      }
    }
  }

  // ---- deterministic K-split reduction: waves 1.. -> LDS, wave 0 sums in wave order ----
  __shared__ f32x4 red[WK - 1][MT * NT][64];
  __shared__ float ssr[WK - 1][NT][64];
  if (w > 0) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) red[w - 1][mt * NT + nt][lane] = acc[mt][nt];
    if (NORM) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) ssr[w - 1][nt][lane] = ss[nt];
    }
  }
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int ww = 0; ww < WK - 1; ++ww) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] += red[ww][mt * NT + nt][lane];
    if (NORM) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) ss[nt] += ssr[ww][nt][lane];
    }
  }
  float scale[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    scale[nt] = 1.f;
    if (NORM) {
      float t = ss[nt];
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      scale[nt] = 1.0f / sqrtf(t / (float)a.K + a.eps);
    }
  }

  // ---- epilogue: lane (batch col c, group g) holds weight rows 16 mt + 4 g + i ----------
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
      if (!bok || nb >= a.N) continue;
      if (EPI == EPI_STORE) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a.Y[(size_t)b * a.ystride + nb + i] = v[i];
      } else if (EPI == EPI_RESID) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a.Y[(size_t)b * a.ystride + nb + i] += v[i];
      } else if (EPI == EPI_SILU) {
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          const float gt = v[i], up = v[i + 1];
          a.Y[(size_t)b * (a.N >> 1) + ((nb + i) >> 1)] = gt / (1.0f + expf(-gt)) * up;
        }
      } else if (EPI == EPI_QKV) {
        const int slot = a.row_slot[b], pos = a.row_pos[b];
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          const int n = nb + i;
          const int hh = n >> 7, within = n & 127, p = within >> 1;
          const float x1 = v[i], x2 = v[i + 1];
          if (hh < a.heads + a.kv_heads) {
            const float cs = a.rope_cos[(size_t)pos * 64 + p];
            const float sn = a.rope_sin[(size_t)pos * 64 + p];
            const float o1 = x1 * cs - x2 * sn;
            const float o2 = x2 * cs + x1 * sn;
            if (hh < a.heads) {
              float* q = a.Q + ((size_t)b * a.heads + hh) * 128;
              q[p] = o1;
              q[p + 64] = o2;
            } else {
              uint16_t* kc = a.kcache +
                  (((size_t)slot * a.kv_heads + (hh - a.heads)) * a.max_pos + pos) * 128;
              kc[p] = f32_to_bf16(o1);
              kc[p + 64] = f32_to_bf16(o2);
            }
          } else {
            uint16_t* vc = a.vcache +
                ((size_t)slot * a.kv_heads + (hh - a.heads - a.kv_heads)) * 128 * a.max_pos;
            vc[(size_t)within * a.max_pos + pos] = f32_to_bf16(x1);
            vc[(size_t)(within + 1) * a.max_pos + pos] = f32_to_bf16(x2);
          }
        }
      } else if (EPI == EPI_ARGMAX) {
        const int slot = a.row_slot[b];
        const uint8_t* seen = a.seen + (size_t)slot * a.N;
        const float pen = a.penalty[0];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = nb + i;
          if (n >= a.N) continue;
          float x = v[i];
          if (seen[n]) x = x > 0.f ? x / pen : x * pen;
          if (a.logits) a.logits[(size_t)b * a.N + n] = x;
          const unsigned long long key = argmax_key(x, (uint32_t)n);
          best[nt] = key > best[nt] ? key : best[nt];
        }
      }
    }
  }
  if (EPI == EPI_ARGMAX) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      unsigned long long k = best[nt];
#pragma unroll
      for (int m = 16; m <= 32; m <<= 1) {
        const unsigned long long o = __shfl_xor(k, m, 64);
        k = o > k ? o : k;
      }
      const int b = r0 + 16 * nt + c;
      if (g == 0 && b < a.R && k) atomicMax(a.best + b, k);
    }
  }
}

template <int MT, int NT, int EPI, bool NORM>
static hipError_t launch_rows_t(const GemvArgs& a, hipStream_t st) {
  constexpr int WK = 8;
  const dim3 grid((a.N + 16 * MT - 1) / (16 * MT), (a.R + 16 * NT - 1) / (16 * NT));
  hipLaunchKernelGGL((gemm_rows_kernel<MT, NT, 3, EPI, NORM, WK>), grid, dim3(WK * 64), 0, st, a);
  return hipGetLastError();
}

// R >= 2 rows.  Returns hipErrorNotSupported for shapes the kernel does not cover.
hipError_t launch_gemm_rows(const GemvArgs& a, int epi, bool norm, hipStream_t st) {
  if (a.K % (32 * 8) || a.R < 1) return hipErrorNotSupported;
  const int nt = a.R <= 16 ? 1 : a.R <= 32 ? 2 : 4;
  // 64-row tiles carry half the weight rows per wave (register budget: no spills)
#define MX_R(MT_, EPI_, NORM_)                                                            \
  if (epi == EPI_ && norm == NORM_) {                                                     \
    if (nt == 1) return launch_rows_t<MT_, 1, EPI_, NORM_>(a, st);                        \
    if (nt == 2) return launch_rows_t<MT_, 2, EPI_, NORM_>(a, st);                        \
    return launch_rows_t<(MT_ > 1 ? MT_ / 2 : 1), 4, EPI_, NORM_>(a, st);                 \
  }
  MX_R(2, EPI_QKV, true)
  MX_R(1, EPI_RESID, false)
  MX_R(2, EPI_SILU, true)
  MX_R(4, EPI_ARGMAX, true)
  MX_R(2, EPI_STORE, false)
  MX_R(2, EPI_STORE, true)
#undef MX_R
  return hipErrorNotSupported;
}

}  // namespace mx
