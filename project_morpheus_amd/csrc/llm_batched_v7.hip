// Multi-row decode GEMM, generation 7 (2 <= R <= 32 rows): option "rows_kernel" = 7.
//
// Replaces the batched decode GEMMs of vLLM's engine (continuous batching of concurrent
// requests, Orpheus-TTS/orpheus_tts_pypi/orpheus_tts/engine_class.py:117) for BASELINE
// configs[2] (32 streams per GPU) and configs[4] (8 fp8 streams per GPU).
//
// Why a new generation: generations 4 and 5 split K over BLOCKS, so every launch paid an
// activation staging round trip, a write-through partial per K range, an arrival ticket and a
// last-arriver merge: 6-10 us per launch on top of the weight stream, i.e. the qkv / o-proj /
// down launches ran at 1.2-2.5 TB/s at 8-32 rows (scripts/bench_rows.py).
// Here one block owns one 16-row weight tile over the WHOLE K, split over its WPB waves:
//   * every wave streams its K slice's weight A-fragments (16 B per lane, non-temporal) and
//     the matching activation B-fragments (fp32 rows from L2, RMS-norm-weighted and split
//     into three bf16 parts in registers: fp32-exact products) with PF k-steps
//     of loads in flight, consuming each slot then refilling it (exact in-order vmcnt waits);
//   * nothing is shared between waves until the end: the WPB partial tiles and sums of
//     squares are reduced in LDS in wave order (deterministic) and wave 0 runs the epilogue
//     (RoPE + K/V append, SiLU*up, residual, penalty + argmax) in the MFMA D layout;
//   * no cross-block traffic at all: no partial workspace, no tickets.
// Activation re-reads: each block reads its K slice of every batch row once (L2-resident,
// 2 NT KB per 1 KB of weights), the price of not staging through LDS.
#include "mx_common.h"
#include "mx_llm_kernels.h"

namespace mx {
namespace v7 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// x[0..7] -> three bf16x8 fragments with x = p0 + p1 + p2 (to fp32 rounding)
__device__ __forceinline__ void split3(float* x, bf16x8* f) {
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    uint32_t wv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t pk = pack2_bf16(x[2 * j], x[2 * j + 1]);
      wv[j] = pk;
      if (p < 2) {
        x[2 * j] -= bf16_lo(pk);
        x[2 * j + 1] -= bf16_hi(pk);
      }
    }
    f[p] = __builtin_bit_cast(bf16x8, make_uint4(wv[0], wv[1], wv[2], wv[3]));
  }
}

// fp8: a lane's 16 bytes hold k = 64 P + 16 g .. +15; k-step 2P + h contracts 8 h .. 8 h + 7
__device__ __forceinline__ bf16x8 afrag8(const uint4& q, int h) {
  const uint32_t d0 = h ? q.z : q.x, d1 = h ? q.w : q.y;
  const bf16x2_t e0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d0, 1.0f, false);
  const bf16x2_t e1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d0, 1.0f, true);
  const bf16x2_t e2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d1, 1.0f, false);
  const bf16x2_t e3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d1, 1.0f, true);
  return __builtin_bit_cast(bf16x8, make_uint4(__builtin_bit_cast(uint32_t, e0),
                                               __builtin_bit_cast(uint32_t, e1),
                                               __builtin_bit_cast(uint32_t, e2),
                                               __builtin_bit_cast(uint32_t, e3)));
}

// Epilogue of the block's tile: lane (batch col c, group g) holds weight rows n0 + 4 g + i
// for batch rows r0 + 16 nt + c (MFMA C/D layout).
template <int NT, int EPI>
__device__ __forceinline__ void epilogue(const GemvArgs& a, const f32x4 (&acc)[NT],
                                         const float (&scale)[NT], int n0, int r0, int c, int g) {
  unsigned long long best[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) best[nt] = 0ull;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int b = r0 + 16 * nt + c;
    const int nb = n0 + 4 * g;
    if (b >= a.R || nb >= a.N) continue;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = acc[nt][i] * scale[nt];
      if (a.wdtype == WT_FP8) v[i] *= a.wscale[min(nb + i, a.N - 1)];
    }
    if (EPI == EPI_RESID) {
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

// One block = one 16-row weight tile x 16 NT batch rows; wave w owns K slice
// [w KS 32, (w + 1) KS 32).  G k-steps per 16-byte weight load (1 bf16, 2 fp8).
template <int NT, int EPI, bool NORM, int WPB, int KS, bool F8>
__global__ __launch_bounds__(WPB * 64) void gemm_rows7_kernel(GemvArgs a) {
  constexpr int G = F8 ? 2 : 1;                 // k-steps per load group
  constexpr int NG = KS / G;                    // load groups per wave
  constexpr int PFS = WPB == 16 ? (NORM ? 3 : 4) : 6;  // k-steps of loads in flight
  constexpr int PF = (PFS + G - 1) / G < NG ? (PFS + G - 1) / G : NG;  // groups in flight
  static_assert(KS % G == 0, "fp8: a load covers two k-steps");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16, r0 = blockIdx.y * 16 * NT;
  const int k0 = w * KS * 32;
  const int n = min(n0 + c, a.N - 1);
  const uint4* wp = F8 ? reinterpret_cast<const uint4*>(static_cast<const uint8_t*>(a.W) + (size_t)n * a.K + k0) + g
                       : reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(a.W) + (size_t)n * a.K + k0) + g;
  const float* xp[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) xp[nt] = a.X + (size_t)min(r0 + 16 * nt + c, a.R - 1) * a.xstride + k0;
  // the lane's 8 activations of k-step s (same k order as the weight fragment)
  auto xoff = [&](int s) { return F8 ? 64 * (s >> 1) + 16 * g + 8 * (s & 1) : 32 * s + 8 * g; };

  uint4 wr[PF];
  float4 xr[PF][G][NT][2];
  float4 nr[PF][G][2];
  auto issue = [&](int q, int slot) {
    wr[slot] = load_nt(wp + 4 * q);
#pragma unroll
    for (int h = 0; h < G; ++h) {
      const int o = xoff(G * q + h);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        xr[slot][h][nt][0] = *reinterpret_cast<const float4*>(xp[nt] + o);
        xr[slot][h][nt][1] = *reinterpret_cast<const float4*>(xp[nt] + o + 4);
      }
      if (NORM) {
        nr[slot][h][0] = *reinterpret_cast<const float4*>(a.norm_w + k0 + o);
        nr[slot][h][1] = *reinterpret_cast<const float4*>(a.norm_w + k0 + o + 4);
      }
    }
  };
#pragma unroll
  for (int q = 0; q < PF; ++q) issue(q, q);

  f32x4 acc[NT];
  float ssl[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    ssl[nt] = 0.f;
  }
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const int slot = q % PF;
#pragma unroll
    for (int h = 0; h < G; ++h) {
      const bf16x8 af = F8 ? afrag8(wr[slot], h) : __builtin_bit_cast(bf16x8, wr[slot]);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        float x[8] = {xr[slot][h][nt][0].x, xr[slot][h][nt][0].y, xr[slot][h][nt][0].z,
                      xr[slot][h][nt][0].w, xr[slot][h][nt][1].x, xr[slot][h][nt][1].y,
                      xr[slot][h][nt][1].z, xr[slot][h][nt][1].w};
        if (NORM) {
#pragma unroll
          for (int j = 0; j < 8; ++j) ssl[nt] = fmaf(x[j], x[j], ssl[nt]);
          x[0] *= nr[slot][h][0].x; x[1] *= nr[slot][h][0].y;
          x[2] *= nr[slot][h][0].z; x[3] *= nr[slot][h][0].w;
          x[4] *= nr[slot][h][1].x; x[5] *= nr[slot][h][1].y;
          x[6] *= nr[slot][h][1].z; x[7] *= nr[slot][h][1].w;
        }
        bf16x8 pf[3];
        split3(x, pf);
#pragma unroll
        for (int p = 0; p < 3; ++p)
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, pf[p], acc[nt], 0, 0, 0);
      }
    }
    if (q + PF < NG) issue(q + PF, slot);
    __builtin_amdgcn_sched_barrier(0);  // issue order = use order (vmcnt is in order)
  }

  // ---- block reduction in wave order (deterministic), epilogue by wave 0 ----
  __shared__ float red[WPB][NT][4][64];
  __shared__ float ssr[WPB][NT][16];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) red[w][nt][i][lane] = acc[nt][i];
    if (NORM) {
      float t = ssl[nt];
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      if (g == 0) ssr[w][nt][c] = t;
    }
  }
  __syncthreads();
  if (w != 0) return;
  f32x4 sum[NT];
  float scale[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < WPB; ++v) s += red[v][nt][i][lane];
      sum[nt][i] = s;
    }
    float ss = 0.f;
    if (NORM) {
#pragma unroll
      for (int v = 0; v < WPB; ++v) ss += ssr[v][nt][c];
    }
    scale[nt] = NORM ? 1.0f / sqrtf(ss / (float)a.K + a.eps) : 1.f;
  }
  epilogue<NT, EPI>(a, sum, scale, n0, r0, c, g);
}

template <int EPI, bool NORM, int WPB, int KS>
static hipError_t launch7(const GemvArgs& a, int nt, dim3 grid, hipStream_t st) {
  const bool f8 = a.wdtype == WT_FP8;
  const dim3 blk(WPB * 64);
  if (nt == 1) {
    if (f8) hipLaunchKernelGGL((gemm_rows7_kernel<1, EPI, NORM, WPB, KS, true>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((gemm_rows7_kernel<1, EPI, NORM, WPB, KS, false>), grid, blk, 0, st, a);
  } else {
    if (f8) hipLaunchKernelGGL((gemm_rows7_kernel<2, EPI, NORM, WPB, KS, true>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((gemm_rows7_kernel<2, EPI, NORM, WPB, KS, false>), grid, blk, 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace v7

// 2..32 rows at the Orpheus-3B projection shapes; hipErrorNotSupported otherwise (the caller
// falls back to generation 4).  Waves per block: 8, or 16 where the weight tiles are fewer
// than the CUs (o-proj, down: 192 tiles) so the K slices stay short and the chip full.
hipError_t launch_gemm_rows_v7(const GemvArgs& a, int epi, bool norm, hipStream_t st) {
  if (a.R < 2 || a.R > 32) return hipErrorNotSupported;
  const int nt = a.R <= 16 ? 1 : 2;
  const int tn = (a.N + 15) / 16;
  const int wpb = tn >= 256 ? 8 : 16;
  if (a.K % (wpb * 32)) return hipErrorNotSupported;
  const int ks = a.K / (wpb * 32);
  const dim3 grid(tn, (a.R + 16 * nt - 1) / (16 * nt));
#define MX7(EPI_, NORM_, WPB_, KS_)                                              \
  if (epi == EPI_ && norm == NORM_ && wpb == WPB_ && ks == KS_)                  \
    return v7::launch7<EPI_, NORM_, WPB_, KS_>(a, nt, grid, st);
  MX7(EPI_QKV, true, 8, 12)       // qkv  [5120 x 3072]
  MX7(EPI_RESID, false, 16, 6)    // o    [3072 x 3072]
  MX7(EPI_SILU, true, 8, 12)      // gate/up [16384 x 3072]
  MX7(EPI_RESID, false, 16, 16)   // down [3072 x 8192]
  MX7(EPI_ARGMAX, true, 8, 12)    // lm_head [V x 3072]
#undef MX7
  return hipErrorNotSupported;
}

}  // namespace mx
