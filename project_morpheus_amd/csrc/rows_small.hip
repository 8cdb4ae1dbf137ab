// Small-batch decode GEMV (2 <= R <= 8 activation rows) on the VALU, for MI355X (gfx950).
//
// The B = 1 kernel (gemv1_kernel) streams every weight row once with all of a wave's loads
// issued first; this is the same design for a handful of rows.  Each wave owns RPW whole
// weight rows (16-byte non-temporal loads, KCH per lane per row) and multiplies them with
// up to RT fp32 activation rows staged once per block in LDS, in fp32 (packed v_pk_fma_f32:
// even and odd k accumulate in the two halves, so the products are the oracle's fp32
// products and only the summation order differs).  No MFMA: at R <= 8 the MFMA tile would be
// half padding and its fp32-activation split costs three bf16 passes (mx_rows_v4.inc), while
// the VALU work per weight byte stays under the HBM time:
//   bf16, R = 8: 6.5 weights/clk/CU at 8 TB/s x 8 rows = 52 FMA/clk of the 128 (packed);
//   e4m3, R = 8: 104 of 128; LDS: RT x 4 B per weight element / RPW, <= 104 B/clk of 256.
// Blocks are persistent (one per CU when the staged rows fill the LDS): the activation rows
// are staged once per CU, then each wave walks its weight-row groups with the next group's
// loads in flight under the current group's FMAs (two register buffers, ping-pong, so the
// load counter stays exact).  With two row tiles (K = ffn: RT x K x 4 B caps RT at 4),
// blocks b and b + 8 -- the same XCD, dispatched together -- take the same weight rows, so
// the second tile's reads meet the first one's lines in that XCD's L2.
// Epilogues as gemv1_kernel: RESID (+= into the residual), SILU (gate/up pairs), QKV (RoPE,
// KV append), ARGMAX (repetition penalty, kept logits, packed-key argmax).
#include "mx_common.h"
#include "mx_llm_kernels.h"

namespace mx {
namespace small {

constexpr int WPB = 8;
constexpr int NT = WPB * 64;
constexpr int LDS_MAX = 128 * 1024;  // dynamic LDS per block (RT x K x 4 B)

__device__ __forceinline__ f32x2_t pfma(f32x2_t a, f32x2_t b, f32x2_t c) {
  return __builtin_elementwise_fma(a, b, c);
}

template <int KCH, int RPW, bool F8>
__device__ __forceinline__ void load_group(const GemvArgs& a, int g, int lane, uint4 (&w)[RPW][KCH]) {
  constexpr int KC = KCH * 64;
  const uint4* wp = reinterpret_cast<const uint4*>(a.W) + (size_t)g * RPW * KC + lane;
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int c = 0; c < KCH; ++c) w[r][c] = load_nt(wp + (size_t)r * KC + c * 64);
}

template <int KCH, int RPW, int RT, int EPI, bool F8>
__device__ __forceinline__ void process(const GemvArgs& a, const float4* xs, int g, int r0,
                                        int nr, int lane, const uint4 (&w)[RPW][KCH],
                                        unsigned long long& best) {
  constexpr int EPC = F8 ? 16 : 8;
  constexpr int PL = EPC / 4;
  constexpr int KC = KCH * 64;
  // the staged rows are loop-invariant: an opaque copy of the lane index keeps the compiler
  // from hoisting every group's LDS reads (RT x KCH x PL float4) out of the group loop
  int xl = lane;
  asm volatile("" : "+v"(xl));
  f32x2_t acc[RPW][RT];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int t = 0; t < RT; ++t) acc[r][t] = f32x2_t{0.f, 0.f};
#pragma unroll
  for (int c = 0; c < KCH; ++c) {
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      float4 xq[PL];
#pragma unroll
      for (int q = 0; q < PL; ++q) xq[q] = xs[(t * PL + q) * KC + c * 64 + xl];
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        const uint32_t wd[4] = {w[r][c].x, w[r][c].y, w[r][c].z, w[r][c].w};
        if (F8) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x2_t lo = __builtin_amdgcn_cvt_pk_f32_fp8(wd[q], false);
            const f32x2_t hi = __builtin_amdgcn_cvt_pk_f32_fp8(wd[q], true);
            acc[r][t] = pfma(lo, f32x2_t{xq[q].x, xq[q].y}, acc[r][t]);
            acc[r][t] = pfma(hi, f32x2_t{xq[q].z, xq[q].w}, acc[r][t]);
          }
        } else {
          const float4 xa[2] = {xq[0], xq[1]};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x2_t wv = {bf16_lo(wd[j]), bf16_hi(wd[j])};
            const float4 xv = xa[j >> 1];
            acc[r][t] = pfma(wv, (j & 1) ? f32x2_t{xv.z, xv.w} : f32x2_t{xv.x, xv.y}, acc[r][t]);
          }
        }
      }
    }
  }
  float s[RPW][RT];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int t = 0; t < RT; ++t) s[r][t] = wave_sum(acc[r][t].x + acc[r][t].y);
  const int n0 = g * RPW;
  if (F8) {
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const float sc = a.wscale[n0 + r];
#pragma unroll
      for (int t = 0; t < RT; ++t) s[r][t] *= sc;
    }
  }

  // every lane holds every total; lane j writes output j (pairs for SILU / QKV)
  constexpr int PAIR = (EPI == EPI_SILU || EPI == EPI_QKV) ? 2 : 1;
  constexpr int NOUT = RPW / PAIR * RT;
  static_assert(NOUT <= 64, "outputs per group exceed a wave");
  float v0 = 0.f, v1 = 0.f;
  int ri = 0, t = 0;
#pragma unroll
  for (int i = 0; i < RPW / PAIR; ++i)
#pragma unroll
    for (int tt = 0; tt < RT; ++tt)
      if (lane == i * RT + tt) {
        v0 = s[i * PAIR][tt];
        if (PAIR == 2) v1 = s[i * PAIR + 1][tt];
        ri = i * PAIR;
        t = tt;
      }
  if (lane >= NOUT || t >= nr) return;
  const int r = r0 + t, n = n0 + ri;
  if (EPI == EPI_RESID) {
    a.Y[(size_t)r * a.ystride + n] += v0;
  } else if (EPI == EPI_STORE) {
    a.Y[(size_t)r * a.N + n] = v0;
  } else if (EPI == EPI_SILU) {
    a.Y[(size_t)r * (a.N >> 1) + (n >> 1)] = v0 / (1.0f + expf(-v0)) * v1;
  } else if (EPI == EPI_QKV) {
    const int slot = a.row_slot[r], pos = a.row_pos[r];
    const int hh = n >> 7, within = n & 127, p = within >> 1;
    if (hh < a.heads + a.kv_heads) {
      const float cs = a.rope_cos[(size_t)pos * 64 + p];
      const float sn = a.rope_sin[(size_t)pos * 64 + p];
      const float o1 = v0 * cs - v1 * sn;
      const float o2 = v1 * cs + v0 * sn;
      if (hh < a.heads) {
        float* q = a.Q + ((size_t)r * a.heads + hh) * 128;
        q[p] = o1;
        q[p + 64] = o2;
      } else {
        uint16_t* k = a.kcache + ((size_t)slot * a.kv_heads + (hh - a.heads)) * a.max_pos * 128;
        k[kv_k_off(pos, p)] = f32_to_bf16(o1);
        k[kv_k_off(pos, p + 64)] = f32_to_bf16(o2);
      }
    } else {
      uint16_t* vc = a.vcache +
          ((size_t)slot * a.kv_heads + (hh - a.heads - a.kv_heads)) * 128 * a.max_pos;
      vc[kv_v_off(pos, within)] = f32_to_bf16(v0);
      vc[kv_v_off(pos, within + 1)] = f32_to_bf16(v1);
    }
  } else if (EPI == EPI_ARGMAX) {
    const int slot = a.row_slot[r];
    float v = v0;
    if (a.seen[(size_t)slot * a.N + n]) v = v > 0.f ? v / a.penalty[slot] : v * a.penalty[slot];
    if (a.logits && (a.logits_all || a.samp_temp[slot] > 0.f)) a.logits[(size_t)r * a.N + n] = v;
    const unsigned long long key = argmax_key(v, (uint32_t)n);
    best = key > best ? key : best;
  }
}

// grid: gblocks x ytiles blocks (ytiles 1 or 2, gblocks a multiple of 8 when 2)
template <int KCH, int RPW, int RT, int EPI, bool NORM, bool F8>
__global__ __launch_bounds__(NT, 1) void gemv_small_kernel(GemvArgs a, int ytiles, int gblocks) {
  constexpr int EPC = F8 ? 16 : 8;
  constexpr int PL = EPC / 4;
  constexpr int KC = KCH * 64;
  constexpr int XN = KC * PL;              // float4 per activation row
  constexpr int XPT = (XN + NT - 1) / NT;  // per thread
  extern __shared__ __attribute__((aligned(16))) float4 xs[];  // [RT][PL][KC]
  __shared__ float red[RT][WPB];
  __shared__ unsigned long long bred[RT];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int tile = 0, gb = blockIdx.x;
  if (ytiles == 2) {
    const int s = blockIdx.x >> 3;
    tile = s & 1;
    gb = (s >> 1) * 8 + (blockIdx.x & 7);
  }
  const int r0 = tile * RT, nr = min(RT, a.R - r0);
  const int G = a.N / RPW;
  const int stride = gblocks * WPB;
  int g = gb * WPB + wid;

  // 1. the first group's weight loads, then the activation rows under their latency
  uint4 w0[RPW][KCH], w1[RPW][KCH];
  load_group<KCH, RPW, F8>(a, min(g, G - 1), lane, w0);
  const float4* NW4 = reinterpret_cast<const float4*>(a.norm_w);
  float4 xv[RT][XPT], nv[XPT];
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int idx = min(tid + i * NT, XN - 1);
    if (NORM) nv[i] = NW4[idx];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const float4* X4 = reinterpret_cast<const float4*>(a.X + (size_t)(r0 + min(t, nr - 1)) * a.xstride);
      xv[t][i] = X4[idx];
    }
  }
  if (tid < RT) bred[tid] = 0ull;
  float scale[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) scale[t] = 1.f;
  if (NORM) {
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < XPT; ++i)
        if (tid + i * NT < XN)
          ss += xv[t][i].x * xv[t][i].x + xv[t][i].y * xv[t][i].y + xv[t][i].z * xv[t][i].z +
                xv[t][i].w * xv[t][i].w;
      ss = wave_sum(ss);
      if (lane == 0) red[t][wid] = ss;
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      float tot = 0.f;
#pragma unroll
      for (int i = 0; i < WPB; ++i) tot += red[t][i];
      scale[t] = 1.0f / sqrtf(tot / (float)(KC * EPC) + a.eps);
    }
  }
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int idx = tid + i * NT;
    if (idx < XN) {
      const int m = idx / PL, q = idx % PL;
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        float4 v = xv[t][i];
        if (t >= nr) v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (NORM) {
          v.x = v.x * scale[t] * nv[i].x; v.y = v.y * scale[t] * nv[i].y;
          v.z = v.z * scale[t] * nv[i].z; v.w = v.w * scale[t] * nv[i].w;
        }
        xs[(t * PL + q) * KC + m] = v;
      }
    }
  }
  __syncthreads();

  // 2. the wave's groups, the next group's loads in flight under the current FMAs
  unsigned long long best = 0ull;
  if (g < G) {
    while (true) {
      if (g + stride < G) {
        load_group<KCH, RPW, F8>(a, g + stride, lane, w1);
        process<KCH, RPW, RT, EPI, F8>(a, xs, g, r0, nr, lane, w0, best);
      } else {
        process<KCH, RPW, RT, EPI, F8>(a, xs, g, r0, nr, lane, w0, best);
        break;
      }
      g += stride;
      if (g + stride < G) {
        load_group<KCH, RPW, F8>(a, g + stride, lane, w0);
        process<KCH, RPW, RT, EPI, F8>(a, xs, g, r0, nr, lane, w1, best);
      } else {
        process<KCH, RPW, RT, EPI, F8>(a, xs, g, r0, nr, lane, w1, best);
        break;
      }
      g += stride;
    }
  }
  if (EPI == EPI_ARGMAX) {  // lane i * RT + t carried row t's best over its groups
    if (lane < RPW * RT) atomicMax(&bred[lane % RT], best);
    __syncthreads();
    if (tid < nr) atomicMax(a.best + r0 + tid, bred[tid]);
  }
}

template <int KCH, int RPW, int RT, int EPI, bool NORM, bool F8>
static hipError_t launch_t(const GemvArgs& a, hipStream_t st) {
  const size_t lds = (size_t)RT * a.K * 4;
  if (lds > LDS_MAX || a.N % RPW) return hipErrorNotSupported;
  const int ytiles = (a.R + RT - 1) / RT;
  if (ytiles > 2) return hipErrorNotSupported;
  const int G = a.N / RPW;
  int gblocks = (G + WPB - 1) / WPB;
  const int per_cu = lds <= 72 * 1024 ? 2 : 1;  // blocks the LDS lets share a CU
  const int cap = 256 * per_cu / ytiles;
  if (gblocks > cap) gblocks = cap;
  if (ytiles == 2) gblocks = (gblocks + 7) / 8 * 8;
  hipLaunchKernelGGL((gemv_small_kernel<KCH, RPW, RT, EPI, NORM, F8>), dim3(gblocks * ytiles),
                     dim3(NT), lds, st, a, ytiles, gblocks);
  return hipGetLastError();
}

template <int KCH, int RPW, int RT, int EPI, bool NORM, bool F8>
static hipError_t prep_t() {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemv_small_kernel<KCH, RPW, RT, EPI, NORM, F8>),
                             hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
}

// The instantiated shapes: Llama-3.2-3B (hidden 3072, ffn 8192).  Rows per wave keep
// 12-16 weight loads of 16 B per lane in flight: bf16 K = 3072 is 6 loads per row, e4m3 3.
#define MX_SMALL_SHAPES(X)                                                                 \
  X(6, 2, 8, EPI_QKV, true, false) X(6, 2, 4, EPI_QKV, true, false)                        \
  X(6, 2, 8, EPI_RESID, false, false) X(6, 2, 4, EPI_RESID, false, false)                  \
  X(6, 2, 8, EPI_SILU, true, false) X(6, 2, 4, EPI_SILU, true, false)                      \
  X(16, 1, 4, EPI_RESID, false, false)                                                     \
  X(6, 2, 8, EPI_ARGMAX, true, false) X(6, 2, 4, EPI_ARGMAX, true, false)                  \
  X(3, 4, 8, EPI_QKV, true, true) X(3, 4, 4, EPI_QKV, true, true)                          \
  X(3, 2, 8, EPI_RESID, false, true) X(3, 2, 4, EPI_RESID, false, true)                    \
  X(3, 4, 8, EPI_SILU, true, true) X(3, 4, 4, EPI_SILU, true, true)                        \
  X(8, 2, 4, EPI_RESID, false, true)                                                       \
  X(3, 4, 8, EPI_ARGMAX, true, true) X(3, 4, 4, EPI_ARGMAX, true, true)

}  // namespace small

hipError_t gemv_small_prepare() {
  hipError_t e = hipSuccess;
#define MX_P(KCH_, RPW_, RT_, EPI_, NORM_, F8_) \
  if (e == hipSuccess) e = small::prep_t<KCH_, RPW_, RT_, EPI_, NORM_, F8_>();
  MX_SMALL_SHAPES(MX_P)
#undef MX_P
  return e;
}

hipError_t launch_gemv_small(const GemvArgs& a, int epi, bool norm, hipStream_t st) {
  const bool f8 = a.wdtype == WT_FP8;
  const int epc = f8 ? 1024 : 512;
  if (a.R < 2 || a.R > 8 || a.K % epc) return hipErrorNotSupported;
  const int kch = a.K / epc;
  int rt = a.R <= 4 ? 4 : 8;
  if ((size_t)rt * a.K * 4 > small::LDS_MAX) rt = 4;
#define MX_L(KCH_, RPW_, RT_, EPI_, NORM_, F8_)                                         \
  if (kch == KCH_ && rt == RT_ && epi == EPI_ && norm == NORM_ && f8 == F8_)              \
    return small::launch_t<KCH_, RPW_, RT_, EPI_, NORM_, F8_>(a, st);
  MX_SMALL_SHAPES(MX_L)
#undef MX_L
  return hipErrorNotSupported;
}

}  // namespace mx
