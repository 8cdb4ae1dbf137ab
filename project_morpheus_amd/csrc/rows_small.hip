// Small-batch decode GEMV (2 <= R <= 8 activation rows; R = 1 for the lm_head) on the VALU,
// for MI355X (gfx950).
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

template <int EPI>
constexpr int pair_of() { return (EPI == EPI_SILU || EPI == EPI_QKV) ? 2 : 1; }

// Lane j < NOUT = RPW / PAIR x RT owns output j of every group: weight row (pair) ri,
// activation row t of the tile; its row constants are loaded once.
struct LaneOut {
  int ri, t, r;  // r: the activation row (clamped into the tile for idle lanes)
  bool on;
  int slot, pos;
  float pen;
  bool keep;
};

// Epilogue operands of one group, loaded BEFORE the next group's weight loads: the load
// counter is in order, so a load issued after them would make the epilogue wait for the
// whole prefetch.  Every address is valid (clamped), so no load is predicated.
struct EpiIn {
  float y, ws0, ws1, cs, sn;
  uint8_t seen;
};

template <int RPW, int EPI, bool F8>
__device__ __forceinline__ EpiIn epi_load(const GemvArgs& a, int g, const LaneOut& L) {
  EpiIn e{};
  const int n = g * RPW + L.ri;
  if (EPI == EPI_RESID) e.y = a.Y[(size_t)L.r * a.ystride + n];
  if (F8) {
    e.ws0 = a.wscale[n];
    if (pair_of<EPI>() == 2) e.ws1 = a.wscale[n + 1];
  }
  if (EPI == EPI_QKV) {
    const int p = (n & 127) >> 1;
    e.cs = a.rope_cos[(size_t)L.pos * 64 + p];
    e.sn = a.rope_sin[(size_t)L.pos * 64 + p];
  }
  if (EPI == EPI_ARGMAX) e.seen = a.seen[(size_t)L.slot * a.N + n];
  return e;
}

template <int KCH, int RPW, int RT, int EPI, bool F8>
__device__ __forceinline__ void process(const GemvArgs& a, const float4* xs, int g, int lane,
                                        const uint4 (&w)[RPW][KCH], const LaneOut& L,
                                        const EpiIn& e, unsigned long long& best) {
  constexpr int EPC = F8 ? 16 : 8;
  constexpr int PL = EPC / 4;
  constexpr int KC = KCH * 64;
  constexpr int PAIR = pair_of<EPI>();
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
  // transposing butterfly: each exchange halves the values a lane carries, so RPW x RT
  // totals cost NV - 1 + log2(64 / NV) shuffles instead of 6 NV; afterwards the 64 / NV
  // consecutive lanes from SPAN * f hold total f = r * RT + t
  constexpr int NV = RPW * RT;
  float v[NV];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int t = 0; t < RT; ++t) v[r * RT + t] = acc[r][t].x + acc[r][t].y;
#pragma unroll
  for (int m = 32, cnt = NV; m >= 1; m >>= 1) {
    if (cnt > 1) {
      const bool up = lane & m;
      cnt >>= 1;
#pragma unroll
      for (int i = 0; i < NV / 2; ++i) {
        if (i < cnt) {
          const float send = up ? v[i] : v[i + cnt];
          const float keep = up ? v[i + cnt] : v[i];
          v[i] = keep + __shfl_xor(send, m, MX_WAVE);
        }
      }
    } else {
      v[0] += __shfl_xor(v[0], m, MX_WAVE);
    }
  }
  constexpr int SPAN = 64 / NV;
  float v0 = v[0], v1 = 0.f;
  if (PAIR == 2) v1 = __shfl(v0, (lane + RT * SPAN) & 63, MX_WAVE);  // total (r + 1, t)
  if (F8) {
    v0 *= e.ws0;
    v1 *= e.ws1;
  }
  if (!L.on) return;
  const int r = L.r, n = g * RPW + L.ri;
  if (EPI == EPI_RESID) {
    a.Y[(size_t)r * a.ystride + n] = e.y + v0;
  } else if (EPI == EPI_STORE) {
    a.Y[(size_t)r * a.N + n] = v0;
  } else if (EPI == EPI_SILU) {
    a.Y[(size_t)r * (a.N >> 1) + (n >> 1)] = v0 / (1.0f + expf(-v0)) * v1;
  } else if (EPI == EPI_QKV) {
    const int hh = n >> 7, within = n & 127, p = within >> 1;
    if (hh < a.heads + a.kv_heads) {
      const float o1 = v0 * e.cs - v1 * e.sn;
      const float o2 = v1 * e.cs + v0 * e.sn;
      if (hh < a.heads) {
        float* q = a.Q + ((size_t)r * a.heads + hh) * 128;
        q[p] = o1;
        q[p + 64] = o2;
      } else {
        uint16_t* k = a.kcache + ((size_t)L.slot * a.kv_heads + (hh - a.heads)) * a.max_pos * 128;
        k[kv_k_off(L.pos, p)] = f32_to_bf16(o1);
        k[kv_k_off(L.pos, p + 64)] = f32_to_bf16(o2);
      }
    } else {
      uint16_t* vc = a.vcache +
          ((size_t)L.slot * a.kv_heads + (hh - a.heads - a.kv_heads)) * 128 * a.max_pos;
      vc[kv_v_off(L.pos, within)] = f32_to_bf16(v0);
      vc[kv_v_off(L.pos, within + 1)] = f32_to_bf16(v1);
    }
  } else if (EPI == EPI_ARGMAX) {
    float v = v0;
    if (e.seen) v = v > 0.f ? v / L.pen : v * L.pen;
    if (L.keep) a.logits[(size_t)r * a.N + n] = v;
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

  constexpr int NV = RPW * RT;
  static_assert(NV <= 64 && (NV & (NV - 1)) == 0, "RPW x RT must be a power of two <= 64");
  LaneOut L{};
  {
    const int f = lane / (64 / NV);  // the total this lane holds after the butterfly
    L.ri = f / RT;
    L.t = f % RT;
    L.on = lane % (64 / NV) == 0 && L.ri % pair_of<EPI>() == 0 && L.t < nr;
    L.r = r0 + min(L.t, nr - 1);
    if (EPI == EPI_QKV || EPI == EPI_ARGMAX) L.slot = a.row_slot[L.r];
    if (EPI == EPI_QKV) L.pos = a.row_pos[L.r];
    if (EPI == EPI_ARGMAX) {
      L.pen = a.penalty[L.slot];
      L.keep = a.logits && (a.logits_all || a.samp_temp[L.slot] > 0.f);
    }
  }
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

  // 2. the wave's groups, the next group's loads in flight under the current FMAs (each
  // group's epilogue operands are loaded before that prefetch)
  unsigned long long best = 0ull;
  if (g < G) {
    while (true) {
      if (g + stride < G) {
        const EpiIn e = epi_load<RPW, EPI, F8>(a, g, L);
        load_group<KCH, RPW, F8>(a, g + stride, lane, w1);
        process<KCH, RPW, RT, EPI, F8>(a, xs, g, lane, w0, L, e, best);
      } else {
        const EpiIn e = epi_load<RPW, EPI, F8>(a, g, L);
        process<KCH, RPW, RT, EPI, F8>(a, xs, g, lane, w0, L, e, best);
        break;
      }
      g += stride;
      if (g + stride < G) {
        const EpiIn e = epi_load<RPW, EPI, F8>(a, g, L);
        load_group<KCH, RPW, F8>(a, g + stride, lane, w0);
        process<KCH, RPW, RT, EPI, F8>(a, xs, g, lane, w1, L, e, best);
      } else {
        const EpiIn e = epi_load<RPW, EPI, F8>(a, g, L);
        process<KCH, RPW, RT, EPI, F8>(a, xs, g, lane, w1, L, e, best);
        break;
      }
      g += stride;
    }
  }
  if (EPI == EPI_ARGMAX) {  // an "on" lane carried its row t's best over its groups
    if (L.on) atomicMax(&bred[L.t], best);
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
  // persistent: no more blocks than are resident at once (registers, LDS), on every CU
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      return hipErrorInvalidDevice;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per_cu, reinterpret_cast<const void*>(&gemv_small_kernel<KCH, RPW, RT, EPI, NORM, F8>),
          NT, lds) != hipSuccess || per_cu < 1)
    return hipErrorInvalidConfiguration;
  const int cap = cus * per_cu / ytiles;
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
  X(6, 2, 1, EPI_ARGMAX, true, false) X(3, 4, 1, EPI_ARGMAX, true, true)                   \
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
  if (a.R < 1 || a.R > 8 || a.K % epc) return hipErrorNotSupported;
  const int kch = a.K / epc;
  int rt = a.R == 1 ? 1 : a.R <= 4 ? 4 : 8;
  if ((size_t)rt * a.K * 4 > small::LDS_MAX) rt = 4;
#define MX_L(KCH_, RPW_, RT_, EPI_, NORM_, F8_)                                         \
  if (kch == KCH_ && rt == RT_ && epi == EPI_ && norm == NORM_ && f8 == F8_)              \
    return small::launch_t<KCH_, RPW_, RT_, EPI_, NORM_, F8_>(a, st);
  MX_SMALL_SHAPES(MX_L)
#undef MX_L
  return hipErrorNotSupported;
}

}  // namespace mx
