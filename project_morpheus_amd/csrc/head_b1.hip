// One-row (B = 1) lm_head + repetition penalty + argmax as a persistent VALU GEMV, for
// MI355X (gfx950).  Replaces the vocabulary projection of the decode step inside vLLM /
// llama.cpp (Orpheus-TTS/orpheus_tts_pypi/orpheus_tts/engine_class.py:117,
// Morpheus_Client/tts_engine/llama_local.py:77); the penalty and greedy pick follow
// oracle/llama_ref.py.
//
// 156,940 x 3,072 weights (964 MB bf16, 482 MB e4m3) against one activation row.  Blocks
// are persistent -- as many as are resident at once on every CU -- so the RMS-normalised row
// is staged in LDS once per block, not once per weight-row group; each wave then walks its
// row groups (RPW rows x whole K, 16-byte non-temporal loads, 12 per lane) with the NEXT
// group's loads in flight under the current group's FMAs: two register buffers, ping-pong,
// so the in-order load counter stays exact.  The group's epilogue operands (seen flag, e4m3
// row scales) are loaded before that prefetch for the same reason.  fp32 products and
// accumulation (packed v_pk_fma_f32: even / odd k in the two halves), e4m3 converted in
// registers (v_cvt_pk_f32_fp8, exact).  Measured against the grid-stride gemv_kernel it
// replaces: step -24 us bf16, -45 us e4m3 (profiles/r04_ab_small_rows_v1_head_options.log).
// The same persistent design for the one-row gate/up and down projections was slower than
// gemv1_kernel (+19 / +9 us per step bf16; profiles/r04_b1_persistent_projections_not_kept.log):
// with 1.5-4 row groups per wave there is little stream to pipeline, and one block per CU
// hides less latency than gemv1's many one-shot blocks.
#include "mx_common.h"
#include "mx_llm_kernels.h"

namespace mx {
namespace head1 {

constexpr int WPB = 8;
constexpr int NT = WPB * 64;

__device__ __forceinline__ f32x2_t pfma(f32x2_t a, f32x2_t b, f32x2_t c) {
  return __builtin_elementwise_fma(a, b, c);
}

template <int KCH, int RPW>
__device__ __forceinline__ void load_group(const GemvArgs& a, int g, int lane, uint4 (&w)[RPW][KCH]) {
  constexpr int KC = KCH * 64;
  const uint4* wp = reinterpret_cast<const uint4*>(a.W) + (size_t)g * RPW * KC + lane;
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int c = 0; c < KCH; ++c) w[r][c] = load_nt(wp + (size_t)r * KC + c * 64);
}

// the operands of a group's epilogue for this lane's row (lane r * 64 / RPW holds row r)
struct EpiIn {
  float ws;
  uint8_t seen;
};

template <int RPW, bool F8>
__device__ __forceinline__ EpiIn epi_load(const GemvArgs& a, int g, int ri, int slot) {
  EpiIn e{};
  const int n = g * RPW + ri;
  if (F8) e.ws = a.wscale[n];
  e.seen = a.seen[(size_t)slot * a.N + n];
  return e;
}

template <int KCH, int RPW, bool F8>
__device__ __forceinline__ void process(const GemvArgs& a, const float4* xs, int g, int lane,
                                        const uint4 (&w)[RPW][KCH], int ri, bool on, float pen,
                                        bool keep, const EpiIn& e, unsigned long long& best) {
  constexpr int EPC = F8 ? 16 : 8;
  constexpr int PL = EPC / 4;
  constexpr int KC = KCH * 64;
  // the staged row is loop-invariant: an opaque copy of the lane index keeps the compiler
  // from hoisting every group's LDS reads (KCH x PL float4) out of the group loop
  int xl = lane;
  asm volatile("" : "+v"(xl));
  f32x2_t acc[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) acc[r] = f32x2_t{0.f, 0.f};
#pragma unroll
  for (int c = 0; c < KCH; ++c) {
    float4 xq[PL];
#pragma unroll
    for (int q = 0; q < PL; ++q) xq[q] = xs[q * KC + c * 64 + xl];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const uint32_t wd[4] = {w[r][c].x, w[r][c].y, w[r][c].z, w[r][c].w};
      if (F8) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x2_t lo = __builtin_amdgcn_cvt_pk_f32_fp8(wd[q], false);
          const f32x2_t hi = __builtin_amdgcn_cvt_pk_f32_fp8(wd[q], true);
          acc[r] = pfma(lo, f32x2_t{xq[q].x, xq[q].y}, acc[r]);
          acc[r] = pfma(hi, f32x2_t{xq[q].z, xq[q].w}, acc[r]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x2_t wv = {bf16_lo(wd[j]), bf16_hi(wd[j])};
          const float4 xv = xq[j >> 1];
          acc[r] = pfma(wv, (j & 1) ? f32x2_t{xv.z, xv.w} : f32x2_t{xv.x, xv.y}, acc[r]);
        }
      }
    }
  }
  // transposing butterfly: each exchange halves the values a lane carries (RPW - 1 +
  // log2(64 / RPW) shuffles for RPW totals); afterwards lanes [r * 64 / RPW, (r + 1) * 64 /
  // RPW) hold row r's total
  float v[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) v[r] = acc[r].x + acc[r].y;
#pragma unroll
  for (int m = 32, cnt = RPW; m >= 1; m >>= 1) {
    if (cnt > 1) {
      const bool up = lane & m;
      cnt >>= 1;
#pragma unroll
      for (int i = 0; i < RPW / 2; ++i) {
        if (i < cnt) {
          const float send = up ? v[i] : v[i + cnt];
          const float kept = up ? v[i + cnt] : v[i];
          v[i] = kept + __shfl_xor(send, m, MX_WAVE);
        }
      }
    } else {
      v[0] += __shfl_xor(v[0], m, MX_WAVE);
    }
  }
  if (!on) return;
  const int n = g * RPW + ri;
  float y = F8 ? v[0] * e.ws : v[0];
  if (e.seen) y = y > 0.f ? y / pen : y * pen;
  if (keep) a.logits[n] = y;
  const unsigned long long key = argmax_key(y, (uint32_t)n);
  best = key > best ? key : best;
}

template <int KCH, int RPW, bool F8>
__global__ __launch_bounds__(NT, 1) void head_b1_kernel(GemvArgs a) {
  constexpr int EPC = F8 ? 16 : 8;
  constexpr int PL = EPC / 4;
  constexpr int KC = KCH * 64;
  constexpr int XN = KC * PL;              // float4 of the activation row
  constexpr int XPT = (XN + NT - 1) / NT;  // per thread
  static_assert(RPW <= 64 && (RPW & (RPW - 1)) == 0, "RPW must be a power of two");
  __shared__ __attribute__((aligned(16))) float4 xs[PL * KC];  // plane q at [q * KC + m]
  __shared__ float red[WPB];
  __shared__ unsigned long long bred;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int G = a.N / RPW;
  const int stride = gridDim.x * WPB;
  int g = blockIdx.x * WPB + wid;
  // this lane's row within a group, and the slot's constants
  const int ri = lane / (64 / RPW);
  const bool on = lane % (64 / RPW) == 0;
  const int slot = a.row_slot[0];
  const float pen = a.penalty[slot];
  const bool keep = a.logits && (a.logits_all || a.samp_temp[slot] > 0.f);

  // 1. the first group's weight loads, then the activation row under their latency
  uint4 w0[RPW][KCH], w1[RPW][KCH];
  load_group<KCH, RPW>(a, min(g, G - 1), lane, w0);
  const float4* X4 = reinterpret_cast<const float4*>(a.X);
  const float4* NW4 = reinterpret_cast<const float4*>(a.norm_w);
  float4 xv[XPT], nv[XPT];
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int idx = min(tid + i * NT, XN - 1);
    xv[i] = X4[idx];
    nv[i] = NW4[idx];
  }
  if (tid == 0) bred = 0ull;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < XPT; ++i)
    if (tid + i * NT < XN)
      ss += xv[i].x * xv[i].x + xv[i].y * xv[i].y + xv[i].z * xv[i].z + xv[i].w * xv[i].w;
  ss = wave_sum(ss);
  if (lane == 0) red[wid] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int i = 0; i < WPB; ++i) tot += red[i];
  const float scale = 1.0f / sqrtf(tot / (float)(KC * EPC) + a.eps);
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int idx = tid + i * NT;
    if (idx < XN) {
      float4 v = xv[i];
      v.x = v.x * scale * nv[i].x; v.y = v.y * scale * nv[i].y;
      v.z = v.z * scale * nv[i].z; v.w = v.w * scale * nv[i].w;
      xs[(idx % PL) * KC + idx / PL] = v;
    }
  }
  __syncthreads();

  // 2. the wave's groups, the next group's loads in flight under the current FMAs
  unsigned long long best = 0ull;
  if (g < G) {
    while (true) {
      if (g + stride < G) {
        const EpiIn e = epi_load<RPW, F8>(a, g, ri, slot);
        load_group<KCH, RPW>(a, g + stride, lane, w1);
        process<KCH, RPW, F8>(a, xs, g, lane, w0, ri, on, pen, keep, e, best);
      } else {
        const EpiIn e = epi_load<RPW, F8>(a, g, ri, slot);
        process<KCH, RPW, F8>(a, xs, g, lane, w0, ri, on, pen, keep, e, best);
        break;
      }
      g += stride;
      if (g + stride < G) {
        const EpiIn e = epi_load<RPW, F8>(a, g, ri, slot);
        load_group<KCH, RPW>(a, g + stride, lane, w0);
        process<KCH, RPW, F8>(a, xs, g, lane, w1, ri, on, pen, keep, e, best);
      } else {
        const EpiIn e = epi_load<RPW, F8>(a, g, ri, slot);
        process<KCH, RPW, F8>(a, xs, g, lane, w1, ri, on, pen, keep, e, best);
        break;
      }
      g += stride;
    }
  }
  if (on) atomicMax(&bred, best);
  __syncthreads();
  if (tid == 0) atomicMax(a.best, bred);
}

template <int KCH, int RPW, bool F8>
static hipError_t launch_t(const GemvArgs& a, hipStream_t st) {
  if (a.N % RPW) return hipErrorNotSupported;
  const int G = a.N / RPW;
  int blocks = (G + WPB - 1) / WPB;
  // persistent: no more blocks than are resident at once (registers, LDS), on every CU.  The
  // CU count and the occupancy answer are cached per device (a process may drive several
  // GPUs; each value is idempotent, so concurrent first calls write the same number)
  constexpr int MAXDEV = 64;
  static int cus_of[MAXDEV] = {}, per_cu_of[MAXDEV] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAXDEV) return hipErrorInvalidDevice;
  if (!cus_of[dev]) {
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      return hipErrorInvalidDevice;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, reinterpret_cast<const void*>(&head_b1_kernel<KCH, RPW, F8>), NT, 0) != hipSuccess ||
        per_cu < 1)
      return hipErrorInvalidConfiguration;
    per_cu_of[dev] = per_cu;
    cus_of[dev] = cus;
  }
  const int cus = cus_of[dev], per_cu = per_cu_of[dev];
  if (blocks > cus * per_cu) blocks = cus * per_cu;
  hipLaunchKernelGGL((head_b1_kernel<KCH, RPW, F8>), dim3(blocks), dim3(NT), 0, st, a);
  return hipGetLastError();
}

}  // namespace head1

// K = 3072 (Llama-3.2-3B hidden): bf16 2 rows per wave (12 loads of 16 B per lane), e4m3 4.
hipError_t launch_head_b1(const GemvArgs& a, hipStream_t st) {
  if (a.R != 1 || a.K != 3072) return hipErrorNotSupported;
  return a.wdtype == WT_FP8 ? head1::launch_t<3, 4, true>(a, st) : head1::launch_t<6, 2, false>(a, st);
}

}  // namespace mx
