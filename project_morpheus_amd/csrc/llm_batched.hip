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
//   * K is split into a few ranges whose partial tiles are merged in a fixed order
//     (deterministic) by the last arriving wave, which runs the epilogue (RoPE + KV append,
//     SiLU*up, residual, penalty + argmax) in the MFMA result's lane layout.
#include "mx_common.h"
#include "mx_llm_kernels.h"

#include <algorithm>
#include <type_traits>

namespace mx {

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

// Epilogue of one wave's tile: lane (batch col c, group g) holds weight rows
// n0 + 16 mt + 4 g + i for batch rows r0 + 16 nt + c (MFMA C/D layout).
template <int MT, int NT, int EPI>
__device__ __forceinline__ void rows_epilogue(const GemvArgs& a, f32x4 (&acc)[MT][NT],
                                              const float (&scale)[NT], int n0, int r0, int c,
                                              int g) {
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
        for (int i = 0; i < 4; ++i) v[i] *= a.wscale[min(nb + i, a.N - 1)];
      }
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

__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Geometry (host plan, rows_plan): NT 16-row batch tiles (R <= 16 NT), MT 16-row weight
// tiles per wave unit, K split into nkc ranges of kr (<= RowsGeo::KR_MAX) columns.
//
// One block (8 waves, 1 per CU) owns ONE K range of the batch tile: its activations are
// read once, RMS-norm-weighted, split into three bf16 parts and written to LDS in MFMA
// B-fragment order (<= 144 KB) before the main loop; after that the waves never
// synchronise.  The nb blocks of a range deal the weight row tiles round-robin to their
// 8 nb waves (tile x + nb (w + 8 i)).  A wave issues ALL LS 16-byte weight loads of its tile
// (non-temporal, LS <= 32 per lane), then runs the tile's k-steps in straight-line code:
// one A fragment from registers against NT x 3 B fragments from LDS (next step's LDS reads
// in flight under this step's MFMAs); each slot is refilled with the wave's next tile as
// soon as its MFMAs have read it, so every wait is an exact in-order vmcnt and the stream
// continues across tiles (the slot is overwritten in place: no copies, no drain).
// The first tile issues a short head of P loads before the activation staging (vmcnt is in
// order: a whole tile per wave ahead of the staging loads would hold them ~10 us).
// Each (tile, range) partial is published write-through (sc1) with the range's sum of
// squares; the wave whose ticket comes last sums the nkc partials in range order
// (deterministic) and runs the epilogue (MI355X_MICROARCH.md "Valid forms", row 1, at wave
// granularity: the wave's own stores drained by vmcnt(0) before its add).
// F8: weights are OCP e4m3 (one 16-byte load = 16 k of a row = two MFMA k-steps, converted
// to bf16 in registers by v_cvt_scalef32_pk_bf16_fp8, exact), per-row scale in the epilogue;
// a lane's 16 bytes hold k = 64 P + 16 g .. +15, so k-step 2P + h contracts k = 64 P + 16 g
// + 8 h + j and the activation fragments are staged in that (consistent) k order.
template <int NT, bool F8>
struct RowsGeo {
  static constexpr int KR_MAX = F8 ? 1536 / NT : (NT == 1 ? 1024 : 1536 / NT);
  static constexpr int KS_MAX = KR_MAX / 32;               // MFMA k-steps per range
  static constexpr int LS = KR_MAX / (F8 ? 64 : 32);       // weight loads per lane per tile
};

template <int MT, int NT, int EPI, bool NORM, bool F8>
__global__ __launch_bounds__(512) void gemm_rows_kernel(GemvArgs a, int kr, int nb, int T) {
  constexpr int NP = 3;
  constexpr int KS = RowsGeo<NT, F8>::KS_MAX;
  constexpr int LS = RowsGeo<NT, F8>::LS;
  constexpr int TILEF = MT * NT * 4 * 64;   // floats of one partial tile
  constexpr int SLAB = TILEF + 16 * NT;     // + the range's sum of squares per batch row
  constexpr int U = NT == 4 ? 3 : 6;        // activation items per staging round (<= 48 = 8 x 6)
  constexpr int P = 4;                      // first-tile weight loads issued ahead of staging
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int y = blockIdx.y, nkc = gridDim.y;
  const int k0 = y * kr, klen = min(kr, a.K - k0);
  const int ks = klen >> 5;                 // MFMA k-steps in this range
  const int ls = F8 ? ks >> 1 : ks;         // weight loads per lane per tile in this range
  const int r0 = blockIdx.z * 16 * NT;
  const int nw = nb * 8;

  __shared__ uint4 xs[NP][NT][KS][64];
  __shared__ float ssw[8][16 * NT];
  __shared__ float ssrow[16 * NT];

  const size_t rowq = F8 ? (size_t)a.K / 16 : (size_t)a.K / 8;  // row length in 16-byte units
  const size_t kq0 = F8 ? (size_t)k0 / 16 : (size_t)k0 / 8;
  // timing experiments only (results invalid unless 0; bit flags): 1 timestamps, 2 skip the
  // activation staging, 4 tile-contiguous weight addressing
  const int dbg = a.rows_dbg;
  const int wstep = (dbg & 4) ? 64 : 4;  // uint4 units between consecutive weight loads
  uint4 wv[LS][MT];
  const uint4* wp[MT];
  // loads [LO, HI) of tile t (branch-free: a short range re-reads its last step)
  auto wbase = [&](int t, int mt) -> const uint4* {
    if (dbg & 4) {
      const size_t rg = (size_t)min(t * MT + mt, (a.N - 1) / 16);
      return static_cast<const uint4*>(a.W) + (rg * (rowq / 4) + kq0 / 4) * 64 + lane;
    }
    const int n = min(t * 16 * MT + 16 * mt + c, a.N - 1);
    return static_cast<const uint4*>(a.W) + (size_t)n * rowq + kq0 + g;
  };
  auto issue = [&](int t, auto lo_c, auto hi_c) {
    constexpr int LO = decltype(lo_c)::value, HI = decltype(hi_c)::value;
    if (LO == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) wp[mt] = wbase(t, mt);
    }
#pragma unroll
    for (int d = LO; d < HI; ++d) {
      const int s = min(d, ls - 1);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) wv[d][mt] = load_nt(wp[mt] + wstep * s);
      __builtin_amdgcn_sched_barrier(0);  // keep issue order = use order (vmcnt is in order)
    }
  };
  using C0 = std::integral_constant<int, 0>;
  using CP = std::integral_constant<int, P>;
  using CL = std::integral_constant<int, LS>;

  const unsigned long long ts0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long ts2 = 0, ts3 = 0;
  int t = blockIdx.x + nb * w;
  if (t < T) issue(t, C0{}, CP{});
  asm volatile("" ::: "memory");  // the head loads stay ahead of the staging

  // ---- stage this range's activations: wave item u = (nt, s), lane (jg = lane&3, cc) ----
  {
    float ssp[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ssp[nt] = 0.f;
    const int jg = lane & 3, cc = lane >> 2;
    const int items = NT * ks;
    for (int u0 = (dbg & 2) ? items : w; u0 < items; u0 += 8 * U) {
      float4 xr[U][2], nr[U][2];
#pragma unroll
      for (int i = 0; i < U; ++i) {
        const int u = u0 + 8 * i;
        const int nt = u % NT, s = u / NT;
        const int b = r0 + 16 * nt + cc;
        const int k = k0 + 32 * s + 8 * jg;
        xr[i][0] = xr[i][1] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (u < items && b < a.R) {
          const float* xp = a.X + (size_t)b * a.xstride + k;
          xr[i][0] = *reinterpret_cast<const float4*>(xp);
          xr[i][1] = *reinterpret_cast<const float4*>(xp + 4);
        }
        if (NORM && u < items) {
          nr[i][0] = *reinterpret_cast<const float4*>(a.norm_w + k);
          nr[i][1] = *reinterpret_cast<const float4*>(a.norm_w + k + 4);
        }
      }
#pragma unroll
      for (int i = 0; i < U; ++i) {
        const int u = u0 + 8 * i;
        if (u >= items) continue;
        const int nt = u % NT, s = u / NT;
        float x[8] = {xr[i][0].x, xr[i][0].y, xr[i][0].z, xr[i][0].w,
                      xr[i][1].x, xr[i][1].y, xr[i][1].z, xr[i][1].w};
        if (NORM) {
          float q = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) q = fmaf(x[j], x[j], q);
#pragma unroll
          for (int n = 0; n < NT; ++n)
            if (n == nt) ssp[n] += q;
          x[0] *= nr[i][0].x; x[1] *= nr[i][0].y; x[2] *= nr[i][0].z; x[3] *= nr[i][0].w;
          x[4] *= nr[i][1].x; x[5] *= nr[i][1].y; x[6] *= nr[i][1].z; x[7] *= nr[i][1].w;
        }
        bf16x8 pf[NP];
        split_parts<NP>(x, pf);
        const int j = 4 * s + jg;  // 8-column piece index within the range
        const int st = F8 ? 2 * (j >> 3) + (j & 1) : s;
        const int gq = F8 ? (j & 7) >> 1 : jg;
#pragma unroll
        for (int p = 0; p < NP; ++p) xs[p][nt][st][gq * 16 + cc] = __builtin_bit_cast(uint4, pf[p]);
      }
    }
    if (NORM) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        float q = ssp[nt];
        q += __shfl_xor(q, 1, 64);
        q += __shfl_xor(q, 2, 64);
        if (jg == 0) ssw[w][16 * nt + cc] = q;
      }
    }
    __syncthreads();
    if (NORM && tid < 16 * NT) {
      float q = 0.f;
#pragma unroll
      for (int v = 0; v < 8; ++v) q += ssw[v][tid];
      ssrow[tid] = q;
    }
    __syncthreads();
  }
  ts2 = __builtin_amdgcn_s_memrealtime();

  auto afrag8 = [&](const uint4& q, int h) -> bf16x8 {
    const uint32_t d0 = h ? q.z : q.x, d1 = h ? q.w : q.y;
    const bf16x2_t e0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d0, 1.0f, false);
    const bf16x2_t e1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d0, 1.0f, true);
    const bf16x2_t e2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d1, 1.0f, false);
    const bf16x2_t e3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d1, 1.0f, true);
    return __builtin_bit_cast(bf16x8, make_uint4(__builtin_bit_cast(uint32_t, e0),
                                                 __builtin_bit_cast(uint32_t, e1),
                                                 __builtin_bit_cast(uint32_t, e2),
                                                 __builtin_bit_cast(uint32_t, e3)));
  };
  // B fragments of one k-step, double-buffered: step k+1's LDS reads fly under step k's MFMAs
  bf16x8 xb[2][NT][NP];
  int kb = 0;  // opaque per tile: stops LICM hoisting 3 NT KS LDS addresses out of the tile loop
  auto ldx = [&](int kst, int buf) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int p = 0; p < NP; ++p)
        xb[buf][nt][p] = __builtin_bit_cast(bf16x8, xs[p][nt][kb + kst][lane]);
  };
  float ss[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) ss[nt] = NORM ? ssrow[16 * nt + c] : 0.f;

  // the tile's k-steps over the loads already in flight (ls <= LS; short ranges skip the rest)
  // the tile's k-steps over the loads already in flight (ls <= LS; short ranges skip the
  // rest).  With a next tile tn, slot s is refilled with tn's step s as soon as step s's
  // MFMAs have read it, so the wave's stream never stops between its tiles (in-order waits
  // stay exact: the next tile consumes its slots in the same order).
  auto compute = [&](f32x4 (&acc)[MT][NT], int tn, auto refill_c) {
    constexpr bool REFILL = decltype(refill_c)::value;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint4* wpn[MT];
    if (REFILL) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) wpn[mt] = wbase(tn, mt);
    }
    kb = 0;
    asm volatile("" : "+v"(kb));
    ldx(0, 0);
#pragma unroll
    for (int s = 0; s < LS; ++s) {
      if (s >= ls) break;
#pragma unroll
      for (int h = 0; h < (F8 ? 2 : 1); ++h) {
        const int kst = F8 ? 2 * s + h : s;
        const int b = F8 ? h : (s & 1);
        ldx(min(kst + 1, ks - 1), b ^ 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const bf16x8 af = F8 ? afrag8(wv[s][mt], h) : __builtin_bit_cast(bf16x8, wv[s][mt]);
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int p = 0; p < NP; ++p)
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, xb[b][nt][p], acc[mt][nt], 0, 0, 0);
        }
      }
      if (REFILL) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) wv[s][mt] = load_nt(wpn[mt] + wstep * s);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  auto finish = [&](int t, f32x4 (&acc)[MT][NT]) {
    const int n0 = t * 16 * MT;
    float sc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) sc[nt] = ss[nt];
    if (nkc > 1) {  // publish this range's partial; the last arriving range merges
      const size_t tile = (size_t)blockIdx.z * T + t;
      float* base = a.ws + tile * nkc * SLAB;
      float* mine = base + (size_t)y * SLAB;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) st_wt(mine + ((mt * NT + nt) * 4 + i) * 64 + lane, acc[mt][nt][i]);
      if (NORM && lane < 16 * NT) st_wt(mine + TILEF + lane, ssrow[lane]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      int last = 0;
      if (lane == 0) {
        const int k = __hip_atomic_fetch_add(a.tickets + tile, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        last = k == nkc - 1;
        if (last) __hip_atomic_store(a.tickets + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (!__shfl(last, 0, 64)) return;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) sc[nt] = 0.f;
      for (int q = 0; q < nkc; ++q) {
        const float* src = base + (size_t)q * SLAB;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[mt][nt][i] += ld_wt(src + ((mt * NT + nt) * 4 + i) * 64 + lane);
        if (NORM) {
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) sc[nt] += ld_wt(src + TILEF + 16 * nt + c);
        }
      }
    }
    float scale[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      scale[nt] = NORM ? 1.0f / sqrtf(sc[nt] / (float)a.K + a.eps) : 1.f;
    rows_epilogue<MT, NT, EPI>(a, acc, scale, n0, r0, c, g);
  };

  int ntiles = 0;
  if (t < T) {
    f32x4 acc[MT][NT];
    issue(t, CP{}, CL{});
    while (true) {
      const int tn = t + nw;
      if (tn < T) compute(acc, tn, std::true_type{});
      else compute(acc, tn, std::false_type{});
      if (!ntiles++) ts3 = __builtin_amdgcn_s_memrealtime();
      finish(t, acc);
      if (tn >= T) break;
      t = tn;
    }
  }
  if ((dbg & 1) && lane == 0 && (blockIdx.x == 0 || blockIdx.x == nb - 1 || blockIdx.x == nb / 2) &&
      (w == 0 || w == 7)) {
    const unsigned long long te = __builtin_amdgcn_s_memrealtime();
    printf("TS b%d y%d w%d tiles %d: t0 %llu staged +%llu tile1 +%llu end +%llu\n", blockIdx.x,
           y, w, ntiles, ts0, ts2 - ts0, ts3 ? ts3 - ts0 : 0ull, te - ts0);
  }
}

struct RowsPlan {
  int mt, nt, kr, nkc, nb, T, tr;
};

static int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  return cus;
}

// K ranges as few as the LDS allows (partials cost R x N x 4 bytes each way per range),
// near-equal and 64-aligned; one block per CU over all ranges of a batch tile.
static RowsPlan rows_plan(int N, int K, int R, bool f8, int cus) {
  RowsPlan p;
  p.nt = R <= 16 ? 1 : R <= 32 ? 2 : 4;
  p.mt = p.nt == 4 ? 2 : 1;
  const int krmax = f8 ? 1536 / p.nt : (p.nt == 1 ? 1024 : 1536 / p.nt);  // RowsGeo::KR_MAX
  p.nkc = (K + krmax - 1) / krmax;
  p.kr = ((K + p.nkc - 1) / p.nkc + 63) / 64 * 64;
  p.nkc = (K + p.kr - 1) / p.kr;
  p.T = (N + 16 * p.mt - 1) / (16 * p.mt);
  p.tr = (R + 16 * p.nt - 1) / (16 * p.nt);
  p.nb = std::max(1, std::min(p.T, cus / p.nkc));
  return p;
}

template <int MT, int NT, int EPI, bool NORM, bool F8>
static hipError_t launch_rows_t(const GemvArgs& a, const RowsPlan& p, hipStream_t st) {
  if (p.kr > RowsGeo<NT, F8>::KR_MAX) return hipErrorInvalidValue;
  const dim3 grid(p.nb, p.nkc, p.tr);
  hipLaunchKernelGGL((gemm_rows_kernel<MT, NT, EPI, NORM, F8>), grid, dim3(512), 0, st, a,
                     p.kr, p.nb, p.T);
  return hipGetLastError();
}

// Workspace (floats) and tickets a launch of this shape needs (0 when K is one range).
void gemm_rows_workspace(int N, int K, int R, int epi, size_t* ws_floats, size_t* tickets) {
  (void)epi;
  *ws_floats = 0;
  *tickets = 0;
  for (bool f8 : {false, true}) {  // the larger need of both weight types
    const RowsPlan p = rows_plan(N, K, R, f8, device_cus());
    const size_t slab = (size_t)p.mt * p.nt * 4 * 64 + 16 * p.nt;
    *ws_floats = std::max(*ws_floats, p.nkc > 1 ? (size_t)p.tr * p.T * p.nkc * slab : (size_t)0);
    *tickets = std::max(*tickets, (size_t)p.tr * p.T);
  }
}

// R >= 2 rows (and fp8 shapes).  hipErrorNotSupported for shapes the kernel does not cover.
hipError_t launch_gemm_rows(const GemvArgs& a, int epi, bool norm, hipStream_t st) {
  if (a.R < 1 || a.K % 64) return hipErrorNotSupported;
  const bool f8 = a.wdtype == WT_FP8;
  const RowsPlan p = rows_plan(a.N, a.K, a.R, f8, device_cus());
  if (p.nkc > 1) {
    const size_t slab = (size_t)p.mt * p.nt * 4 * 64 + 16 * p.nt;
    const size_t need = (size_t)p.tr * p.T * p.nkc * slab;
    if (!a.ws || !a.tickets || need > a.ws_floats || (size_t)p.tr * p.T > a.tickets_n)
      return hipErrorInvalidValue;
  }
#define MX_R(EPI_, NORM_)                                                                   \
  if (epi == EPI_ && norm == NORM_) {                                                       \
    if (p.nt == 1) return f8 ? launch_rows_t<1, 1, EPI_, NORM_, true>(a, p, st)             \
                             : launch_rows_t<1, 1, EPI_, NORM_, false>(a, p, st);           \
    if (p.nt == 2) return f8 ? launch_rows_t<1, 2, EPI_, NORM_, true>(a, p, st)             \
                             : launch_rows_t<1, 2, EPI_, NORM_, false>(a, p, st);           \
    return f8 ? launch_rows_t<2, 4, EPI_, NORM_, true>(a, p, st)                            \
              : launch_rows_t<2, 4, EPI_, NORM_, false>(a, p, st);                          \
  }
  MX_R(EPI_QKV, true)
  MX_R(EPI_RESID, false)
  MX_R(EPI_SILU, true)
  MX_R(EPI_ARGMAX, true)
  MX_R(EPI_STORE, false)
  MX_R(EPI_STORE, true)
#undef MX_R
  return hipErrorNotSupported;
}

}  // namespace mx
