// Multi-row decode GEMM, generation 4 (the only multi-row generation built; generations 5
// and 7 were measured 3.6-5 % and 13-60 % slower and were retired).
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

#include <algorithm>

namespace mx {
namespace v4 {

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
        const float pen = a.penalty[slot];
        const bool keep = a.logits && (a.logits_all || a.samp_temp[slot] > 0.f);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = nb + i;
          if (n >= a.N) continue;
          float x = v[i];
          if (seen[n]) x = x > 0.f ? x / pen : x * pen;
          if (keep) a.logits[(size_t)b * a.N + n] = x;
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

// One block = 8 waves; wave w owns weight rows n0 + 16 MT w .. (+16 MT) of the block's tile
// and the tile's 16 NT batch rows, over the block's K range of SUB sub-chunks of 128.
// Activations are shared, not re-read per wave: each sub-chunk of X is loaded ONCE per block
// (one 32-byte piece per thread), RMS-norm-weighted, split into three bf16 parts and written
// to LDS in MFMA B-fragment order (ds_read_b128, lane-linear, conflict-free); the weights
// stream straight to registers one sub-chunk ahead.  Issue order per sub-chunk: X(s+1)
// then W(s+1), so staging X(s+1) never waits behind the weight stream (vmcnt is in order).
// K ranges (gridDim.y of them) give the grid its parallelism; each publishes its partial
// tiles with write-through (sc1) stores, and the last arriving range sums them in range
// order (deterministic) and runs the epilogue (MI355X_MICROARCH.md "Valid forms", row 1).
// F8: weights are OCP e4m3 (16 per 16-byte load = two MFMA k-steps; converted to bf16 in
// registers by v_cvt_scalef32_pk_bf16_fp8, exact) with a per-row scale in the epilogue.  A
// lane's 16 bytes hold k = 64 P + 16 g .. +15, so k-step 2P + h contracts k = 64 P + 16 g +
// 8 h + j, and the activation fragments are staged in that (consistent) k order.
// PW: weight prefetch distance in sub-chunks (1 = the original double buffer); with PW > 1 the
// activation pieces run DX = 2 sub-chunks ahead and are issued BEFORE each sub-chunk's
// weights, so the in-order vmcnt wait that stages X(s+1) only drains weights already needed.
template <int MT, int NT, int EPI, bool NORM, int SUB, bool F8, int PW = 1>
__global__ __launch_bounds__(512) void gemm_rows_kernel(GemvArgs a) {
  constexpr int NP = 3, ST = 4;             // activation parts; k-steps per sub-chunk
  constexpr int DX = PW > 1 ? 2 : 1, NBX = DX + 1, NBW = PW + 1;  // prefetch distances, buffers
  constexpr int ITEMS = (NT * 16 * 16) / 512 > 0 ? (NT * 16 * 16) / 512 : 1;  // X pieces/thread
  constexpr int WSLAB = MT * NT * 4 * 64;   // floats per wave partial
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * (8 * 16 * MT) + w * 16 * MT;
  const int kc = blockIdx.y, nkc = gridDim.y;
  const int r0 = blockIdx.z * (16 * NT);
  const int kr0 = kc * SUB * 128;

  __shared__ uint4 xs[2][NP][NT][ST][64];
  __shared__ float ssrow[16 * NT];
  __shared__ int last_s;

  // X piece of thread t (item it): batch row b = (t + 512 it) >> 4, 8 k at 8 ((t) & 15)
  const bool xact = tid < NT * 16 * 16;
  int xb[ITEMS], xj[ITEMS];
  const float* xrow[ITEMS];
#pragma unroll
  for (int it = 0; it < ITEMS; ++it) {
    const int q = tid + 512 * it;
    xb[it] = min(q >> 4, 16 * NT - 1);
    xj[it] = q & 15;
    xrow[it] = a.X + (size_t)min(r0 + xb[it], a.R - 1) * a.xstride + 8 * xj[it];
  }
  const uint4* wrow[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int n = min(n0 + 16 * mt + c, a.N - 1);
    wrow[mt] = F8 ? reinterpret_cast<const uint4*>(static_cast<const uint8_t*>(a.W) + (size_t)n * a.K) + g
                  : reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(a.W) + (size_t)n * a.K) + g;
  }
  float ssp[ITEMS];
#pragma unroll
  for (int it = 0; it < ITEMS; ++it) ssp[it] = 0.f;

  float4 xr[NBX][ITEMS][2], nr[NBX][ITEMS][2];
  constexpr int WL = F8 ? ST / 2 : ST;      // 16-byte weight loads per row per sub-chunk
  uint4 wv[NBW][WL][MT];
  auto load_x = [&](int sub, int buf) {
    const int k = kr0 + 128 * sub;
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
      xr[buf][it][0] = *reinterpret_cast<const float4*>(xrow[it] + k);
      xr[buf][it][1] = *reinterpret_cast<const float4*>(xrow[it] + k + 4);
      if (NORM) {
        const float* nw = a.norm_w + k + 8 * xj[it];
        nr[buf][it][0] = *reinterpret_cast<const float4*>(nw);
        nr[buf][it][1] = *reinterpret_cast<const float4*>(nw + 4);
      }
    }
  };
  auto load_w = [&](int sub, int buf) {
    const int kq = (kr0 + 128 * sub) / (F8 ? 16 : 8);  // in 16-byte units of a row
#pragma unroll
    for (int l = 0; l < WL; ++l)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) wv[buf][l][mt] = load_nt(wrow[mt] + kq + 4 * l);
  };
  // A fragment of k-step st for weight tile mt
  auto afrag = [&](int buf, int st, int mt) -> bf16x8 {
    if (!F8) return __builtin_bit_cast(bf16x8, wv[buf][st][mt]);
    const uint4 q = wv[buf][st >> 1][mt];
    const uint32_t d0 = (st & 1) ? q.z : q.x, d1 = (st & 1) ? q.w : q.y;
    const bf16x2_t e0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d0, 1.0f, false);
    const bf16x2_t e1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d0, 1.0f, true);
    const bf16x2_t e2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d1, 1.0f, false);
    const bf16x2_t e3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d1, 1.0f, true);
    return __builtin_bit_cast(bf16x8, make_uint4(__builtin_bit_cast(uint32_t, e0),
                                                 __builtin_bit_cast(uint32_t, e1),
                                                 __builtin_bit_cast(uint32_t, e2),
                                                 __builtin_bit_cast(uint32_t, e3)));
  };
  auto stage_x2 = [&](int buf, int lb) {
    if (!xact) return;
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
      float x[8] = {xr[buf][it][0].x, xr[buf][it][0].y, xr[buf][it][0].z, xr[buf][it][0].w,
                    xr[buf][it][1].x, xr[buf][it][1].y, xr[buf][it][1].z, xr[buf][it][1].w};
      if (NORM) {
#pragma unroll
        for (int j = 0; j < 8; ++j) ssp[it] = fmaf(x[j], x[j], ssp[it]);
        x[0] *= nr[buf][it][0].x; x[1] *= nr[buf][it][0].y;
        x[2] *= nr[buf][it][0].z; x[3] *= nr[buf][it][0].w;
        x[4] *= nr[buf][it][1].x; x[5] *= nr[buf][it][1].y;
        x[6] *= nr[buf][it][1].z; x[7] *= nr[buf][it][1].w;
      }
      bf16x8 pf[NP];
      split_parts<NP>(x, pf);
      const int b = xb[it], j = xj[it];  // 8 activations at k = 8 j of the sub-chunk
      const int st = F8 ? 2 * (j >> 3) + (j & 1) : j >> 2;
      const int gq = F8 ? (j & 7) >> 1 : j & 3;
#pragma unroll
      for (int p = 0; p < NP; ++p)
        xs[lb][p][b >> 4][st][gq * 16 + (b & 15)] = __builtin_bit_cast(uint4, pf[p]);
    }
  };
  auto stage_x = [&](int buf) { stage_x2(buf, 0); };

  // one accumulator per activation part: NP x NT x MT independent MFMA chains, so consecutive
  // MFMAs never wait on each other's result (SQ_WAIT_INST_ANY was 38 % of wave cycles)
  f32x4 pacc[NP][MT][NT];
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) pacc[p][mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int d = 0; d < DX; ++d)
    if (d < SUB) load_x(d, d % NBX);
#pragma unroll
  for (int d = 0; d < PW; ++d)
    if (d < SUB) load_w(d, d % NBW);
  stage_x(0);
  __syncthreads();
#pragma unroll
  for (int sub = 0; sub < SUB; ++sub) {
    const int cur = sub & 1, nxt = cur ^ 1;  // LDS buffers
    if (sub + DX < SUB) load_x(sub + DX, (sub + DX) % NBX);
    if (sub + PW < SUB) load_w(sub + PW, (sub + PW) % NBW);
    const int wb = sub % NBW;
#pragma unroll
    for (int st = 0; st < ST; ++st) {
      bf16x8 af[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) af[mt] = afrag(wb, st, mt);
#pragma unroll
      for (int p = 0; p < NP; ++p) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const bf16x8 xb8 = __builtin_bit_cast(bf16x8, xs[cur][p][nt][st][lane]);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
            pacc[p][mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], xb8,
                                                                      pacc[p][mt][nt], 0, 0, 0);
        }
      }
    }
    if (sub + 1 < SUB) stage_x2((sub + 1) % NBX, nxt);
    __syncthreads();
  }
  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = (pacc[0][mt][nt] + pacc[1][mt][nt]) + pacc[2][mt][nt];
  // per-row sum of squares of this K range: the 16 threads of a row are 16 adjacent lanes
  if (NORM) {
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
      float t = ssp[it];
      t += __shfl_xor(t, 1, 64);
      t += __shfl_xor(t, 2, 64);
      t += __shfl_xor(t, 4, 64);
      t += __shfl_xor(t, 8, 64);
      if (xact && xj[it] == 0) ssrow[xb[it]] = t;
    }
    __syncthreads();
  }
  float ss[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) ss[nt] = NORM ? ssrow[16 * nt + c] : 0.f;

  if (nkc > 1) {  // publish this K range's partial, last arriver merges in range order
    const size_t tile = (size_t)blockIdx.z * gridDim.x + blockIdx.x;
    const size_t slab_floats = 8 * (size_t)WSLAB + 16 * NT;
    float* base = a.ws + tile * nkc * slab_floats;
    float* mine = base + (size_t)kc * slab_floats;
    // lane-major partial: a lane's MT x NT quads are contiguous (16-byte sc1 accesses); the
    // buffer descriptor stays block-uniform (a per-lane base would be a waterfall loop)
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const size_t lofs = (size_t)wu * WSLAB + (size_t)lane * (4 * MT * NT);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) st4_wt(mine, lofs + (mt * NT + nt) * 4, acc[mt][nt]);
    if (NORM && tid < 16 * NT) st_wt(mine + 8 * (size_t)WSLAB + tid, ssrow[tid]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const int t = __hip_atomic_fetch_add(a.tickets + tile, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == nkc - 1;
      if (last) __hip_atomic_store(a.tickets + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_s = last;
    }
    __syncthreads();
    if (!last_s) return;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ss[nt] = 0.f;
    // the K ranges' partials, four ranges' loads in flight at a time, summed in range order
    for (int q0 = 0; q0 < nkc; q0 += 4) {
      f32x4 t[4][MT][NT];
      float sq[4][NT];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float* src = base + (size_t)min(q0 + j, nkc - 1) * slab_floats;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) t[j][mt][nt] = ld4_wt(src, lofs + (mt * NT + nt) * 4);
        if (NORM) {
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) sq[j][nt] = ld_wt(src + 8 * (size_t)WSLAB + 16 * nt + c);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (q0 + j >= nkc) break;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[mt][nt][i] += t[j][mt][nt][i];
        if (NORM) {
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) ss[nt] += sq[j][nt];
        }
      }
    }
  }
  float scale[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
    scale[nt] = NORM ? 1.0f / sqrtf(ss[nt] / (float)a.K + a.eps) : 1.f;
  rows_epilogue<MT, NT, EPI>(a, acc, scale, n0, r0, c, g);
}

// K ranges per launch: enough blocks to fill the chip without inflating the partial-tile
// traffic (each range adds R x N x 4 bytes of write-through partials).
static int rows_nkc(int N, int K, int R, int MT, int NT, int target = 384) {
  const int subs = K / 128;
  const int tiles = ((N + 128 * MT - 1) / (128 * MT)) * ((R + 16 * NT - 1) / (16 * NT));
  int nkc = 1;
  while (tiles * nkc < target && subs % (2 * nkc) == 0 && subs / (2 * nkc) >= 2) nkc *= 2;
  while (tiles * nkc < target && subs % (3 * nkc) == 0 && subs / (3 * nkc) >= 2) nkc *= 3;
  return nkc;
}

template <int MT, int NT, int EPI, bool NORM, int SUB, int PW>
static hipError_t launch_rows_pw(const GemvArgs& a, int nkc, hipStream_t st) {
  if (a.wdtype == WT_FP8 && a.K % 128) return hipErrorNotSupported;
  const int tiles_n = (a.N + 128 * MT - 1) / (128 * MT), tiles_r = (a.R + 16 * NT - 1) / (16 * NT);
  if (nkc > 1) {
    const size_t need = (size_t)tiles_n * tiles_r * nkc * (8 * MT * NT * 4 * 64 + 16 * NT);
    if (!a.ws || !a.tickets || need > a.ws_floats || (size_t)tiles_n * tiles_r > a.tickets_n)
      return hipErrorInvalidValue;
  }
  const dim3 grid(tiles_n, nkc, tiles_r);
  if (a.wdtype == WT_FP8) {
    hipLaunchKernelGGL((gemm_rows_kernel<MT, NT, EPI, NORM, SUB, true, PW>), grid, dim3(512), 0, st, a);
  } else {
    if constexpr (PW <= 2)
      hipLaunchKernelGGL((gemm_rows_kernel<MT, NT, EPI, NORM, SUB, false, PW>), grid, dim3(512), 0, st, a);
    else
      return hipErrorNotSupported;
  }
  return hipGetLastError();
}

// Prefetch distance 2 (bf16): measured 97.3 vs 103.5 us per layer of projections at 32 rows,
// neutral at 8 rows; distance 3 was slower (scripts/gpu_pw.sh).  e4m3 weights (half the bytes
// per sub-chunk): distance 2 measured 53.6 vs 66.3 us per layer at 8 rows, 3 no better
// (scripts/gpu_f8pw.sh).
template <int MT, int NT, int EPI, bool NORM, int SUB>
static hipError_t launch_rows_sub(const GemvArgs& a, int nkc, hipStream_t st) {
  const int pw = a.wdtype == WT_FP8 ? a.rows_pw_f8 : a.rows_pw;
  if (pw >= 2 && SUB > 1) return launch_rows_pw<MT, NT, EPI, NORM, SUB, 2>(a, nkc, st);
  return launch_rows_pw<MT, NT, EPI, NORM, SUB, 1>(a, nkc, st);
}

template <int MT, int NT, int EPI, bool NORM>
static hipError_t launch_rows_k(const GemvArgs& a, hipStream_t st) {
  if (a.K % 128) return hipErrorNotSupported;
  // K-range split target (blocks): measured at 8 and 32 rows (scripts/gpu_target.sh) the qkv
  // projection is fastest aiming at 128 blocks, the others at 192 (384 was the old default)
  const int target = a.rows_target > 0 ? a.rows_target : (EPI == EPI_QKV ? 128 : 192);
  const int nkc = rows_nkc(a.N, a.K, a.R, MT, NT, target);
  switch (a.K / 128 / nkc) {
    case 1: return launch_rows_sub<MT, NT, EPI, NORM, 1>(a, nkc, st);
    case 2: return launch_rows_sub<MT, NT, EPI, NORM, 2>(a, nkc, st);
    case 3: return launch_rows_sub<MT, NT, EPI, NORM, 3>(a, nkc, st);
    case 4: return launch_rows_sub<MT, NT, EPI, NORM, 4>(a, nkc, st);
    case 6: return launch_rows_sub<MT, NT, EPI, NORM, 6>(a, nkc, st);
    case 8: return launch_rows_sub<MT, NT, EPI, NORM, 8>(a, nkc, st);
    case 12: return launch_rows_sub<MT, NT, EPI, NORM, 12>(a, nkc, st);
    case 16: return launch_rows_sub<MT, NT, EPI, NORM, 16>(a, nkc, st);
    case 24: return launch_rows_sub<MT, NT, EPI, NORM, 24>(a, nkc, st);
    default: return hipErrorNotSupported;
  }
}

// Batch tile: 16 NT rows (nt_max caps it: option rows_nt_max).  Measured at 32 rows: a 16-row
// cap is slower (102.7 vs 87.9 us per layer of projections), and 32 weight rows per wave
// (one staged activation sub-chunk feeding twice the weights) far slower (141.7 us: half the
// tiles leave CUs idle), so the weight tile stays 16 rows per wave.
static void rows_tiles(int epi, int R, int* mt, int* nt, int nt_max = 4) {
  *nt = R <= 16 ? 1 : R <= 32 ? 2 : 4;
  if (nt_max > 0 && *nt > nt_max) *nt = nt_max;
  *mt = 1;
}

// Workspace (floats) and tickets a launch of this shape needs (0 when K is one range).
void gemm_rows_workspace_v4(int N, int K, int R, int epi, size_t* ws_floats, size_t* tickets) {
  *ws_floats = 0;
  *tickets = 0;
  for (int cap : {1, 2, 4}) {  // every batch-tile cap option rows_nt_max may pick
    int mt, nt;
    rows_tiles(epi, R, &mt, &nt, cap);
    const int nkc = K % 128 ? 1 : rows_nkc(N, K, R, mt, nt);
    const size_t tn = (N + 128 * mt - 1) / (128 * mt), tr = (R + 16 * nt - 1) / (16 * nt);
    *ws_floats = std::max(*ws_floats, nkc > 1 ? tn * tr * nkc * (8 * (size_t)mt * nt * 4 * 64 + 16 * nt) : (size_t)0);
    *tickets = std::max(*tickets, tn * tr);
  }
}

// R >= 2 rows.  Returns hipErrorNotSupported for shapes the kernel does not cover.
hipError_t launch_gemm_rows_v4(const GemvArgs& a, int epi, bool norm, hipStream_t st) {
  if (a.R < 1) return hipErrorNotSupported;
  int mt, nt;
  rows_tiles(epi, a.R, &mt, &nt, a.rows_nt_max);
#define MX_R(EPI_, NORM_)                                                                 \
  if (epi == EPI_ && norm == NORM_) {                                                     \
    if (nt == 1) return launch_rows_k<1, 1, EPI_, NORM_>(a, st);                          \
    if (nt == 2) return launch_rows_k<1, 2, EPI_, NORM_>(a, st);                          \
    return launch_rows_k<1, 4, EPI_, NORM_>(a, st);                                       \
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

}  // namespace v4
}  // namespace mx
