// Orpheus / Llama-3.2-3B decode-step kernels for MI355X (gfx950).
//
// Replaces the bf16 decode inside vLLM AsyncLLMEngine.generate
// (Orpheus-TTS/orpheus_tts_pypi/orpheus_tts/engine_class.py:117) and llama.cpp
// Llama.text_to_speech (Morpheus_Client/tts_engine/llama_local.py:77).
//
// Precision contract: bf16 weights, fp32 activations and accumulation,
// bf16 KV cache (RNE), fp32 logits.  Every weight byte is streamed once per step:
// the step is HBM-bound, so the GEMVs are written for bytes in flight,
// not for MFMA: 16-byte non-temporal weight loads, activations staged once per block in
// LDS (split lo/hi float4 planes -> conflict-free ds_read_b128), wave64 butterflies.
#include "mx_common.h"
#include "mx_llm_kernels.h"

#include <initializer_list>

namespace mx {

// ---------------------------------------------------------------------------------
// Weight-streaming GEMV with fused prologue (RMSNorm) and epilogues.
//   y[r][n] = sum_k W[n][k] * xn[r][k]   for r in the block's RT activation rows.
// Grid: x = row-group workers (grid-stride over N / RPW groups, one wave per group),
//       y = ceil(R / RT) activation-row tiles.
// ---------------------------------------------------------------------------------
template <int RT, int RPW, int EPI, bool NORM, bool F8 = false>
__global__ __launch_bounds__(256) void gemv_kernel(GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K8 = a.K >> 3;
  float4* xlo = reinterpret_cast<float4*>(smem);
  float4* xhi = xlo + RT * K8;
  float* red = reinterpret_cast<float*>(xhi + RT * K8);  // [8] scratch
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r0 = blockIdx.y * RT;
  const int nr = min(RT, a.R - r0);

  // ---- prologue: stage (optionally RMS-normalised) activation rows in LDS -------------
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float ss = 0.f;
    if (rt < nr) {
      const float4* src = reinterpret_cast<const float4*>(a.X + (size_t)(r0 + rt) * a.xstride);
      for (int c = tid; c < K8; c += 256) {
        float4 lo = src[2 * c], hi = src[2 * c + 1];
        xlo[rt * K8 + c] = lo;
        xhi[rt * K8 + c] = hi;
        if (NORM) {
          ss += lo.x * lo.x + lo.y * lo.y + lo.z * lo.z + lo.w * lo.w;
          ss += hi.x * hi.x + hi.y * hi.y + hi.z * hi.z + hi.w * hi.w;
        }
      }
    } else {
      for (int c = tid; c < K8; c += 256) {
        xlo[rt * K8 + c] = make_float4(0.f, 0.f, 0.f, 0.f);
        xhi[rt * K8 + c] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    if (NORM) {
      ss = wave_sum(ss);
      if (lane == 0) red[wid] = ss;
      __syncthreads();
      const float tot = red[0] + red[1] + red[2] + red[3];
      const float scale = 1.0f / sqrtf(tot / (float)a.K + a.eps);
      __syncthreads();
      if (rt < nr) {
        const float4* nw = reinterpret_cast<const float4*>(a.norm_w);
        for (int c = tid; c < K8; c += 256) {
          float4 lo = xlo[rt * K8 + c], hi = xhi[rt * K8 + c];
          const float4 wl = nw[2 * c], wh = nw[2 * c + 1];
          lo.x = lo.x * scale * wl.x; lo.y = lo.y * scale * wl.y;
          lo.z = lo.z * scale * wl.z; lo.w = lo.w * scale * wl.w;
          hi.x = hi.x * scale * wh.x; hi.y = hi.y * scale * wh.y;
          hi.z = hi.z * scale * wh.z; hi.w = hi.w * scale * wh.w;
          xlo[rt * K8 + c] = lo;
          xhi[rt * K8 + c] = hi;
        }
      }
    }
  }
  __syncthreads();

  // ---- main loop: one wave per group of RPW consecutive weight rows -------------------
  const int G = (a.N + RPW - 1) / RPW;
  const int nworkers = gridDim.x * 4;
  unsigned long long best[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) best[rt] = 0ull;

  for (int g = blockIdx.x * 4 + wid; g < G; g += nworkers) {
    const int n0 = g * RPW;
    float acc[RPW][RT];
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[i][rt] = 0.f;
    const uint4* wp[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int n = min(n0 + i, a.N - 1);  // tail rows (lm_head) re-read the last row
      wp[i] = F8 ? reinterpret_cast<const uint4*>(static_cast<const uint8_t*>(a.W) + (size_t)n * a.K)
                 : reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(a.W) + (size_t)n * a.K);
    }
    if (F8) {  // 16 e4m3 weights per 16-byte chunk = activation chunks 2c, 2c+1
#pragma unroll 4
      for (int c = lane; c < (K8 >> 1); c += 64) {
        uint4 w[RPW];
#pragma unroll
        for (int i = 0; i < RPW; ++i) w[i] = load_nt(wp[i] + c);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const float4 x0 = xlo[rt * K8 + 2 * c], x1 = xhi[rt * K8 + 2 * c];
          const float4 x2 = xlo[rt * K8 + 2 * c + 1], x3 = xhi[rt * K8 + 2 * c + 1];
#pragma unroll
          for (int i = 0; i < RPW; ++i) {
            const uint32_t wd[4] = {w[i].x, w[i].y, w[i].z, w[i].w};
            const float4 xx[4] = {x0, x1, x2, x3};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const f32x2_t lo = __builtin_amdgcn_cvt_pk_f32_fp8(wd[q], false);
              const f32x2_t hi = __builtin_amdgcn_cvt_pk_f32_fp8(wd[q], true);
              acc[i][rt] = fmaf(lo.x, xx[q].x, acc[i][rt]);
              acc[i][rt] = fmaf(lo.y, xx[q].y, acc[i][rt]);
              acc[i][rt] = fmaf(hi.x, xx[q].z, acc[i][rt]);
              acc[i][rt] = fmaf(hi.y, xx[q].w, acc[i][rt]);
            }
          }
        }
      }
    } else {
#pragma unroll 4
      for (int c = lane; c < K8; c += 64) {
        uint4 w[RPW];
#pragma unroll
        for (int i = 0; i < RPW; ++i) w[i] = load_nt(wp[i] + c);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const float4 lo = xlo[rt * K8 + c], hi = xhi[rt * K8 + c];
#pragma unroll
          for (int i = 0; i < RPW; ++i) acc[i][rt] = dot8(w[i], lo, hi, acc[i][rt]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        acc[i][rt] = wave_sum(acc[i][rt]);
        if (F8) acc[i][rt] *= a.wscale[min(n0 + i, a.N - 1)];
      }

    // ---- epilogues (every lane holds every total; lane 0 writes) -----------------------
    if (EPI == EPI_ARGMAX) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        if (rt < nr) {
          const int slot = a.row_slot[r0 + rt];
          const uint8_t* seen = a.seen + (size_t)slot * a.N;
          const float pen = a.penalty[slot];
          const bool keep = a.logits && (a.logits_all || a.samp_temp[slot] > 0.f);
#pragma unroll
          for (int i = 0; i < RPW; ++i) {
            const int n = n0 + i;
            if (n < a.N) {
              float v = acc[i][rt];
              if (seen[n]) v = v > 0.f ? v / pen : v * pen;
              if (keep && lane == 0) a.logits[(size_t)(r0 + rt) * a.N + n] = v;
              const unsigned long long key = argmax_key(v, (uint32_t)n);
              best[rt] = key > best[rt] ? key : best[rt];
            }
          }
        }
      }
    } else if (lane == 0) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        if (rt >= nr) continue;
        const int r = r0 + rt;
        if (EPI == EPI_STORE) {
#pragma unroll
          for (int i = 0; i < RPW; ++i) a.Y[(size_t)r * a.N + n0 + i] = acc[i][rt];
        } else if (EPI == EPI_RESID) {
#pragma unroll
          for (int i = 0; i < RPW; ++i) a.Y[(size_t)r * a.ystride + n0 + i] += acc[i][rt];
        } else if (EPI == EPI_SILU) {
#pragma unroll
          for (int i = 0; i < RPW; i += 2) {
            const float g = acc[i][rt], u = acc[i + 1][rt];
            a.Y[(size_t)r * (a.N >> 1) + ((n0 + i) >> 1)] = g / (1.0f + expf(-g)) * u;
          }
        } else if (EPI == EPI_QKV) {
          const int slot = a.row_slot[r], pos = a.row_pos[r];
#pragma unroll
          for (int i = 0; i < RPW; i += 2) {
            const int n = n0 + i;
            const int hh = n >> 7, within = n & 127, p = within >> 1;
            const float x1 = acc[i][rt], x2 = acc[i + 1][rt];
            if (hh < a.heads + a.kv_heads) {
              const float c = a.rope_cos[(size_t)pos * 64 + p];
              const float s = a.rope_sin[(size_t)pos * 64 + p];
              const float o1 = x1 * c - x2 * s;
              const float o2 = x2 * c + x1 * s;
              if (hh < a.heads) {
                float* q = a.Q + ((size_t)r * a.heads + hh) * 128;
                q[p] = o1;
                q[p + 64] = o2;
              } else {
                uint16_t* k = a.kcache +
                    ((size_t)slot * a.kv_heads + (hh - a.heads)) * a.max_pos * 128;
                k[kv_k_off(pos, p)] = f32_to_bf16(o1);
                k[kv_k_off(pos, p + 64)] = f32_to_bf16(o2);
              }
            } else {
              // fragment-major chunks (mx_common.h kv_v_off, see attn_kernel)
              uint16_t* v = a.vcache +
                  ((size_t)slot * a.kv_heads + (hh - a.heads - a.kv_heads)) * 128 * a.max_pos;
              v[kv_v_off(pos, within)] = f32_to_bf16(x1);
              v[kv_v_off(pos, within + 1)] = f32_to_bf16(x2);
            }
          }
        }
      }
    }
  }

  if (EPI == EPI_ARGMAX) {
    __shared__ unsigned long long bred[4][RT];
    if (lane == 0) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) bred[wid][rt] = best[rt];
    }
    __syncthreads();
    if (tid < RT && tid < nr) {
      unsigned long long k = bred[0][tid];
      for (int w = 1; w < 4; ++w) k = bred[w][tid] > k ? bred[w][tid] : k;
      atomicMax(a.best + r0 + tid, k);
    }
  }
}

// ---------------------------------------------------------------------------------
// Single-row (B = 1 decode) weight-streaming GEMV.
//   One wave owns RPW consecutive weight rows over the whole K = 512*KCH; 8 waves per
//   block share one LDS copy of the (RMS-normalised) activation row.  Load order is the
//   point (cdna_hip_programming.md §5 row "GEMV / M <= 16"): the activation / norm loads
//   go first, then every weight load of the wave (RPW*KCH x 16 B per lane, non-temporal),
//   and only then the prologue (norm, LDS staging) runs, under the weight loads' latency.
//   All loads are unconditional (addresses clamped), so hipcc can count vmcnt exactly.
//   Epilogue operands that do not depend on the result (residual, RoPE row) are fetched
//   with the activation.
// ---------------------------------------------------------------------------------
// F8: weights are OCP e4m3 bytes with one fp32 scale per row (16 weights per 16-byte load,
// converted in registers by v_cvt_pk_f32_fp8 -- exact), else bf16 (8 per load).
// MRG (NSM > 0, the R = 1 o-projection): the activation is the attention output, merged
// here from its split partials (attn_kernel no_merge mode): for 8-dim group j of head hh,
// att = sum_s e^(m_s - M) acc_s / sum_s e^(m_s - M) l_s over the row's live splits (at most
// NSM).  The partial loads go out first, the weight loads behind them, and the merge runs
// under the weight latency -- the split merge costs no extra launch, ticket or round trip.
template <int NSM>
struct MergeIn {  // one 8-dim group's split partials, loaded
  float2 ml[NSM];
  float4 lo[NSM], hi[NSM];
};
template <int NSM>
__device__ __forceinline__ void merge_load(const GemvArgs& a, int j, int ns, MergeIn<NSM>& in) {
  const int GRP = a.heads / a.kv_heads;
  const int hh = j >> 4, d0 = (j & 15) * 8;
  const int kvh = hh / GRP, hin = hh - kvh * GRP;
  const size_t pb = (size_t)kvh * a.att_stride;
#pragma unroll
  for (int s = 0; s < NSM; ++s) {
    const size_t sp = pb + min(s, ns - 1);
    in.ml[s] = *reinterpret_cast<const float2*>(a.att_ml + (sp * GRP + hin) * 2);
    const float4* ac = reinterpret_cast<const float4*>(a.att_acc + (sp * GRP + hin) * 128 + d0);
    in.lo[s] = ac[0];
    in.hi[s] = ac[1];
  }
}
template <int NSM>
__device__ __forceinline__ void merge_apply(const MergeIn<NSM>& in, int ns, float* x) {
  float M = -INFINITY;
#pragma unroll
  for (int s = 0; s < NSM; ++s)
    if (s < ns) M = fmaxf(M, in.ml[s].x);
  float den = 0.f;
  float num[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NSM; ++s) {
    const float f = s < ns ? expf(in.ml[s].x - M) : 0.f;
    den = fmaf(f, in.ml[s].y, den);
    num[0] = fmaf(f, in.lo[s].x, num[0]); num[1] = fmaf(f, in.lo[s].y, num[1]);
    num[2] = fmaf(f, in.lo[s].z, num[2]); num[3] = fmaf(f, in.lo[s].w, num[3]);
    num[4] = fmaf(f, in.hi[s].x, num[4]); num[5] = fmaf(f, in.hi[s].y, num[5]);
    num[6] = fmaf(f, in.hi[s].z, num[6]); num[7] = fmaf(f, in.hi[s].w, num[7]);
  }
  const float inv = 1.0f / den;
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = num[i] * inv;
}

template <int KCH, int RPW, int EPI, bool NORM, int WPB, bool F8, int NSM = 0>
__global__ __launch_bounds__(WPB * 64) void gemv1_kernel(GemvArgs a) {
  constexpr int NT = WPB * 64;
  constexpr int EPC = F8 ? 16 : 8;             // weights per 16-byte chunk
  constexpr int PL = EPC / 4;                  // float4 planes of the staged activation
  constexpr int KC = KCH * 64;                 // 16-byte weight chunks per row
  constexpr int XPT = (KC + NT - 1) / NT;      // activation chunks per thread
  __shared__ __attribute__((aligned(16))) float4 xs[PL * KC];  // plane q at [q * KC + m]
  __shared__ float red[WPB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int G = a.N / RPW;
  int g = blockIdx.x * WPB + wid;
  const bool active = g < G;
  g = active ? g : G - 1;
  const int n0 = g * RPW;

  // 1. activation (+ norm weight, + epilogue operands)
  const float4* X4 = reinterpret_cast<const float4*>(a.X);
  const float4* NW4 = reinterpret_cast<const float4*>(a.norm_w);
  float4 xv[XPT][PL], nv[XPT][PL];
  constexpr int NG = KC * EPC / 8;  // 8-dim groups of the merged activation (MRG)
  int ns = 1;
  MergeIn<(NSM > 0 ? NSM : 1)> mi;
  if constexpr (NSM > 0) {
    const int L = a.row_pos[0] + 1;
    ns = (L + a.att_S - 1) / a.att_S;
    merge_load<NSM>(a, min(tid, NG - 1), ns, mi);  // group tid's partial loads go first
  } else {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int m = min(tid + i * NT, KC - 1);
#pragma unroll
      for (int q = 0; q < PL; ++q) {
        xv[i][q] = X4[PL * m + q];
        if (NORM) nv[i][q] = NW4[PL * m + q];
      }
    }
  }
  float res[RPW], wsc[RPW];
  if (EPI == EPI_RESID) {
#pragma unroll
    for (int r = 0; r < RPW; ++r) res[r] = a.Y[n0 + r];
  }
  if (F8) {
#pragma unroll
    for (int r = 0; r < RPW; ++r) wsc[r] = a.wscale[n0 + r];
  }
  // 2. every weight load of this wave
  uint4 w[RPW][KCH];
  const uint4* wp = reinterpret_cast<const uint4*>(a.W) + (size_t)n0 * KC + lane;
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int c = 0; c < KCH; ++c) w[r][c] = load_nt(wp + (size_t)r * KC + c * 64);
  __builtin_amdgcn_sched_barrier(0);

  // 3. prologue under the weight latency
  if constexpr (NSM > 0) {
    // merged 8-dim group j -> chunk m = 8j / EPC, planes q0, q0 + 1 of the staged layout
    for (int j = tid; j < NG; j += NT) {
      if (j != tid) merge_load<NSM>(a, j, ns, mi);
      float xm[8];
      merge_apply<NSM>(mi, ns, xm);
      const int m = (8 * j) / EPC, q0 = ((8 * j) % EPC) / 4;
      xs[q0 * KC + m] = make_float4(xm[0], xm[1], xm[2], xm[3]);
      xs[(q0 + 1) * KC + m] = make_float4(xm[4], xm[5], xm[6], xm[7]);
    }
    __syncthreads();
  }
  float scale = 1.f;
  if (NORM) {
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      if (tid + i * NT < KC) {
#pragma unroll
        for (int q = 0; q < PL; ++q)
          ss += xv[i][q].x * xv[i][q].x + xv[i][q].y * xv[i][q].y + xv[i][q].z * xv[i][q].z +
                xv[i][q].w * xv[i][q].w;
      }
    }
    ss = wave_sum(ss);
    if (lane == 0) red[wid] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < WPB; ++i) tot += red[i];
    scale = 1.0f / sqrtf(tot / (float)(KC * EPC) + a.eps);
  }
#pragma unroll
  for (int i = 0; i < XPT && NSM == 0; ++i) {
    const int m = tid + i * NT;
    if (m < KC) {
#pragma unroll
      for (int q = 0; q < PL; ++q) {
        float4 v = xv[i][q];
        if (NORM) {
          v.x = v.x * scale * nv[i][q].x; v.y = v.y * scale * nv[i][q].y;
          v.z = v.z * scale * nv[i][q].z; v.w = v.w * scale * nv[i][q].w;
        }
        xs[q * KC + m] = v;
      }
    }
  }
  __syncthreads();

  // 4. dot products (fp32 accumulate), wave butterfly
  float acc[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) acc[r] = 0.f;
#pragma unroll
  for (int c = 0; c < KCH; ++c) {
    float4 xq[PL];
#pragma unroll
    for (int q = 0; q < PL; ++q) xq[q] = xs[q * KC + c * 64 + lane];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      if (F8) {
        const uint32_t wd[4] = {w[r][c].x, w[r][c].y, w[r][c].z, w[r][c].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x2_t lo = __builtin_amdgcn_cvt_pk_f32_fp8(wd[q], false);
          const f32x2_t hi = __builtin_amdgcn_cvt_pk_f32_fp8(wd[q], true);
          acc[r] = fmaf(lo.x, xq[q].x, acc[r]);
          acc[r] = fmaf(lo.y, xq[q].y, acc[r]);
          acc[r] = fmaf(hi.x, xq[q].z, acc[r]);
          acc[r] = fmaf(hi.y, xq[q].w, acc[r]);
        }
      } else {
        acc[r] = dot8(w[r][c], xq[0], xq[1], acc[r]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    acc[r] = wave_sum(acc[r]);
    if (F8) acc[r] *= wsc[r];
  }
  if (!active || lane != 0) return;

  // 5. epilogues
  if (EPI == EPI_STORE) {
#pragma unroll
    for (int r = 0; r < RPW; ++r) a.Y[n0 + r] = acc[r];
  } else if (EPI == EPI_RESID) {
#pragma unroll
    for (int r = 0; r < RPW; ++r) a.Y[n0 + r] = res[r] + acc[r];
  } else if (EPI == EPI_SILU) {
#pragma unroll
    for (int r = 0; r < RPW; r += 2) {
      const float gt = acc[r], up = acc[r + 1];
      a.Y[(n0 + r) >> 1] = gt / (1.0f + expf(-gt)) * up;
    }
  } else if (EPI == EPI_QKV) {
    const int slot = a.row_slot[0], pos = a.row_pos[0];
#pragma unroll
    for (int r = 0; r < RPW; r += 2) {
      const int n = n0 + r;
      const int hh = n >> 7, within = n & 127, p = within >> 1;
      const float x1 = acc[r], x2 = acc[r + 1];
      if (hh < a.heads + a.kv_heads) {
        const float cs = a.rope_cos[(size_t)pos * 64 + p];
        const float sn = a.rope_sin[(size_t)pos * 64 + p];
        const float o1 = x1 * cs - x2 * sn;
        const float o2 = x2 * cs + x1 * sn;
        if (hh < a.heads) {
          float* q = a.Q + (size_t)hh * 128;
          q[p] = o1;
          q[p + 64] = o2;
        } else {
          uint16_t* k = a.kcache + ((size_t)slot * a.kv_heads + (hh - a.heads)) * a.max_pos * 128;
          k[kv_k_off(pos, p)] = f32_to_bf16(o1);
          k[kv_k_off(pos, p + 64)] = f32_to_bf16(o2);
        }
      } else {
        uint16_t* v = a.vcache +
            ((size_t)slot * a.kv_heads + (hh - a.heads - a.kv_heads)) * 128 * a.max_pos;
        v[kv_v_off(pos, within)] = f32_to_bf16(x1);
        v[kv_v_off(pos, within + 1)] = f32_to_bf16(x2);
      }
    }
  }
}

// ---------------------------------------------------------------------------------
// Decode / prefill attention on bf16 MFMA, one launch: split-KV partials + in-launch merge.
//   Grid (nsplit, kv_heads, R), block 256 = 4 waves; a wave owns CPW chunks of 32 positions
//   (split S = 128 * CPW), streaming them with an online softmax.  Per chunk:
//   * S^T = K Q^T with mfma_f32_16x16x32_bf16: A = K rows straight from the cache (16 B per
//     lane), B = the GRP q-heads of this kv-head (GQA 3:1), padded to 16 columns.  Q is
//     fp32; it enters as three bf16 parts q0 + q1 + q2 (24 mantissa bits), so the scores
//     are the fp32 products of the oracle up to summation order.  MFMA row r of tile T
//     holds position 8(r>>2) + 4T + (r&3): after the MFMA the lane (head h, group g) owns
//     the scores of positions 8g .. 8g+7, which is exactly its A fragment for P.V.
//   * O^T += P V with the same instruction: A = P (three bf16 parts, lane-local, no data
//     movement), B = V^T fragments.  The V cache chunks are stored in that fragment order (kv_v_off)
//     so a lane's B fragment (8 consecutive positions of one dim) is one 16-byte load.
//   Waves merge in LDS; with several splits the block publishes (m, l, acc) with
//   write-through (sc1) stores, takes a ticket on a per-(row, kv-head) counter and the last
//   arriver merges every split with sc1 loads (MI355X_MICROARCH.md "Valid forms", row 1),
//   then resets the counter for the next launch.
// ---------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// x = p0 + p1 + p2 with p_i bf16 (exact to fp32 rounding); 8 values -> three fragments
__device__ __forceinline__ void split3(const float* x, bf16x8& f0, bf16x8& f1, bf16x8& f2) {
  uint32_t w0[4], w1[4], w2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float a = x[2 * j], b = x[2 * j + 1];
    w0[j] = pack2_bf16(a, b);
    const float a1 = a - bf16_lo(w0[j]), b1 = b - bf16_hi(w0[j]);
    w1[j] = pack2_bf16(a1, b1);
    w2[j] = pack2_bf16(a1 - bf16_lo(w1[j]), b1 - bf16_hi(w1[j]));
  }
  f0 = __builtin_bit_cast(bf16x8, make_uint4(w0[0], w0[1], w0[2], w0[3]));
  f1 = __builtin_bit_cast(bf16x8, make_uint4(w1[0], w1[1], w1[2], w1[3]));
  f2 = __builtin_bit_cast(bf16x8, make_uint4(w2[0], w2[1], w2[2], w2[3]));
}

// One block = NW waves over S = 32 NW CPW positions of one (row, kv head); wave w takes the
// 32-position chunks w, w + NW, ... (CPW of them), with the next chunk's K / V^T loads in
// flight under the current chunk's MFMAs and softmax.  NW = 8, CPW = 4 covers
// 1,024 positions in one block, so a single-row step up to that length needs no split merge.
template <int GRP, int CPW, int NW>
__global__ __launch_bounds__(NW * 64) void attn_kernel(AttnArgs a) {
  constexpr int S = 32 * NW * CPW;
  constexpr int NT = NW * 64;
  constexpr int KM = (GRP * 128 + NT - 1) / NT;  // (head, dim) outputs per thread in merges
  const int split = blockIdx.x, kvh = blockIdx.y, r = blockIdx.z;
  const int L = a.row_pos[r] + 1;
  const int nsplit = (L + S - 1) / S;
  if (split >= nsplit) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int slot = a.row_slot[r];
  const size_t head = (size_t)slot * a.kv_heads + kvh;
  // K and V in fragment-major 32-position chunks (mx_common.h kv_k_off / kv_v_off): every
  // fragment load below is one lane-linear 1 KB run
  const uint4* Kf = reinterpret_cast<const uint4*>(a.kcache) + head * a.max_pos * 16;
  const uint4* Vf = reinterpret_cast<const uint4*>(a.vcache) + head * a.max_pos * 16;

  // K fragments (A operand): tile T, MFMA row rr -> position 8(rr>>2) + 4T + (rr&3);
  // V fragments (B operand): lane (dim 16 t + c, group g) <- positions base + 8g .. +8.
  // Positions of the last chunk at or past L hold stale (finite) cache data: their scores are
  // masked to -inf below, so their P is exactly 0.
  uint4 kf[2][2][4], vf[2][8];
  auto load_kv = [&](int base, int b) {
    const uint4* kc = Kf + (size_t)(base >> 5) * 512 + lane;
    const uint4* vc = Vf + (size_t)(base >> 5) * 512 + lane;
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
      for (int st = 0; st < 4; ++st) kf[b][T][st] = kc[(T * 4 + st) * 64];
#pragma unroll
    for (int t = 0; t < 8; ++t) vf[b][t] = vc[t * 64];
  };
  // chunks are dealt round-robin over the waves (wave w: chunks w, w + NW, ...), so a split
  // longer than the context still keeps every wave busy with ~equal work
  const int base0 = split * S + wid * 32;
  // (qkv_parts: the wave whose first chunk holds the new position loads it only after it has
  // appended that position, below)
  const bool late0 = a.qkv_parts != nullptr && base0 == ((L - 1) & ~31);
  if (base0 < L && !late0) load_kv(base0, 0);

  // Multi-row decode after the seam-free qkv GEMM (AttnArgs::qkv_parts): q, k and v of the new
  // position L - 1 are the sums of the qkv launch's K-range partials (range order), scaled by
  // the RMSNorm factor of the summed partial sums of squares, RoPE'd (q, k) -- the epilogue the
  // qkv GEMM's last arriving range ran before (rows_epilogue EPI_QKV).  Every split block
  // stages its q in LDS.  In the block whose split holds L - 1, the wave that will load the
  // chunk holding it computes that position's k / v and appends them to the cache itself, so
  // its own later loads of those addresses are ordered after the stores (one wave: program
  // order); if that chunk is its first one, its early load above was skipped (late0).
  const bool parts = a.qkv_parts != nullptr;
  __shared__ __attribute__((aligned(16))) float qs[GRP][128];
  if (parts) {
    const int N = a.qkv_n, NQ = a.heads * 128, KVD = a.kv_heads * 128, R = gridDim.z;
    const int pos = L - 1;
    // every range's loads issued at once (clamped addresses, fixed trip count), summed in
    // range order: a runtime loop here was one dependent round trip per range
    const int nk = a.qkv_nkc;
    float ssv[ATT_QKV_NKC_MAX];
#pragma unroll
    for (int kc = 0; kc < ATT_QKV_NKC_MAX; ++kc) ssv[kc] = a.qkv_ss[(size_t)min(kc, nk - 1) * R + r];
    float ss = 0.f;
#pragma unroll
    for (int kc = 0; kc < ATT_QKV_NKC_MAX; ++kc)
      if (kc < nk) ss += ssv[kc];
    const float scl = 1.0f / sqrtf(ss / (float)a.hidden + a.eps);
    auto pair = [&](int idx, float& x1, float& x2) {
      float2 v[ATT_QKV_NKC_MAX];
#pragma unroll
      for (int kc = 0; kc < ATT_QKV_NKC_MAX; ++kc)
        v[kc] = *reinterpret_cast<const float2*>(a.qkv_parts + ((size_t)min(kc, nk - 1) * R + r) * N + idx);
      x1 = 0.f;
      x2 = 0.f;
#pragma unroll
      for (int kc = 0; kc < ATT_QKV_NKC_MAX; ++kc) {
        if (kc < nk) {
          x1 += v[kc].x;
          x2 += v[kc].y;
        }
      }
      x1 *= scl;
      x2 *= scl;
    };
    // q: pair (h, p) -> dims p, p + 64 (the packed wqkv rows are pair-interleaved)
    for (int i = tid; i < GRP * 64; i += NT) {
      const int h = i >> 6, p = i & 63;
      float x1, x2;
      pair((kvh * GRP + h) * 128 + 2 * p, x1, x2);
      const float cs = a.rope_cos[(size_t)pos * 64 + p], sn = a.rope_sin[(size_t)pos * 64 + p];
      qs[h][p] = x1 * cs - x2 * sn;
      qs[h][p + 64] = x2 * cs + x1 * sn;
    }
    if (split == pos / S && wid == ((((pos & ~31) - split * S) >> 5) % NW)) {
      const int p = lane;  // k dims (p, p + 64); v dims (2p, 2p + 1)
      float k1, k2, v1, v2;
      pair(NQ + kvh * 128 + 2 * p, k1, k2);
      pair(NQ + KVD + kvh * 128 + 2 * p, v1, v2);
      const float cs = a.rope_cos[(size_t)pos * 64 + p], sn = a.rope_sin[(size_t)pos * 64 + p];
      uint16_t* kcw = const_cast<uint16_t*>(a.kcache) + head * a.max_pos * 128;
      uint16_t* vcw = const_cast<uint16_t*>(a.vcache) + head * a.max_pos * 128;
      kcw[kv_k_off(pos, p)] = f32_to_bf16(k1 * cs - k2 * sn);
      kcw[kv_k_off(pos, p + 64)] = f32_to_bf16(k2 * cs + k1 * sn);
      vcw[kv_v_off(pos, 2 * p)] = f32_to_bf16(v1);
      vcw[kv_v_off(pos, 2 * p + 1)] = f32_to_bf16(v2);
      if (late0) load_kv(base0, 0);
    }
    __syncthreads();
  }

  // Q^T fragments: lane (col c = head, group g) holds q[c][32 s + 8 g + j], 3 bf16 parts
  bf16x8 qf[3][4];
  {
    const int hq = c < GRP ? c : 0;
    const float* qb = a.Q + ((size_t)r * a.heads + kvh * GRP + hq) * 128 + 8 * g;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      float x[8];
      float4 lo, hi;
      if (parts) {  // (LDS-typed pointer: a generic one would make these flat loads)
        typedef const __attribute__((address_space(3))) f32x4 lds_f4;
        const f32x4 l4 = *(lds_f4*)(&qs[hq][32 * st + 8 * g]);
        const f32x4 h4 = *(lds_f4*)(&qs[hq][32 * st + 8 * g + 4]);
        lo = make_float4(l4[0], l4[1], l4[2], l4[3]);
        hi = make_float4(h4[0], h4[1], h4[2], h4[3]);
      } else {
        lo = *reinterpret_cast<const float4*>(qb + 32 * st);
        hi = *reinterpret_cast<const float4*>(qb + 32 * st + 4);
      }
      x[0] = lo.x; x[1] = lo.y; x[2] = lo.z; x[3] = lo.w;
      x[4] = hi.x; x[5] = hi.y; x[6] = hi.z; x[7] = hi.w;
      if (c >= GRP) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = 0.f;
      }
      split3(x, qf[0][st], qf[1][st], qf[2][st]);
    }
  }

  float M = -INFINITY, lsum = 0.f;
  f32x4 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // one chunk; false once the wave runs past the context (wave-uniform).  cb (the K / V
  // register buffer) must fold to a constant at every call site.
  auto chunk = [&](const int ch, const int cb) __attribute__((always_inline)) -> bool {
    const int base = base0 + ch * 32 * NW;
    if (base >= L) return false;
    if (ch + 1 < CPW && base + 32 * NW < L) load_kv(base + 32 * NW, cb ^ 1);
    __builtin_amdgcn_sched_barrier(0);
    // scores
    f32x4 sc[2];
#pragma unroll
    for (int T = 0; T < 2; ++T) {
      sc[T] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const bf16x8 kb = __builtin_bit_cast(bf16x8, kf[cb][T][st]);
#pragma unroll
        for (int pt = 0; pt < 3; ++pt)
          sc[T] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kb, qf[pt][st], sc[T], 0, 0, 0);
      }
    }
    // online softmax: this lane holds head c, positions base + 8g + j (j = 4T + i)
    float sv[8];
    float mc = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int p = base + 8 * g + j;
      sv[j] = p < L ? sc[j >> 2][j & 3] * a.scale : -INFINITY;
      mc = fmaxf(mc, sv[j]);
    }
    mc = fmaxf(mc, __shfl_xor(mc, 16, 64));
    mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
    const float Mn = fmaxf(M, mc);  // finite: position base < L is in this chunk
    const float alpha = expf(M - Mn);  // M = -inf on the first chunk -> 0
    float pv[8], ps = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      pv[j] = expf(sv[j] - Mn);
      ps += pv[j];
    }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    lsum = lsum * alpha + ps;
    M = Mn;
    // rescale O^T rows (row = head 4 g + i): alpha of head h lives in lane h
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float al = __shfl(alpha, (4 * g + i) & 15, 64);
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t][i] *= al;
    }
    bf16x8 pf[3];
    split3(pv, pf[0], pf[1], pf[2]);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const bf16x8 vb = __builtin_bit_cast(bf16x8, vf[cb][t]);
#pragma unroll
      for (int pt = 0; pt < 3; ++pt)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf[pt], vb, acc[t], 0, 0, 0);
    }
    return true;
  };
  if constexpr (CPW <= 4) {
#pragma unroll
    for (int ch = 0; ch < CPW; ++ch)
      if (!chunk(ch, ch & 1)) break;
  } else {
    // longer splits: a fully unrolled loop spills (CPW 6 / 8: 100 / 180 B scratch per lane);
    // a runtime loop whose body is the CPW = 4 sequence: CPW 6 fits, CPW 8 spills 20 B
#pragma unroll 1
    for (int ch = 0; ch < CPW; ch += 4) {
      if (!chunk(ch, 0)) break;
      if (ch + 1 >= CPW || !chunk(ch + 1, 1)) break;
      if (ch + 2 >= CPW || !chunk(ch + 2, 0)) break;
      if (ch + 3 >= CPW || !chunk(ch + 3, 1)) break;
    }
  }

  __shared__ __attribute__((aligned(16))) float wacc[NW][GRP][128];
  __shared__ float wml[NW][GRP][2];
  __shared__ float sml[ATT_MAX_SPLITS][GRP][2];
  __shared__ int last_s;
  // (M, lsum) of head c sit in lanes c (any g); O^T row h = 4 g + i, dim 16 t + c
  if (g == 0 && c < GRP) {
    wml[wid][c][0] = M;
    wml[wid][c][1] = lsum;
  }
  if (g == 0) {
#pragma unroll
    for (int i = 0; i < GRP && i < 4; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t) wacc[wid][i][16 * t + c] = acc[t][i];
  }
  __syncthreads();
  // block merge: thread -> outputs (head, dim) = idx / 128, idx % 128 for idx = tid + NT k
  float bm[KM], bl[KM], bn[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    bm[k] = bl[k] = bn[k] = 0.f;
    const int idx = tid + NT * k;
    if (idx < GRP * 128) {
      const int h = idx >> 7, td = idx & 127;
      float Mb = -INFINITY;
#pragma unroll
      for (int w = 0; w < NW; ++w) Mb = fmaxf(Mb, wml[w][h][0]);
      float num = 0.f, den = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const float mw = wml[w][h][0];
        const float f = (mw == -INFINITY) ? 0.f : expf(mw - Mb);
        num = fmaf(f, wacc[w][h][td], num);
        den = fmaf(f, wml[w][h][1], den);
      }
      bm[k] = Mb;
      bl[k] = den;
      bn[k] = num;
    }
  }
  float* out = a.out + ((size_t)r * a.heads + kvh * GRP) * 128;
  if (a.no_merge) {  // one-row step: the o-proj GEMV merges the splits in its prologue
    const size_t pb = ((size_t)r * a.kv_heads + kvh) * a.split_stride + split;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int idx = tid + NT * k;
      if (idx < GRP * 128) {
        const int h = idx >> 7, td = idx & 127;
        a.part_acc[(pb * GRP + h) * 128 + td] = bn[k];
        if (td == 0) {
          a.part_ml[(pb * GRP + h) * 2] = bm[k];
          a.part_ml[(pb * GRP + h) * 2 + 1] = bl[k];
        }
      }
    }
    return;
  }
  if (nsplit == 1) {
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int idx = tid + NT * k;
      if (idx < GRP * 128) out[idx] = bn[k] / bl[k];
    }
    return;
  }
  // publish this split's partial (write-through), then take a ticket
  const size_t pb = ((size_t)r * a.kv_heads + kvh) * a.split_stride;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int idx = tid + NT * k;
    if (idx < GRP * 128) {
      const int h = idx >> 7, td = idx & 127;
      st_wt(a.part_acc + ((pb + split) * GRP + h) * 128 + td, bn[k]);
      if (td == 0) {
        st_wt(a.part_ml + ((pb + split) * GRP + h) * 2, bm[k]);
        st_wt(a.part_ml + ((pb + split) * GRP + h) * 2 + 1, bl[k]);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    int* cnt = a.counter + (size_t)r * a.kv_heads + kvh;
    const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (t == nsplit - 1);
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_s = last;
  }
  __syncthreads();
  if (!last_s) return;
  // last arriver: the (m, l) pairs and this thread's accumulator columns of every split are
  // loaded in ONE round trip (ATT_MERGE_CHUNK splits at a time), then merged.
  for (int i = tid; i < nsplit * GRP * 2; i += NT)
    (&sml[0][0][0])[i] = ld_wt(a.part_ml + pb * GRP * 2 + i);
  float col[KM][ATT_MERGE_CHUNK];
  const int n0 = min(nsplit, ATT_MERGE_CHUNK);
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int idx = min(tid + NT * k, GRP * 128 - 1);
#pragma unroll
    for (int sp = 0; sp < ATT_MERGE_CHUNK; ++sp)
      col[k][sp] = ld_wt(a.part_acc + ((pb + min(sp, n0 - 1)) * GRP) * 128 + idx);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int idx = tid + NT * k;
    if (idx >= GRP * 128) continue;
    const int h = idx >> 7;
    float Mb = -INFINITY;
    for (int sp = 0; sp < nsplit; ++sp) Mb = fmaxf(Mb, sml[sp][h][0]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int sp = 0; sp < ATT_MERGE_CHUNK; ++sp) {
      if (sp < n0) {
        const float f = expf(sml[sp][h][0] - Mb);
        num = fmaf(f, col[k][sp], num);
        den = fmaf(f, sml[sp][h][1], den);
      }
    }
    for (int sp = ATT_MERGE_CHUNK; sp < nsplit; ++sp) {  // long contexts only
      const float f = expf(sml[sp][h][0] - Mb);
      num = fmaf(f, ld_wt(a.part_acc + ((pb + sp) * GRP) * 128 + idx), num);
      den = fmaf(f, sml[sp][h][1], den);
    }
    out[idx] = num / den;
  }
}

// ---------------------------------------------------------------------------------
// Commit: argmax key -> token; record history (host-mapped), mark seen, advance
// position, gather the next input embedding.  Grid R, block 256.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void commit_kernel(CommitArgs a) {
  const int r = blockIdx.x;
  const int dst = a.dst_row ? a.dst_row[r] : r;
  __shared__ int tok_s;
  if (threadIdx.x == 0) {
    const unsigned long long key = a.best[r];
    const int tok = (int)argmax_index(key);
    tok_s = tok;
    a.best[r] = 0ull;
    const int slot = a.row_slot[dst];
    const bool gave_up = a.abort_word &&
        __hip_atomic_load(a.abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    if (gave_up) {  // the step's outputs are invalid: no advance, the history slot reads -1,
                    // and h is the step's input again (the engine overwrites it in place)
      if (slot != a.scratch_slot)
        a.hist[(size_t)slot * a.max_pos + min(a.row_pos[dst] + a.pos_advance, a.max_pos - 1)] = -1;
      tok_s = a.row_token[dst];
    } else if (slot != a.scratch_slot) {  // parked rows stay at position 0 of the scratch slot
      const int pos = min(a.row_pos[dst] + a.pos_advance, a.max_pos - 1);  // new token
      a.row_pos[dst] = pos;
      a.row_token[dst] = tok;
      a.seen[(size_t)slot * a.vocab + tok] = 1;
      a.hist[(size_t)slot * a.max_pos + pos] = tok;
    }
  }
  __syncthreads();
  const int tok = tok_s;
  const uint4* e = reinterpret_cast<const uint4*>(a.embed + (size_t)tok * a.hidden);
  float4* h = reinterpret_cast<float4*>(a.h + (size_t)dst * a.hidden);
  for (int c = threadIdx.x; c < (a.hidden >> 3); c += 256) {
    const uint4 w = e[c];
    h[2 * c] = make_float4(bf16_lo(w.x), bf16_hi(w.x), bf16_lo(w.y), bf16_hi(w.y));
    h[2 * c + 1] = make_float4(bf16_lo(w.z), bf16_hi(w.z), bf16_lo(w.w), bf16_hi(w.w));
  }
}

// Prefill rows: h[r] = embed[ids[r]], seen[slot][ids[r]] = 1.  Grid R, block 256.
__global__ __launch_bounds__(256) void embed_rows_kernel(const int32_t* ids, int slot,
                                                         const uint16_t* embed, int hidden,
                                                         int vocab, uint8_t* seen, float* h) {
  const int r = blockIdx.x;
  const int tok = ids[r];
  if (threadIdx.x == 0) seen[(size_t)slot * vocab + tok] = 1;
  const uint4* e = reinterpret_cast<const uint4*>(embed + (size_t)tok * hidden);
  float4* out = reinterpret_cast<float4*>(h + (size_t)r * hidden);
  for (int c = threadIdx.x; c < (hidden >> 3); c += 256) {
    const uint4 w = e[c];
    out[2 * c] = make_float4(bf16_lo(w.x), bf16_hi(w.x), bf16_lo(w.y), bf16_hi(w.y));
    out[2 * c + 1] = make_float4(bf16_lo(w.z), bf16_hi(w.z), bf16_lo(w.w), bf16_hi(w.w));
  }
}

// Weight packing: source row i -> destination row dmap[i].  mode 0: bf16 -> bf16,
// 1: f32 -> bf16 (RNE), 2: bytes (fp8 e4m3) -> bytes.
__global__ void scatter_rows_kernel(void* dst, const void* src, const int32_t* dmap, int cols,
                                    int mode) {
  const int i = blockIdx.x;
  const size_t d = (size_t)dmap[i] * cols, s = (size_t)i * cols;
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    if (mode == 2) {
      static_cast<uint8_t*>(dst)[d + c] = static_cast<const uint8_t*>(src)[s + c];
    } else {
      const uint16_t v = mode == 1 ? f32_to_bf16(static_cast<const float*>(src)[s + c])
                                   : static_cast<const uint16_t*>(src)[s + c];
      static_cast<uint16_t*>(dst)[d + c] = v;
    }
  }
}

// Row compaction: the stream decoded by row `src` continues in row `dst` (its KV slot, position,
// current token and next input embedding move; `src` is parked on the scratch slot).
__global__ void move_row_kernel(int32_t* slot, int32_t* pos, int32_t* token, float* h, int hidden,
                                int dst, int src, int scratch) {
  const float4* s4 = reinterpret_cast<const float4*>(h + (size_t)src * hidden);
  float4* d4 = reinterpret_cast<float4*>(h + (size_t)dst * hidden);
  for (int c = threadIdx.x; c < (hidden >> 2); c += blockDim.x) d4[c] = s4[c];
  if (threadIdx.x == 0) {
    slot[dst] = slot[src];
    pos[dst] = pos[src];
    token[dst] = token[src];
    slot[src] = scratch;
    pos[src] = 0;
  }
}

hipError_t launch_move_row(int32_t* slot, int32_t* pos, int32_t* token, float* h, int hidden,
                           int dst, int src, int scratch, hipStream_t st) {
  hipLaunchKernelGGL(move_row_kernel, dim3(1), dim3(256), 0, st, slot, pos, token, h, hidden, dst,
                     src, scratch);
  return hipGetLastError();
}

// rows [0,n): slot[i] = slot_val, pos[i] = pos0 + i
__global__ void set_rows_kernel(int32_t* slot, int32_t* pos, int n, int slot_val, int pos0) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    slot[i] = slot_val;
    pos[i] = pos0 + i;
  }
}
__global__ void set_scalar_kernel(float* p, float v) { *p = v; }

hipError_t launch_set_rows(int32_t* slot, int32_t* pos, int n, int slot_val, int pos0,
                           hipStream_t st) {
  hipLaunchKernelGGL(set_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, st, slot, pos, n,
                     slot_val, pos0);
  return hipGetLastError();
}
hipError_t launch_set_scalar(float* p, float v, hipStream_t st) {
  hipLaunchKernelGGL(set_scalar_kernel, dim3(1), dim3(1), 0, st, p, v);
  return hipGetLastError();
}

__global__ void to_f32_kernel(float* dst, const void* src, int64_t n, int src_bf16) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dst[i] = src_bf16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(src)[i])
                    : reinterpret_cast<const float*>(src)[i];
}

// ---------------------------------------------------------------------------------
// Host-side launchers
// ---------------------------------------------------------------------------------
template <int RT, int RPW, int EPI, bool NORM, bool F8 = false>
static hipError_t launch_gemv_t(const GemvArgs& a, int blocks, hipStream_t st) {
  const size_t lds = (size_t)RT * a.K * 4 + 64;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int ytiles = (a.R + RT - 1) / RT;
  hipLaunchKernelGGL((gemv_kernel<RT, RPW, EPI, NORM, F8>), dim3(blocks, ytiles), dim3(256), lds, st, a);
  return hipGetLastError();
}

static int gemv_blocks(int N, int rpw, int ytiles, int target) {
  const int groups = (N + rpw - 1) / rpw;
  int b = (groups + 3) / 4;
  const int cap = (target + ytiles - 1) / ytiles;
  return b < cap ? b : (cap > 0 ? cap : 1);
}

// Option gemv_balance (GemvArgs::gemv_cus = the CU count): the waves per block whose grid puts
// the fewest waves -- i.e. weight bytes -- on the most loaded CU.  A one-row GEMV streams each
// CU's share at the CU's own fetch rate (MI355X_MICROARCH.md: prologue burst ~11 B/cycle/CU),
// so a grid of 640 blocks on 256 CUs (2 or 3 blocks per CU) runs as long as 3 blocks.
static int gemv_wpb_balanced(int G, int cus, std::initializer_list<int> cand) {
  int best = 0, best_w = 1 << 30;
  for (int w : cand) {
    const int blocks = (G + w - 1) / w;
    const int per_cu = (blocks + cus - 1) / cus * w;
    if (per_cu < best_w) {
      best = w;
      best_w = per_cu;
    }
  }
  return best;
}

template <int KCH, int RPW, int EPI, bool NORM, bool F8>
static hipError_t launch_gemv1_t(const GemvArgs& a, hipStream_t st) {
  const int G = a.N / RPW;
  if constexpr (EPI == EPI_RESID && !NORM && (F8 ? (KCH == 1 || KCH == 3)
                                                 : (KCH == 1 || KCH == 2 || KCH == 6))) {
    if (a.att_ml) {  // R = 1 o-projection with the attention split merge (8- or 6-wave blocks)
      const int ns = a.att_nsm;
      if (ns > 8 || (KCH * 64 * (F8 ? 16 : 8)) / 8 > 512) return hipErrorInvalidValue;
      if (a.gemv_cus > 0 && gemv_wpb_balanced(G, a.gemv_cus, {8, 6}) == 6) {
        const dim3 grid((G + 5) / 6), blk(384);
        if (ns <= 2) hipLaunchKernelGGL((gemv1_kernel<KCH, RPW, EPI, NORM, 6, F8, 2>), grid, blk, 0, st, a);
        else if (ns <= 4) hipLaunchKernelGGL((gemv1_kernel<KCH, RPW, EPI, NORM, 6, F8, 4>), grid, blk, 0, st, a);
        else hipLaunchKernelGGL((gemv1_kernel<KCH, RPW, EPI, NORM, 6, F8, 8>), grid, blk, 0, st, a);
        return hipGetLastError();
      }
      const dim3 grid((G + 7) / 8), blk(512);
      if (ns <= 2) hipLaunchKernelGGL((gemv1_kernel<KCH, RPW, EPI, NORM, 8, F8, 2>), grid, blk, 0, st, a);
      else if (ns <= 4) hipLaunchKernelGGL((gemv1_kernel<KCH, RPW, EPI, NORM, 8, F8, 4>), grid, blk, 0, st, a);
      else hipLaunchKernelGGL((gemv1_kernel<KCH, RPW, EPI, NORM, 8, F8, 8>), grid, blk, 0, st, a);
      return hipGetLastError();
    }
  }
  if (a.att_ml) return hipErrorNotSupported;
  if constexpr (EPI == EPI_QKV) {
    if (a.gemv_cus > 0 && gemv_wpb_balanced(G, a.gemv_cus, {4, 5, 8}) == 5) {
      hipLaunchKernelGGL((gemv1_kernel<KCH, RPW, EPI, NORM, 5, F8>), dim3((G + 4) / 5), dim3(320), 0, st, a);
      return hipGetLastError();
    }
  }
  if (a.wpb == 8)
    hipLaunchKernelGGL((gemv1_kernel<KCH, RPW, EPI, NORM, 8, F8>), dim3((G + 7) / 8), dim3(512), 0, st, a);
  else
    hipLaunchKernelGGL((gemv1_kernel<KCH, RPW, EPI, NORM, 4, F8>), dim3((G + 3) / 4), dim3(256), 0, st, a);
  return hipGetLastError();
}

// B = 1 path; returns hipErrorNotSupported when the shape has no instantiation.
// a.rpw (0 = default per epilogue) picks rows per wave: QKV 2, RESID/STORE 1, SILU 2 (e4m3 4).
// KCH = 16-byte weight chunks per lane per row: K / 512 (bf16) or K / 1024 (fp8).
static hipError_t launch_gemv1(const GemvArgs& a, int epi, bool norm, hipStream_t st) {
  const bool f8 = a.wdtype == WT_FP8;
  const int epc = f8 ? 1024 : 512;
  if (a.K % epc) return hipErrorNotSupported;
  const int kch = a.K / epc;
  int rpw = a.rpw;
  // e4m3 gate/up: 4 rows per wave (12 loads of 16 B per lane, not 6): step 1.106 -> 1.099 ms
  // at L 600 (profiles/r04_rows_per_wave_ab.log); bf16 is unchanged by it (1.528 / 1.525)
  if (rpw == 0) rpw = epi == EPI_QKV ? 2 : epi == EPI_SILU ? (f8 ? 4 : 2) : 1;
#define MX_G1(KCH_, RPW_, EPI_, NORM_)                                                  \
  if (kch == KCH_ && rpw == RPW_ && epi == EPI_ && norm == NORM_ && a.N % RPW_ == 0)     \
    return f8 ? launch_gemv1_t<KCH_, RPW_, EPI_, NORM_, true>(a, st)                    \
              : launch_gemv1_t<KCH_, RPW_, EPI_, NORM_, false>(a, st);
#define MX_G1K(KCH_)                                                                     \
  MX_G1(KCH_, 2, EPI_QKV, true) MX_G1(KCH_, 1, EPI_RESID, false)                       \
  MX_G1(KCH_, 2, EPI_RESID, false)                                                      \
  MX_G1(KCH_, 2, EPI_SILU, true) MX_G1(KCH_, 4, EPI_SILU, true)                         \
  MX_G1(KCH_, 1, EPI_STORE, false) MX_G1(KCH_, 1, EPI_STORE, true)
  MX_G1K(1) MX_G1K(2) MX_G1K(3) MX_G1K(4) MX_G1K(6) MX_G1K(8) MX_G1K(16)
#undef MX_G1K
#undef MX_G1
  return hipErrorNotSupported;
}

hipError_t launch_gemv(const GemvArgs& a, int epi, bool norm, hipStream_t st) {
  if (a.R == 1 && epi != EPI_ARGMAX && !a.force_legacy) {
    const hipError_t e = launch_gemv1(a, epi, norm, st);
    if (e != hipErrorNotSupported || a.att_ml) return e;  // (the merge has no other kernel)
  }
  if (a.R == 1 && epi == EPI_ARGMAX && norm && a.head_b1 && !a.force_legacy) {
    const hipError_t e = launch_head_b1(a, st);
    if (e != hipErrorNotSupported) return e;
  }
  // fp8 single-row lm_head: the grid-stride argmax GEMV with e4m3 weights
  // (8 rows per wave: an e4m3 row is 3 KB, so 4 rows left a wave only 12 loads of 16 B in
  // flight; measured 106.8 us = 4.5 TB/s at 4 rows)
  if (a.R == 1 && epi == EPI_ARGMAX && norm && a.wdtype == WT_FP8 && a.K % 1024 == 0) {
    const int blocks = gemv_blocks(a.N, 8, 1, a.max_blocks > 0 ? a.max_blocks : 4096);
    return launch_gemv_t<1, 8, EPI_ARGMAX, true, true>(a, blocks, st);
  }
  // multi-row steps (and any other fp8 shape) run on the MFMA kernel
  if ((a.R >= 2 && !a.force_legacy) || a.wdtype == WT_FP8) {
    const hipError_t e = v4::launch_gemm_rows_v4(a, epi, norm, st);
    if (e != hipErrorNotSupported || a.wdtype == WT_FP8) return e;
  }
  // RT = 1 for the decode batch of 1; RT = 4 otherwise (prefill / batched decode).
  const int RT = a.R == 1 ? 1 : 4;
  const int ytiles = (a.R + RT - 1) / RT;
  const int rpw = (epi == EPI_ARGMAX) ? 4 : 2;
  const int blocks = gemv_blocks(a.N, rpw, ytiles, a.max_blocks > 0 ? a.max_blocks : 4096);
#define MX_G(RT_, RPW_, EPI_, NORM_)                                 \
  if (RT == RT_ && rpw == RPW_ && epi == EPI_ && norm == NORM_)      \
    return launch_gemv_t<RT_, RPW_, EPI_, NORM_>(a, blocks, st);
  MX_G(1, 2, EPI_STORE, false) MX_G(1, 2, EPI_STORE, true)
  MX_G(1, 2, EPI_RESID, false) MX_G(1, 2, EPI_SILU, true)
  MX_G(1, 2, EPI_QKV, true) MX_G(1, 4, EPI_ARGMAX, true)
  MX_G(4, 2, EPI_STORE, false) MX_G(4, 2, EPI_STORE, true)
  MX_G(4, 2, EPI_RESID, false) MX_G(4, 2, EPI_SILU, true)
  MX_G(4, 2, EPI_QKV, true) MX_G(4, 4, EPI_ARGMAX, true)
#undef MX_G
  return hipErrorInvalidValue;
}

// Allow > 64 KiB of dynamic LDS where an instantiation needs it (RT = 4 tiles at
// K = ffn stage RT*K*4 bytes).  The request is sized per instantiation: dynamic + static
// LDS must stay within the 160 KiB of a CU, so asking for the whole 160 KiB on a kernel
// that also declares static __shared__ (the argmax epilogue) is rejected.  Called once per
// context, outside any graph capture.
hipError_t gemv_prepare(int kmax) {
  hipError_t e = hipSuccess;
#define MX_A(RT_, RPW_, EPI_, NORM_)                                                          \
  if (e == hipSuccess) {                                                                      \
    const int need = RT_ * kmax * 4 + 64;                                                     \
    if (need > 64 * 1024)                                                                     \
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemv_kernel<RT_, RPW_, EPI_, NORM_>), \
                              hipFuncAttributeMaxDynamicSharedMemorySize, need);              \
  }
  MX_A(1, 2, EPI_STORE, false) MX_A(1, 2, EPI_STORE, true)
  MX_A(1, 2, EPI_RESID, false) MX_A(1, 2, EPI_SILU, true)
  MX_A(1, 2, EPI_QKV, true) MX_A(1, 4, EPI_ARGMAX, true)
  MX_A(4, 2, EPI_STORE, false) MX_A(4, 2, EPI_STORE, true)
  MX_A(4, 2, EPI_RESID, false) MX_A(4, 2, EPI_SILU, true)
  MX_A(4, 2, EPI_QKV, true) MX_A(4, 4, EPI_ARGMAX, true)
#undef MX_A
  if (e == hipSuccess && kmax * 4 + 64 > 64 * 1024)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemv_kernel<1, 8, EPI_ARGMAX, true, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, kmax * 4 + 64);
  return e;
}

hipError_t launch_attention(const AttnArgs& a, int R, int max_len, hipStream_t st) {
  const int nw = (a.nw == 8 || a.nw == 6 || a.nw == 3 || a.nw == 2) ? a.nw : 4;
  const int S = 32 * nw * a.cpw;
  const int nsplit = (max_len + S - 1) / S;
  if (nsplit > ATT_MAX_SPLITS || (a.max_pos + S - 1) / S > a.split_stride || a.max_pos % 8)
    return hipErrorInvalidValue;
  const dim3 grid(nsplit, a.kv_heads, R);
#define MX_AT(G_, C_, W_)                                                            \
  if (a.heads / a.kv_heads == G_ && a.cpw == C_ && nw == W_) {                       \
    hipLaunchKernelGGL((attn_kernel<G_, C_, W_>), grid, dim3(64 * W_), 0, st, a);    \
    return hipGetLastError();                                                        \
  }
#define MX_ATG(G_) MX_AT(G_, 1, 2) MX_AT(G_, 1, 3) MX_AT(G_, 2, 3) MX_AT(G_, 1, 4) MX_AT(G_, 2, 4) MX_AT(G_, 4, 4) \
                   MX_AT(G_, 1, 6) MX_AT(G_, 2, 6) MX_AT(G_, 3, 6) \
                   MX_AT(G_, 1, 8) MX_AT(G_, 2, 8) MX_AT(G_, 3, 8) MX_AT(G_, 4, 8) \
                   MX_AT(G_, 6, 8) MX_AT(G_, 8, 8)
  MX_ATG(1) MX_ATG(2) MX_ATG(3) MX_ATG(4)
#undef MX_ATG
#undef MX_AT
  return hipErrorInvalidValue;
}

hipError_t launch_commit(const CommitArgs& a, int R, hipStream_t st) {
  hipLaunchKernelGGL(commit_kernel, dim3(R), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_embed_rows(const int32_t* ids, int n, int slot, const uint16_t* embed,
                             int hidden, int vocab, uint8_t* seen, float* h, hipStream_t st) {
  hipLaunchKernelGGL(embed_rows_kernel, dim3(n), dim3(256), 0, st, ids, slot, embed, hidden,
                     vocab, seen, h);
  return hipGetLastError();
}

hipError_t launch_scatter_rows(void* dst, const void* src, const int32_t* dmap, int rows,
                               int cols, int mode, hipStream_t st) {
  hipLaunchKernelGGL(scatter_rows_kernel, dim3(rows), dim3(256), 0, st, dst, src, dmap, cols, mode);
  return hipGetLastError();
}

// Fragment-major copy of an [N][K] weight matrix for the multi-row GEMM: 128-k sub-chunks, then
// 16-row tiles (bf16; e4m3: tiles, then sub-chunks), then the WL = 2 esz load instructions of
// a sub-chunk, then the 64 lanes;
// lane (c, g) of instruction l holds row 16 t + c, bytes 16 (4 l + g) of the sub-chunk (the
// same values the row-major addressing gives that lane).  Rows past N repeat row N - 1.
__global__ void frag_major_kernel(const uint4* src, uint4* dst, int N, int K, int esz) {
  const int WL = 2 * esz, S = K / 128;
  const int64_t total = (int64_t)((N + 15) / 16) * S * WL * 64;
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= total) return;
  const int lane = (int)(u & 63);
  const int64_t q = u >> 6;  // instruction index
  const int l = (int)(q % WL);
  const int64_t ts = q / WL;
  // bf16: [sub-chunk][tile] order; e4m3: [tile][sub-chunk] (mx_rows_v4.inc wbase)
  const int64_t T = (N + 15) / 16;
  const int64_t t = esz == 2 ? ts % T : ts / S;
  const int s = (int)(esz == 2 ? ts / T : ts % S);
  const int row = (int)min<int64_t>(16 * t + (lane & 15), N - 1);
  const int64_t row_units = (int64_t)K * esz / 16;
  dst[u] = src[(int64_t)row * row_units + (int64_t)s * (8 * esz) + 4 * l + (lane >> 4)];
}

hipError_t launch_frag_major(const void* src, void* dst, int N, int K, int esz, hipStream_t st) {
  if (K % 128 || (esz != 1 && esz != 2)) return hipErrorInvalidValue;
  const int64_t total = (int64_t)((N + 15) / 16) * (K / 128) * 2 * esz * 64;
  hipLaunchKernelGGL(frag_major_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     static_cast<const uint4*>(src), static_cast<uint4*>(dst), N, K, esz);
  return hipGetLastError();
}

hipError_t launch_to_f32(float* dst, const void* src, int64_t n, int src_bf16, hipStream_t st) {
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(to_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, st, dst, src, n, src_bf16);
  return hipGetLastError();
}


}  // namespace mx
