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

namespace mx {

// ---------------------------------------------------------------------------------
// Weight-streaming GEMV with fused prologue (RMSNorm) and epilogues.
//   y[r][n] = sum_k W[n][k] * xn[r][k]   for r in the block's RT activation rows.
// Grid: x = row-group workers (grid-stride over N / RPW groups, one wave per group),
//       y = ceil(R / RT) activation-row tiles.
// ---------------------------------------------------------------------------------
template <int RT, int RPW, int EPI, bool NORM>
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
      wp[i] = reinterpret_cast<const uint4*>(a.W + (size_t)n * a.K);
    }
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
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[i][rt] = wave_sum(acc[i][rt]);

    // ---- epilogues (every lane holds every total; lane 0 writes) -----------------------
    if (EPI == EPI_ARGMAX) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        if (rt < nr) {
          const int slot = a.row_slot[r0 + rt];
          const uint8_t* seen = a.seen + (size_t)slot * a.N;
          const float pen = a.penalty[0];
#pragma unroll
          for (int i = 0; i < RPW; ++i) {
            const int n = n0 + i;
            if (n < a.N) {
              float v = acc[i][rt];
              if (seen[n]) v = v > 0.f ? v / pen : v * pen;
              if (a.logits && lane == 0) a.logits[(size_t)(r0 + rt) * a.N + n] = v;
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
                    (((size_t)slot * a.kv_heads + (hh - a.heads)) * a.max_pos + pos) * 128;
                k[p] = f32_to_bf16(o1);
                k[p + 64] = f32_to_bf16(o2);
              }
            } else {
              uint16_t* v = a.vcache +
                  (((size_t)slot * a.kv_heads + (hh - a.heads - a.kv_heads)) * a.max_pos + pos) * 128;
              v[within] = f32_to_bf16(x1);
              v[within + 1] = f32_to_bf16(x2);
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
// Split-KV decode attention, GQA group of (heads / kv_heads) q-heads per kv-head.
// Grid (nsplit, kv_heads, R); block 256.  Split = ATT_CHUNK positions.
// K rows are 256 contiguous bytes: 16 lanes x 16 B per position, 4 positions per
// wave-instruction.  Partial (m, l, acc[128]) per (row, q-head, split).
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_partial_kernel(AttnArgs a) {
  const int split = blockIdx.x, kvh = blockIdx.y, r = blockIdx.z;
  const int pos = a.row_pos[r], L = pos + 1;
  const int s0 = split * ATT_CHUNK;
  if (s0 >= L) return;
  const int n = min(ATT_CHUNK, L - s0);
  const int slot = a.row_slot[r];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = a.heads / a.kv_heads;  // 3 for Orpheus
  __shared__ __attribute__((aligned(16))) float qs[ATT_MAXG][128];
  __shared__ float sc[ATT_MAXG][ATT_CHUNK];

  for (int i = tid; i < grp * 128; i += 256)
    qs[i >> 7][i & 127] = a.Q[((size_t)r * a.heads + kvh * grp) * 128 + i];
  __syncthreads();

  const size_t base = ((size_t)slot * a.kv_heads + kvh) * a.max_pos;
  const uint16_t* K = a.kcache + base * 128;
  const uint16_t* V = a.vcache + base * 128;
  const int sub = lane >> 4, d8 = (lane & 15) * 8;
  const float scale = a.scale;
  // scores: wave wid covers positions [wid*16, wid*16+16) of the chunk
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int j = wid * 16 + it * 4 + sub;
    const bool ok = j < n;
    uint4 kv = make_uint4(0, 0, 0, 0);
    if (ok) kv = *reinterpret_cast<const uint4*>(K + (size_t)(s0 + j) * 128 + d8);
    for (int h = 0; h < grp; ++h) {
      const float4 lo = *reinterpret_cast<const float4*>(&qs[h][d8]);
      const float4 hi = *reinterpret_cast<const float4*>(&qs[h][d8 + 4]);
      float d = dot8(kv, lo, hi, 0.f);
      d = group_sum<16>(d);
      if ((lane & 15) == 0) sc[h][j] = ok ? d * scale : -INFINITY;
    }
  }
  __syncthreads();
  // softmax partial per head (wave h handles head h; 64 lanes <-> 64 positions)
  if (wid < grp) {
    const float v = sc[wid][lane];
    const float m = wave_max(v);
    const float e = lane < n ? expf(v - m) : 0.f;
    const float l = wave_sum(e);
    sc[wid][lane] = e;
    if (lane == 0) {
      float* ml = a.part_ml + (((size_t)r * a.heads + kvh * grp + wid) * a.nsplit_max + split) * 2;
      ml[0] = m;
      ml[1] = l;
    }
  }
  __syncthreads();
  // P.V: wave h -> head h, lane -> two output dims (4-byte bf16x2 loads, 256 B per position)
  if (wid < grp) {
    float o0 = 0.f, o1 = 0.f;
    const int d2 = lane * 2;
    for (int j = 0; j < n; ++j) {
      const uint32_t vv = *reinterpret_cast<const uint32_t*>(V + (size_t)(s0 + j) * 128 + d2);
      const float p = sc[wid][j];
      o0 = fmaf(p, bf16_lo(vv), o0);
      o1 = fmaf(p, bf16_hi(vv), o1);
    }
    float* acc = a.part_acc + (((size_t)r * a.heads + kvh * grp + wid) * a.nsplit_max + split) * 128;
    *reinterpret_cast<float2*>(acc + d2) = make_float2(o0, o1);
  }
}

// Combine split partials -> attention output row [heads*128].  Grid (heads, R), block 128.
__global__ __launch_bounds__(128) void attn_combine_kernel(AttnArgs a) {
  const int h = blockIdx.x, r = blockIdx.y, d = threadIdx.x;
  const int L = a.row_pos[r] + 1;
  const int ns = (L + ATT_CHUNK - 1) / ATT_CHUNK;
  const size_t b = ((size_t)r * a.heads + h) * a.nsplit_max;
  float M = -INFINITY;
  for (int s = 0; s < ns; ++s) M = fmaxf(M, a.part_ml[(b + s) * 2]);
  float den = 0.f, num = 0.f;
  for (int s = 0; s < ns; ++s) {
    const float w = expf(a.part_ml[(b + s) * 2] - M);
    den = fmaf(w, a.part_ml[(b + s) * 2 + 1], den);
    num = fmaf(w, a.part_acc[(b + s) * 128 + d], num);
  }
  a.out[((size_t)r * a.heads + h) * 128 + d] = num / den;
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
    const int pos = a.row_pos[dst] + a.pos_advance;  // position of the new token
    a.row_pos[dst] = pos;
    a.row_token[dst] = tok;
    a.seen[(size_t)slot * a.vocab + tok] = 1;
    if (pos < a.max_pos) a.hist[(size_t)slot * a.max_pos + pos] = tok;
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

// Row permutation copy used to pack weights (dst row i <- src row perm[i]); converts
// f32 sources to bf16 when src_f32.
__global__ void pack_rows_kernel(uint16_t* dst, const void* src, const int32_t* perm,
                                 int cols, int src_f32) {
  const int i = blockIdx.x;
  const int s = perm[i];
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    uint16_t v;
    if (src_f32) v = f32_to_bf16(reinterpret_cast<const float*>(src)[(size_t)s * cols + c]);
    else v = reinterpret_cast<const uint16_t*>(src)[(size_t)s * cols + c];
    dst[(size_t)i * cols + c] = v;
  }
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
template <int RT, int RPW, int EPI, bool NORM>
static hipError_t launch_gemv_t(const GemvArgs& a, int blocks, hipStream_t st) {
  const size_t lds = (size_t)RT * a.K * 4 + 64;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int ytiles = (a.R + RT - 1) / RT;
  hipLaunchKernelGGL((gemv_kernel<RT, RPW, EPI, NORM>), dim3(blocks, ytiles), dim3(256), lds, st, a);
  return hipGetLastError();
}

static int gemv_blocks(int N, int rpw, int ytiles, int target) {
  const int groups = (N + rpw - 1) / rpw;
  int b = (groups + 3) / 4;
  const int cap = (target + ytiles - 1) / ytiles;
  return b < cap ? b : (cap > 0 ? cap : 1);
}

hipError_t launch_gemv(const GemvArgs& a, int epi, bool norm, hipStream_t st) {
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
  return e;
}

hipError_t launch_attention(const AttnArgs& a, int R, hipStream_t st) {
  hipLaunchKernelGGL(attn_partial_kernel, dim3(a.nsplit_max, a.kv_heads, R), dim3(256), 0, st, a);
  hipLaunchKernelGGL(attn_combine_kernel, dim3(a.heads, R), dim3(128), 0, st, a);
  return hipGetLastError();
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

hipError_t launch_pack_rows(uint16_t* dst, const void* src, const int32_t* perm, int rows,
                            int cols, int src_f32, hipStream_t st) {
  hipLaunchKernelGGL(pack_rows_kernel, dim3(rows), dim3(256), 0, st, dst, src, perm, cols, src_f32);
  return hipGetLastError();
}

hipError_t launch_to_f32(float* dst, const void* src, int64_t n, int src_bf16, hipStream_t st) {
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(to_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, st, dst, src, n, src_bf16);
  return hipGetLastError();
}

}  // namespace mx
