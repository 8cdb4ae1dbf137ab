// One-launch decode step for ONE row (B = 1, the configs[1] single stream), MI355X (gfx950).
//
// Replaces, for one stream, the per-token forward of vLLM AsyncLLMEngine.generate
// (Orpheus-TTS/orpheus_tts_pypi/orpheus_tts/engine_class.py:117) / llama.cpp
// Llama.text_to_speech (Morpheus_Client/tts_engine/llama_local.py:77): per layer RMSNorm ->
// QKV + RoPE + KV append -> GQA attention -> O-proj + residual -> RMSNorm -> gate/up + SiLU*up
// -> down + residual; final norm -> lm_head + repetition penalty + argmax -> commit.
//
// Why: at B = 1 the step is a 6.6 GB weight stream cut into ~140 dependent GEMVs.  As separate
// launches each one ramps up and drains (measured: qkv 3.9 TB/s, o-proj 2.8, down 4.7, gate/up
// 5.7 TB/s; profiles/r03_trace_b1_*.txt) -- the weights of launch k+1 cannot start streaming
// until launch k has drained.  Weights never depend on activations, so here every GEMV block
// issues its weight loads FIRST, then waits for its input vector, then computes.
//
// Structure: a DATAFLOW grid, not a persistent one.  Block b's role is a pure function of b:
//   layer l: [qkv x NQ][attention x kvh*nsplit][o x NO][gate/up x NG][down x ND], then the
//   lm_head blocks, then one finish block.  A block waits only on counters that blocks with a
//   SMALLER index increment, and workgroups are dispatched in index order, so every block it
//   waits on is resident or done: the grid cannot deadlock, and no co-residency or grid barrier
//   is needed.  While the blocks of stage s finish, the resident blocks of stages s+1, s+2 ...
//   already have their weights in flight (up to 4-5 blocks x 48-64 KB per CU), so HBM keeps
//   streaming across every stage seam.  Every wait is bounded: a give-up sets a status word,
//   the rest of the grid runs through without waiting (results invalid, the host raises).
//
// Hand-offs (MI355X_MICROARCH.md "Valid forms", row 1): producers store their outputs with
// write-through (sc1) stores, every storing wave drains (s_waitcnt vmcnt(0)), the block meets at
// a barrier, one lane adds to an agent-scope counter; the consumer's wave 0 polls the counter
// (sc1 loads, sharded counters summed across lanes), the block meets at a barrier and every
// wave reads the vector with sc1 loads.  Every hand-off element is written at most once per
// launch (the residual stream has one buffer per layer and stage: hd[l], ho[l]), so no XCD L2
// can hold a stale copy of a line read earlier in the same launch.  Counters are zeroed by the
// finish block (the last block: everything else has passed its waits).
//
// Precision: as the per-kernel step: fp32 activations / accumulation, bf16 or
// e4m3 + row-scale weights, bf16 KV cache (RNE), fp32 logits.  RMSNorm is folded as
// y = (W (x . w)) * rsqrt(mean x^2 + eps).  Attention runs on VALU in fp32 (B = 1 needs ~1
// MFLOP per kv-head and layer): split partials (m, l, acc) over 64-position splits of the old
// positions, merged by the last-arriving split together with the new position's k / v.
#include "mx_common.h"
#include "mx_llm_kernels.h"
#include "mx_step.h"

namespace mx {
namespace step {

constexpr int NT = 256;           // threads per block, every role
constexpr int SPIN = 1 << 20;     // polls (s_sleep 2 between) before a wait gives up
// per-layer counter slots (each STEP_CS ints apart)
constexpr int C_QKV = 0;          // [kvh <= 8] qkv blocks done, per kv-head group
constexpr int C_ATK = 8;          // [kvh] attention split tickets
constexpr int C_ATT = 16;         // merged kv-heads
constexpr int C_O = 17;           // [8 shards] o-proj blocks
constexpr int C_GU = 25;          // [8 shards] gate/up blocks
constexpr int C_DN = 33;          // [8 shards] down blocks
static_assert(C_DN + 8 <= STEP_LAYER_CNT, "counter layout");

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_wt_i(const int* p) {
  return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-byte write-through (sc1) load, idx in floats
__device__ __forceinline__ float4 ld4_wt(const float* base, size_t idx) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff, 0x00020000);
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(idx * 4), 0, 16);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                     __uint_as_float(v.w));
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// Wave-uniform bounded wait: sum of `nsh` counter shards (STEP_CS apart) >= target.
__device__ __noinline__ void wait_for(const int* c, int nsh, int target, int* status, int code) {
  const int lane = threadIdx.x & 63;
  for (int it = 0; it < SPIN; ++it) {
    const int v = wave_sum_i(lane < nsh ? ld_wt_i(c + lane * STEP_CS) : 0);
    if (__builtin_amdgcn_readfirstlane(v) >= target) return;
    if ((it & 15) == 15 && __builtin_amdgcn_readfirstlane(ld_wt_i(status)) != 0) return;
    __builtin_amdgcn_s_sleep(2);
  }
  if (lane == 0) atomicCAS(status, 0, code);
}
// Publish: every wave's write-through stores have left the CU, then one arrival.
__device__ __forceinline__ void signal(int* c) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------------
// GEMV block: 4 waves, RPW consecutive weight rows per wave over the whole K = 64 KCH EPC.
// Load order: weights (non-temporal, 16 B per lane, 1 KB per instruction), norm weights,
// then wave 0 waits for the input vector, the block stages it (sc1 loads) in LDS, and every
// wave dots its rows.  Rows >= N re-read row N - 1 (the caller drops them).
// ---------------------------------------------------------------------------------------
template <int KCH, int RPW, bool F8, bool NORM>
struct GemvBlock {
  static constexpr int EPC = F8 ? 16 : 8;
  static constexpr int PL = EPC / 4;
  static constexpr int KC = KCH * 64;
  static constexpr int XPT = (KC + NT - 1) / NT;
  uint4 w[RPW][KCH];
  float4 nv[NORM ? XPT : 1][PL];

  __device__ __forceinline__ void load(const void* W, int n0, int N, const float* nw) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int n = min(n0 + r, N - 1);
      const uint4* wp = reinterpret_cast<const uint4*>(W) + (size_t)n * KC + lane;
#pragma unroll
      for (int c = 0; c < KCH; ++c) w[r][c] = load_nt(wp + c * 64);
    }
    if (NORM) {
      const float4* nw4 = reinterpret_cast<const float4*>(nw);
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const int m = min((int)threadIdx.x + i * NT, KC - 1);
#pragma unroll
        for (int q = 0; q < PL; ++q) nv[i][q] = nw4[PL * m + q];
      }
    }
  }
  // Stage x (x . nw) into xs planes; returns the RMSNorm scale (1 without NORM).
  __device__ __forceinline__ float stage(const float* x, float eps, float4* xs, float* red) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    float4 xv[XPT][PL];
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int m = min(tid + i * NT, KC - 1);
#pragma unroll
      for (int q = 0; q < PL; ++q) xv[i][q] = ld4_wt(x, (size_t)(PL * m + q) * 4);
    }
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int m = tid + i * NT;
      if (m < KC) {
#pragma unroll
        for (int q = 0; q < PL; ++q) {
          float4 v = xv[i][q];
          if (NORM) {
            ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
            v.x *= nv[i][q].x; v.y *= nv[i][q].y; v.z *= nv[i][q].z; v.w *= nv[i][q].w;
          }
          xs[q * KC + m] = v;
        }
      }
    }
    float scale = 1.f;
    if (NORM) {
      ss = wave_sum(ss);
      if (lane == 0) red[wid] = ss;
    }
    __syncthreads();
    if (NORM) scale = 1.0f / sqrtf((red[0] + red[1] + red[2] + red[3]) / (float)(KC * EPC) + eps);
    return scale;
  }
  // acc[r] = total of row r (every lane), times scale and the fp8 row scale
  __device__ __forceinline__ void dot(const float4* xs, float scale, const float* wscale, int n0,
                                      int N, float acc[RPW]) {
    const int lane = threadIdx.x & 63;
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
      acc[r] = wave_sum(acc[r]) * scale;
      if (F8) acc[r] *= wscale[min(n0 + r, N - 1)];
    }
  }
};

struct Geo {  // block counts of one launch
  int NQ, NA, NO, NG, ND, NH, P;
  __host__ __device__ Geo(const StepArgs& a) {
    NQ = (a.heads + 2 * a.kvh) * 16;  // 8 rows per block, 16 blocks per 128-row head
    NA = a.kvh * a.nsplit;
    NO = a.H / 8;
    NG = a.F / 4;                      // 2F rows, 8 per block
    ND = a.H / 4;                      // 1 row per wave
    NH = (a.V + 7) / 8;
    P = NQ + NA + NO + NG + ND;
  }
};

__device__ __forceinline__ int* ctr(const StepArgs& a, int l, int slot) {
  return a.cnt + ((size_t)l * STEP_LAYER_CNT + slot) * STEP_CS;
}

// ---------------------------------------------------------------------------------------
// Attention split block: kv head g, old positions [64 s, min(64 s + 64, pos)).  Wave w takes
// 16 positions; lane (pp = lane / 4, dq = 32 (lane % 4)) holds 32 dims of one K row, and the
// 16 positions of V^T dims 2 lane, 2 lane + 1.  K / V are loaded before the wait (they were
// written by earlier launches); q arrives through the hand-off.  The last-arriving split of g
// merges every split with the new position (q . k_new, v_new) and publishes att[g heads].
// ---------------------------------------------------------------------------------------
// LDS floats of an attention block (layout in att_block), for up to STEP_MAX_SPLITS splits
constexpr int STEP_MAX_SPLITS = 128;
__host__ __device__ constexpr int att_lds_floats(int grp) {
  return grp * (128 + 4 * 16 + 8 + 4 * 128) + 260 + STEP_MAX_SPLITS * grp * 2;
}

template <int GRP>
__device__ void att_block(const StepArgs& a, int l, int idx, float* lds, int* flag,
                          unsigned long long* tw) {
  const int QD = a.heads * 128;
  const int g = idx / a.nsplit, s = idx - g * a.nsplit;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int pos = a.row_pos[0], slot = a.row_slot[0];
  const size_t head = (size_t)slot * a.kvh + g;
  // fragment-major 32-position chunks (mx_common.h kv_k_off / kv_v_off), in 16-byte units
  const uint4* Kf = reinterpret_cast<const uint4*>(a.kcache + a.kv_layer_elems * l) + head * a.max_pos * 16;
  const uint4* Vf = reinterpret_cast<const uint4*>(a.vcache + a.kv_layer_elems * l) + head * a.max_pos * 16;
  const int p0 = s * STEP_SPLIT + wid * 16;
  const int pp = lane >> 2, dq = (lane & 3) * 32;
  const int p = p0 + pp;
  const bool valid = p < pos;
  uint4 kr[4], vr[2][2];
  {
    // lane: position p, dims dq .. dq + 31 = k-step dq / 32, groups i = 0..3
    const int pk = max(min(p, pos - 1), 0), q = pk & 31;
    const uint4* kp = Kf + (size_t)(pk >> 5) * 512 + (((q >> 2) & 1) * 4 + (dq >> 5)) * 64 +
                      4 * (q >> 3) + (q & 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) kr[i] = kp[16 * i];
    // lane: dims 2 lane + j, positions p0 .. p0 + 15 (two groups of 8; p0 is a multiple of 16)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int d = 2 * lane + j;
      const uint4* vp = Vf + (size_t)(p0 >> 5) * 512 + ((d >> 4) * 4 + ((p0 & 31) >> 3)) * 16 + (d & 15);
      vr[j][0] = vp[0];
      vr[j][1] = vp[16];
    }
  }
  float* qs = lds;                   // [GRP][128]
  float* es = qs + GRP * 128;        // [4][GRP][16]
  float* wm = es + 4 * GRP * 16;     // [4][GRP]
  float* wl = wm + 4 * GRP;          // [4][GRP]
  float* wacc = wl + 4 * GRP;        // [4][GRP][128]
  float* kn = wacc + 4 * GRP * 128;  // [128] merge: k_new, v_new, s_new
  float* vn = kn + 128;
  float* sn = vn + 128;              // [GRP]
  float* sml = sn + 4;               // [nsplit][GRP][2]
  if (s == 0 && tid == 0 && (pos + STEP_SPLIT - 1) / STEP_SPLIT > a.nsplit)
    atomicCAS(a.status, 0, 9);  // the host sized the grid for fewer positions
  if (wid == 0) wait_for(ctr(a, l, C_QKV + g), 1, (GRP + 2) * 16, a.status, 2);
  __syncthreads();
  if (a.trace && tid == 0) *tw = __builtin_amdgcn_s_memrealtime();
  const float* qg = a.q + (size_t)l * QD + (size_t)g * GRP * 128;
  if (tid < GRP * 32) {
    const float4 v = ld4_wt(qg, (size_t)tid * 4);
    reinterpret_cast<float4*>(qs)[tid] = v;
  }
  __syncthreads();
  // scores: 32-dim partials, summed over the 4 lanes of a position
  float sc[GRP];
#pragma unroll
  for (int h = 0; h < GRP; ++h) sc[h] = 0.f;
#pragma unroll 1
  for (int i = 0; i < 4; ++i) {
    const uint32_t kw[4] = {kr[i].x, kr[i].y, kr[i].z, kr[i].w};
#pragma unroll
    for (int h = 0; h < GRP; ++h) {
      const float4 q0 = reinterpret_cast<const float4*>(qs + h * 128 + dq + 8 * i)[0];
      const float4 q1 = reinterpret_cast<const float4*>(qs + h * 128 + dq + 8 * i)[1];
      sc[h] = fmaf(bf16_lo(kw[0]), q0.x, sc[h]);
      sc[h] = fmaf(bf16_hi(kw[0]), q0.y, sc[h]);
      sc[h] = fmaf(bf16_lo(kw[1]), q0.z, sc[h]);
      sc[h] = fmaf(bf16_hi(kw[1]), q0.w, sc[h]);
      sc[h] = fmaf(bf16_lo(kw[2]), q1.x, sc[h]);
      sc[h] = fmaf(bf16_hi(kw[2]), q1.y, sc[h]);
      sc[h] = fmaf(bf16_lo(kw[3]), q1.z, sc[h]);
      sc[h] = fmaf(bf16_hi(kw[3]), q1.w, sc[h]);
    }
  }
  float m[GRP], e[GRP], lsum[GRP];
#pragma unroll
  for (int h = 0; h < GRP; ++h) {
    sc[h] += __shfl_xor(sc[h], 1, 64);
    sc[h] += __shfl_xor(sc[h], 2, 64);
    const float sv = valid ? sc[h] * a.att_scale : -INFINITY;
    m[h] = wave_max(sv);
    e[h] = (valid && m[h] != -INFINITY) ? expf(sv - m[h]) : 0.f;
    lsum[h] = wave_sum((lane & 3) == 0 ? e[h] : 0.f);
    if ((lane & 3) == 0) es[(wid * GRP + h) * 16 + pp] = e[h];
  }
  __syncthreads();
  // P.V for dims 2 lane + j
  float acc[GRP][2];
#pragma unroll
  for (int h = 0; h < GRP; ++h) acc[h][0] = acc[h][1] = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const uint32_t vw[8] = {vr[j][0].x, vr[j][0].y, vr[j][0].z, vr[j][0].w,
                            vr[j][1].x, vr[j][1].y, vr[j][1].z, vr[j][1].w};
#pragma unroll 4
    for (int t = 0; t < 16; ++t) {
      const float v = (p0 + t < pos) ? ((t & 1) ? bf16_hi(vw[t >> 1]) : bf16_lo(vw[t >> 1])) : 0.f;
#pragma unroll
      for (int h = 0; h < GRP; ++h) acc[h][j] = fmaf(es[(wid * GRP + h) * 16 + t], v, acc[h][j]);
    }
  }
#pragma unroll
  for (int h = 0; h < GRP; ++h) {
    if (lane == 0) {
      wm[wid * GRP + h] = m[h];
      wl[wid * GRP + h] = lsum[h];
    }
    wacc[(wid * GRP + h) * 128 + 2 * lane] = acc[h][0];
    wacc[(wid * GRP + h) * 128 + 2 * lane + 1] = acc[h][1];
  }
  __syncthreads();
  // block partial -> write-through stores
  float* pb = a.part + (((size_t)l * a.kvh + g) * a.split_max + s) * GRP * STEP_PART;
  for (int o = tid; o < GRP * 128; o += NT) {
    const int h = o >> 7, d = o & 127;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, wm[w * GRP + h]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float mw = wm[w * GRP + h];
      const float f = mw == -INFINITY ? 0.f : expf(mw - M);
      num = fmaf(f, wacc[(w * GRP + h) * 128 + d], num);
      den = fmaf(f, wl[w * GRP + h], den);
    }
    st_wt(pb + h * STEP_PART + d, num);
    if (d == 0) {
      st_wt(pb + h * STEP_PART + 128, M);
      st_wt(pb + h * STEP_PART + 129, den);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(ctr(a, l, C_ATK + g), 1, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    *flag = (t == a.nsplit - 1);
  }
  __syncthreads();
  if (!*flag) return;
  // ---- last arriver: merge the splits and the new position ----
  const float* p0b = a.part + ((size_t)l * a.kvh + g) * a.split_max * GRP * STEP_PART;
  if (tid < 64) {
    const float* src = tid < 32 ? a.knew : a.vnew;
    const float4 v = ld4_wt(src + ((size_t)l * a.kvh + g) * 128, (size_t)(tid & 31) * 4);
    reinterpret_cast<float4*>(tid < 32 ? kn : vn)[tid & 31] = v;
  }
  for (int i = tid; i < a.nsplit * GRP * 2; i += NT) {
    const int sp = i / (GRP * 2), r = i - sp * GRP * 2;
    sml[i] = ld_wt(p0b + ((size_t)sp * GRP + (r >> 1)) * STEP_PART + 128 + (r & 1));
  }
  __syncthreads();
  if (wid < GRP) {
    float d = qs[wid * 128 + lane] * kn[lane] + qs[wid * 128 + lane + 64] * kn[lane + 64];
    d = wave_sum(d);
    if (lane == 0) sn[wid] = d * a.att_scale;
  }
  __syncthreads();
  float* out = a.att + (size_t)l * QD + (size_t)g * GRP * 128;
  for (int o = tid; o < GRP * 128; o += NT) {
    const int h = o >> 7, d = o & 127;
    float M = sn[h];
    for (int sp = 0; sp < a.nsplit; ++sp) M = fmaxf(M, sml[(sp * GRP + h) * 2]);
    const float fn = expf(sn[h] - M);
    float num = fn * vn[d], den = fn;
    for (int s0 = 0; s0 < a.nsplit; s0 += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] = s0 + j < a.nsplit ? ld_wt(p0b + ((size_t)(s0 + j) * GRP + h) * STEP_PART + d) : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (s0 + j < a.nsplit) {
          const float f = expf(sml[((s0 + j) * GRP + h) * 2] - M);
          num = fmaf(f, v[j], num);
          den = fmaf(f, sml[((s0 + j) * GRP + h) * 2 + 1], den);
        }
      }
    }
    st_wt(out + o, num / den);
  }
  signal(ctr(a, l, C_ATT));
}

// ---------------------------------------------------------------------------------------
template <bool F8, int KH, int KF, int GRP>
__global__ __launch_bounds__(NT) void step_kernel(StepArgs a) {
  constexpr int EPC = F8 ? 16 : 8;
  constexpr int XG = (KF > KH ? KF : KH) * 64 * (EPC / 4);  // float4s of the largest GEMV input
  constexpr int XA = (att_lds_floats(GRP) + 3) / 4;           // attention scratch
  constexpr int XS = XG > XA ? XG : XA;
  __shared__ __attribute__((aligned(16))) float4 xs[XS];
  __shared__ float red[4];
  __shared__ int flag;
  __shared__ unsigned long long bkey[4];
  __shared__ unsigned long long t_w;  // diagnostic trace: when the block's wait ended
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const unsigned long long t_e = a.trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // diagnostic trace (a.trace != null only): per block {entry, wait done, end, role << 32 |
  // layer} on the 100 MHz constant clock
#define STEP_WAITED() \
  if (a.trace && tid == 0) t_w = __builtin_amdgcn_s_memrealtime();
#define STEP_DONE(role_, layer_)                                                    \
  if (a.trace && tid == 0) {                                                        \
    unsigned long long* tr_ = a.trace + (size_t)b * 4;                              \
    tr_[0] = t_e;                                                                   \
    tr_[1] = t_w;                                                                   \
    tr_[2] = __builtin_amdgcn_s_memrealtime();                                      \
    tr_[3] = ((unsigned long long)(role_) << 32) | (unsigned)(layer_);              \
  }
  const Geo G(a);
  const int64_t b = blockIdx.x + a.block0;
  const int H = a.H, QD = a.heads * 128;
  const int esz = F8 ? 1 : 2;
  const int qkv_rows = QD + 2 * a.kvh * 128;

  if (b < (int64_t)a.layers * G.P) {
    const int l = (int)(b / G.P);
    int r = (int)(b - (int64_t)l * G.P);
    const float* hin = l == 0 ? a.h : a.hd + (size_t)(l - 1) * H;
    if (r < G.NQ) {
      // ---- QKV + RoPE + KV append: 8 rows (4 RoPE pairs), one head ----
      GemvBlock<KH, 2, F8, true> gb;
      const int n0 = r * 8 + 2 * wid;
      const uint8_t* W = static_cast<const uint8_t*>(a.wqkv) + (size_t)l * qkv_rows * H * esz;
      gb.load(W, n0, qkv_rows, a.attn_norm + (size_t)l * H);
      const int pos = a.row_pos[0], slot = a.row_slot[0];
      const int hh = n0 >> 7, within = n0 & 127, pr = within >> 1;
      const float cs = a.rope_cos[(size_t)pos * 64 + pr], sn = a.rope_sin[(size_t)pos * 64 + pr];
      if (l > 0 && wid == 0) wait_for(ctr(a, l - 1, C_DN), 8, G.ND, a.status, 1);
      __syncthreads();
      STEP_WAITED()
      const float scale = gb.stage(hin, a.eps, xs, red);
      float acc[2];
      gb.dot(xs, scale, F8 ? a.sqkv + (size_t)l * qkv_rows : nullptr, n0, qkv_rows, acc);
      if (lane == 0) {
        const float x1 = acc[0], x2 = acc[1];
        if (hh < a.heads + a.kvh) {
          const float o1 = x1 * cs - x2 * sn, o2 = x2 * cs + x1 * sn;
          if (hh < a.heads) {
            float* q = a.q + (size_t)l * QD + (size_t)hh * 128;
            st_wt(q + pr, o1);
            st_wt(q + pr + 64, o2);
          } else {
            const int kv = hh - a.heads;
            uint16_t* k = a.kcache + a.kv_layer_elems * l +
                          ((size_t)slot * a.kvh + kv) * a.max_pos * 128;
            const uint16_t b1 = f32_to_bf16(o1), b2 = f32_to_bf16(o2);
            k[kv_k_off(pos, pr)] = b1;
            k[kv_k_off(pos, pr + 64)] = b2;
            float* kn = a.knew + ((size_t)l * a.kvh + kv) * 128;
            st_wt(kn + pr, bf16_to_f32(b1));
            st_wt(kn + pr + 64, bf16_to_f32(b2));
          }
        } else {
          const int kv = hh - a.heads - a.kvh;
          uint16_t* v = a.vcache + a.kv_layer_elems * l + ((size_t)slot * a.kvh + kv) * 128 * a.max_pos;
          const uint16_t b1 = f32_to_bf16(x1), b2 = f32_to_bf16(x2);
          v[kv_v_off(pos, within)] = b1;
          v[kv_v_off(pos, within + 1)] = b2;
          float* vn = a.vnew + ((size_t)l * a.kvh + kv) * 128;
          st_wt(vn + within, bf16_to_f32(b1));
          st_wt(vn + within + 1, bf16_to_f32(b2));
        }
      }
      const int hb = (r * 8) >> 7;  // the block's head
      const int grp = hb < a.heads ? hb / GRP : hb < a.heads + a.kvh ? hb - a.heads
                                                                     : hb - a.heads - a.kvh;
      signal(ctr(a, l, C_QKV + grp));
      STEP_DONE(0, l)
      return;
    }
    r -= G.NQ;
    if (r < G.NA) {
      att_block<GRP>(a, l, r, reinterpret_cast<float*>(xs), &flag, &t_w);
      STEP_DONE(1, l)
      return;
    }
    r -= G.NA;
    if (r < G.NO) {
      // ---- O projection (+ residual): 8 rows ----
      GemvBlock<KH, 2, F8, false> gb;
      const int n0 = r * 8 + 2 * wid;
      gb.load(static_cast<const uint8_t*>(a.wo) + (size_t)l * H * QD * esz, n0, H, nullptr);
      if (wid == 0) wait_for(ctr(a, l, C_ATT), 1, a.kvh, a.status, 3);
      __syncthreads();
      STEP_WAITED()
      const float r0 = ld_wt(hin + n0), r1 = ld_wt(hin + n0 + 1);
      const float scale = gb.stage(a.att + (size_t)l * QD, a.eps, xs, red);
      float acc[2];
      gb.dot(xs, scale, F8 ? a.so + (size_t)l * H : nullptr, n0, H, acc);
      if (lane == 0) {
        float* ho = a.ho + (size_t)l * H;
        st_wt(ho + n0, r0 + acc[0]);
        st_wt(ho + n0 + 1, r1 + acc[1]);
      }
      signal(ctr(a, l, C_O + (r & 7)));
      STEP_DONE(2, l)
      return;
    }
    r -= G.NO;
    if (r < G.NG) {
      // ---- gate/up + SiLU * up: 8 rows = 4 (gate, up) pairs ----
      GemvBlock<KH, 2, F8, true> gb;
      const int n0 = r * 8 + 2 * wid;
      gb.load(static_cast<const uint8_t*>(a.wgu) + (size_t)l * 2 * a.F * H * esz, n0, 2 * a.F,
              a.mlp_norm + (size_t)l * H);
      if (wid == 0) wait_for(ctr(a, l, C_O), 8, G.NO, a.status, 4);
      __syncthreads();
      STEP_WAITED()
      const float scale = gb.stage(a.ho + (size_t)l * H, a.eps, xs, red);
      float acc[2];
      gb.dot(xs, scale, F8 ? a.sgu + (size_t)l * 2 * a.F : nullptr, n0, 2 * a.F, acc);
      if (lane == 0) {
        const float gt = acc[0], up = acc[1];
        st_wt(a.act + (size_t)l * a.F + (n0 >> 1), gt / (1.0f + expf(-gt)) * up);
      }
      signal(ctr(a, l, C_GU + (r & 7)));
      STEP_DONE(3, l)
      return;
    }
    r -= G.NG;
    {
      // ---- down (+ residual): 4 rows, one per wave ----
      GemvBlock<KF, 1, F8, false> gb;
      const int n0 = r * 4 + wid;
      gb.load(static_cast<const uint8_t*>(a.wd) + (size_t)l * H * a.F * esz, n0, H, nullptr);
      if (wid == 0) wait_for(ctr(a, l, C_GU), 8, G.NG, a.status, 5);
      __syncthreads();
      STEP_WAITED()
      const float res = ld_wt(a.ho + (size_t)l * H + n0);
      const float scale = gb.stage(a.act + (size_t)l * a.F, a.eps, xs, red);
      float acc[1];
      gb.dot(xs, scale, F8 ? a.sd + (size_t)l * H : nullptr, n0, H, acc);
      if (lane == 0) st_wt(a.hd + (size_t)l * H + n0, res + acc[0]);
      signal(ctr(a, l, C_DN + (r & 7)));
      STEP_DONE(4, l)
      return;
    }
  }
  const int64_t hb = b - (int64_t)a.layers * G.P;
  int* head_c = a.cnt + (size_t)a.layers * STEP_LAYER_CNT * STEP_CS;
  if (hb < G.NH) {
    // ---- final norm + lm_head + penalty + argmax: 8 rows ----
    GemvBlock<KH, 2, F8, true> gb;
    const int n0 = (int)hb * 8 + 2 * wid;
    gb.load(a.lm, n0, a.V, a.norm);
    const int slot = a.row_slot[0];
    const float pen = a.penalty[slot];
    const bool keep = a.logits_all || a.samp_temp[slot] > 0.f;
    const uint8_t sn0 = a.seen[(size_t)slot * a.V + min(n0, a.V - 1)];
    const uint8_t sn1 = a.seen[(size_t)slot * a.V + min(n0 + 1, a.V - 1)];
    if (wid == 0) wait_for(ctr(a, a.layers - 1, C_DN), 8, G.ND, a.status, 6);
    __syncthreads();
    STEP_WAITED()
    const float scale = gb.stage(a.hd + (size_t)(a.layers - 1) * H, a.eps, xs, red);
    float acc[2];
    gb.dot(xs, scale, F8 ? a.slm : nullptr, n0, a.V, acc);
    unsigned long long best = 0ull;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = n0 + i;
      if (n < a.V) {
        float v = acc[i];
        if (i == 0 ? sn0 : sn1) v = v > 0.f ? v / pen : v * pen;
        if (keep && lane == 0) a.logits[n] = v;
        const unsigned long long k = argmax_key(v, (uint32_t)n);
        best = k > best ? k : best;
      }
    }
    if (lane == 0) bkey[wid] = best;
    __syncthreads();
    if (tid == 0) {
      unsigned long long k = bkey[0];
      for (int w = 1; w < 4; ++w) k = bkey[w] > k ? bkey[w] : k;
      __hip_atomic_fetch_max(a.best_sh + (hb & (STEP_BEST - 1)), k, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    }
    signal(head_c + (hb & 7) * STEP_CS);
    STEP_DONE(5, 0)
    return;
  }
  // ---- finish (the last block): argmax over the shards, commit, reset the counters ----
  if (wid == 0) wait_for(head_c, 8, G.NH, a.status, 7);
  __syncthreads();
  STEP_WAITED()
  __shared__ int tok_s;
  if (wid == 0) {
    unsigned long long k = __hip_atomic_load(a.best_sh + lane, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const unsigned long long o = __shfl_xor(k, d, 64);
      k = o > k ? o : k;
    }
    if (lane == 0) {
      const int tok = min((int)argmax_index(k) & 0x7fffffff, a.V - 1);  // (a failed step only)
      tok_s = tok;
      if (a.commit) {
        const int slot = a.row_slot[0];
        if (slot != a.scratch_slot) {  // parked rows stay at position 0 of the scratch slot
          const int pos = min(a.row_pos[0] + 1, a.max_pos - 1);
          a.row_pos[0] = pos;
          a.row_token[0] = tok;
          a.seen[(size_t)slot * a.V + tok] = 1;
          a.hist[(size_t)slot * a.max_pos + pos] = tok;
        }
      } else {
        *a.best = k;
      }
      const int st = ld_wt_i(a.status);
      if (st) *reinterpret_cast<volatile int*>(a.status_host) = st;
    }
  }
  __syncthreads();
  if (a.commit) {
    const uint4* e = reinterpret_cast<const uint4*>(a.embed + (size_t)tok_s * H);
    float4* h = reinterpret_cast<float4*>(a.h);
    for (int c = tid; c < (H >> 3); c += NT) {
      const uint4 w = e[c];
      h[2 * c] = make_float4(bf16_lo(w.x), bf16_hi(w.x), bf16_lo(w.y), bf16_hi(w.y));
      h[2 * c + 1] = make_float4(bf16_lo(w.z), bf16_hi(w.z), bf16_lo(w.w), bf16_hi(w.w));
    }
  }
  const int ncnt = a.layers * STEP_LAYER_CNT + 8;
  for (int i = tid; i < ncnt; i += NT)
    __hip_atomic_store(a.cnt + (size_t)i * STEP_CS, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid < STEP_BEST)
    __hip_atomic_store(a.best_sh + tid, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  STEP_DONE(6, 0)
#undef STEP_WAITED
#undef STEP_DONE
}

}  // namespace step

int64_t step_blocks(const StepArgs& a) {
  const step::Geo G(a);
  return (int64_t)a.layers * G.P + G.NH + 1;
}

size_t step_counter_ints(int layers) {
  return ((size_t)layers * STEP_LAYER_CNT + 8) * STEP_CS;
}

// Instantiated shapes: Orpheus-3B (H 3072, F 8192, 24 / 8 heads) and the 512 / 1024 test
// shape (4 / 2 heads); bf16 and e4m3 (H 1024 / F 2048 / 8 / 2 heads for the fp8 tests).
#define MX_STEP_SHAPES(X)          \
  X(false, 3072, 8192, 3)          \
  X(false, 512, 1024, 2)           \
  X(true, 3072, 8192, 3)           \
  X(true, 1024, 2048, 4)

bool step_supported(int H, int F, int heads, int kvh, bool f8) {
  if (heads * 128 != H || kvh > 8 || heads % kvh) return false;
  const int grp = heads / kvh;
#define MX_S(F8_, H_, F_, G_) if (f8 == F8_ && H == H_ && F == F_ && grp == G_) return true;
  MX_STEP_SHAPES(MX_S)
#undef MX_S
  return false;
}

// blocks [b0, b0 + nb) of the step's role list as one launch
static hipError_t launch_step_range(StepArgs a, bool f8, int64_t b0, int64_t nb, hipStream_t st) {
  if (a.heads * 128 != a.H || a.kvh > 8 || a.heads % a.kvh || a.nsplit < 1 ||
      a.nsplit > a.split_max || a.split_max > step::STEP_MAX_SPLITS)
    return hipErrorInvalidValue;
  const int grp = a.heads / a.kvh;
  if (nb < 1 || b0 < 0 || b0 + nb > step_blocks(a) || nb >= (int64_t)1 << 31)
    return hipErrorInvalidValue;
  a.block0 = b0;
#define MX_S(F8_, H_, F_, G_)                                                               \
  if (f8 == F8_ && a.H == H_ && a.F == F_ && grp == G_) {                                   \
    constexpr int E_ = F8_ ? 1024 : 512;                                                    \
    hipLaunchKernelGGL((step::step_kernel<F8_, H_ / E_, F_ / E_, G_>), dim3((unsigned)nb), \
                       dim3(step::NT), 0, st, a);                                           \
    return hipGetLastError();                                                               \
  }
  MX_STEP_SHAPES(MX_S)
#undef MX_S
  return hipErrorNotSupported;
}

hipError_t launch_step(const StepArgs& a, bool f8, hipStream_t st) {
  return launch_step_range(a, f8, 0, step_blocks(a), st);
}

hipError_t launch_step_cut(const StepArgs& a, bool f8, int cuts, hipStream_t st) {
  const step::Geo G(a);
  const int64_t s0[6] = {0, G.NQ, G.NQ + G.NA, G.NQ + G.NA + G.NO, G.NQ + G.NA + G.NO + G.NG, G.P};
  cuts |= 1;
  for (int l = 0; l < a.layers; ++l) {
    int s = 0;
    while (s < 5) {
      int e = s + 1;
      while (e < 5 && !((cuts >> e) & 1)) ++e;
      const hipError_t r = launch_step_range(a, f8, (int64_t)l * G.P + s0[s], s0[e] - s0[s], st);
      if (r != hipSuccess) return r;
      s = e;
    }
  }
  return launch_step_range(a, f8, (int64_t)a.layers * G.P, G.NH + 1, st);
}

}  // namespace mx
