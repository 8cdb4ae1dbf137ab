// Single-stream (B = 1) decode step as ONE persistent launch over all layers, gfx950.
//
// Replaces, for one stream, the per-token forward of vLLM AsyncLLMEngine.generate
// (Orpheus-TTS/orpheus_tts_pypi/orpheus_tts/engine_class.py:117) / llama.cpp
// Llama.text_to_speech (Morpheus_Client/tts_engine/llama_local.py:77): per layer RMSNorm ->
// QKV + RoPE + KV append -> GQA attention -> O-proj + residual -> RMSNorm -> gate/up + SiLU*up
// -> down + residual.  The lm_head / penalty / argmax and the commit stay separate launches.
//
// Why one launch: at B = 1 the step is a 6.6 GB weight stream cut into 140
// dependent pieces.  As separate kernels every piece pays a ramp and a drain (the small
// projections ran at 3.6-3.8 TB/s, attention at ~7 us of latency per layer).  Here the
// weight stream never stops at a phase seam: every compute wave owns a fixed, contiguous
// slice of every projection's rows and keeps a register ring of D 1-KB weight pieces
// ("units") in flight ACROSS phase and layer boundaries, so while a block waits for the
// grid-wide hand-off of the next activation vector, its next weights are already landing.
//
// Geometry (Orpheus-3B / Llama-3.2-3B only: hidden 3072, 24 q / 8 kv heads of 128, FFN 8192):
//   * 256 blocks (one per CU; all co-resident, checked on the host) x 5 waves:
//     waves 0-3 stream weights (the ring), wave 4 is the block's control wave.
//   * Every projection splits into whole rows per compute wave: qkv 5, o 3, gate/up 16,
//     down 3 rows (block: 20 / 12 / 64 / 12 rows; x 256 blocks = 5120 / 3072 / 16384 / 3072).
//     A unit is one 16-byte load per lane = 512 bf16 (or 1024 e4m3) consecutive weights of
//     one row; a wave's units for a layer are its rows in order: 192 (bf16) / 96 (fp8).
//   * Compute waves: dot(unit, staged activations in LDS) in fp32, one wave_sum per row,
//     row result -> LDS.  They touch no global memory except their weight loads, and never
//     wait on vmcnt except for the ring slot they consume next.
//   * Control wave, per phase: finalize the block's rows (fold RMSNorm scale, fp8 row
//     scale, RoPE + K/V append, residual, SiLU*up), publish them with write-through (sc1)
//     stores, s_waitcnt vmcnt(0), one agent-scope atomic add on the phase counter; then poll
//     the counter of the NEXT phase's input, load that vector with sc1 loads into LDS and
//     release the compute waves (MI355X_MICROARCH.md "Valid forms" row 1: sc1 stores + one
//     signalling lane per workgroup, sc1 poll, sc1 loads).
//   * Attention (control waves of blocks b < 8 * nsplit, split = 128 positions of one kv
//     head): the split's K rows and V^T rows of positions < L-1 are staged into LDS during
//     the previous layer's gate/up phase (they were written by earlier launches); the new
//     position's k / v (bf16-rounded) come from this launch's qkv vector.  Q.K^T and P.V on
//     bf16 MFMA with q and p split into three bf16 parts (fp32-exact products), online
//     softmax, partial (m, l, acc) published sc1, the last arriver per kv head merges.
//   * Every activation vector of a layer has its own buffer (no in-launch reuse of a line),
//     every polled word is zeroed by a memset node ahead of the launch, every spin is bounded
//     (give-up writes a status word the host can read; the launch still drains).
#include "mx_common.h"
#include "mx_llm_kernels.h"

#include <type_traits>

namespace mx {
namespace mega {

constexpr int H = 3072, QD = 3072, KVH = 8, GRP = 3, QKVR = QD + 2 * KVH * 128, FF = 8192;
constexpr int NB = MEGA_BLOCKS, WPB = 4, NTH = (WPB + 1) * 64;
constexpr int RQ = 5, RO = 3, RG = 16, RD = 3;                         // rows / compute wave
constexpr int BQ = RQ * WPB, BO = RO * WPB, BG = RG * WPB, BD = RD * WPB;  // rows / block
static_assert(BQ * NB == QKVR && BO * NB == H && BG * NB == 2 * FF && BD * NB == H, "geometry");
constexpr int SPL = MEGA_SPLIT;      // attention positions per split
constexpr int PART = MEGA_PART;      // floats per split partial: acc[3][128], m[3], l[3], pad
constexpr int SPIN_MAX = 400000;     // ~0.4 s of polling before a wait gives up

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool F8>
struct Geo {
  static constexpr int EPC = F8 ? 16 : 8;          // weights per 16-byte lane load
  static constexpr int PL = EPC / 4;               // float4 planes of a staged activation vector
  static constexpr int CH = 64 * EPC;              // K elements of one unit
  static constexpr int PS = FF / EPC;              // float4s per plane (sized for K = FF)
  static constexpr int KH = H / CH, KF = FF / CH;  // units per row at K = H and K = FF
  static constexpr int UQ = RQ * KH, UO = RO * KH, UG = RG * KH, UD = RD * KF;
  static constexpr int OO = UQ, OG = UQ + UO, OD = UQ + UO + UG, U = OD + UD;
  static constexpr int ESZ = F8 ? 1 : 2;
  static constexpr size_t RBH = (size_t)H * ESZ, RBF = (size_t)FF * ESZ;  // row bytes
};

// ---- small device helpers ---------------------------------------------------------------
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-byte write-through-coherent load (buffer_load_dwordx4 ... sc1)
__device__ __forceinline__ float4 ld4_sc1(const float* base, int idx4) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff, 0x00020000);
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, idx4 * 16, 0, 16);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                     __uint_as_float(v.w));
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Wave-uniform bounded wait for *p >= target.  `dead` latches the first give-up so the rest
// of the launch runs through without waiting (results invalid, status word set).
__device__ __forceinline__ void wait_ge(int* p, int target, int* status, int code, bool& dead) {
  if (dead) return;
  for (int it = 0; it < SPIN_MAX; ++it) {
    const int v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__builtin_amdgcn_readfirstlane(v) >= target) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  dead = true;
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_store(status, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Per-block arrival flags of one grid seam: block b stores flags[b] = 1 (sc1, after its drain);
// a consumer polls all 256 with ONE 16-byte sc1 load per lane and a wave vote.  No shared
// counter line: 256 same-line atomic arrivals serialise (MI355X_MICROARCH.md, one-row
// contention), which the event trace showed as ~7 us per seam.
__device__ __forceinline__ void set_flag(int* f) {
  drain();
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(f, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wait_flags(const int* f, int* status, int code, bool& dead) {
  if (dead) return;
  const int lane = threadIdx.x & 63;
  for (int it = 0; it < SPIN_MAX; ++it) {
    const float4 v = ld4_sc1(reinterpret_cast<const float*>(f), lane);  // flags 4 lane .. 4 lane + 3
    const bool ok = __float_as_int(v.x) && __float_as_int(v.y) && __float_as_int(v.z) &&
                    __float_as_int(v.w);
    if (__all(ok)) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  dead = true;
  if (lane == 0) __hip_atomic_store(status, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void signal(int* p) {
  drain();  // every sc1 store of this wave has left the CU before the count moves
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// ---- LDS --------------------------------------------------------------------------------
// xs: staged activation vector, PL planes of PS float4 (plane q, index c*64 + m holds
//     elements c*CH + m*EPC + 4q .. +4, the 4 activations lane m of a unit at chunk c needs).
// ks: K rows of the block's attention split, [128 pos][16 granules of 16 B], granule index
//     XOR (pos & 15) (conflict-free MFMA A-fragment reads); vs: V^T rows [128 dim][16
//     granules of 8 positions], granule index XOR (dim & 15).
struct Smem {
  float4 xs[FF / 4];
  uint4 ks[SPL * 16];
  uint4 vs[128 * 16];
  float rowres[64];
};

// ---- control wave: stage an activation vector (sc1 loads) into LDS ------------------------
// returns sum of squares of the raw vector (for the folded RMSNorm scale)
template <bool F8, int K>
__device__ __forceinline__ float stage_x(Smem& sm, const float* src, const float* nw, int lane) {
  using G = Geo<F8>;
  constexpr int NL = K / 256;  // float4 loads per lane
  float4 v[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) v[j] = ld4_sc1(src, 64 * j + lane);
  float4 n[NL];
  if (nw) {
#pragma unroll
    for (int j = 0; j < NL; ++j) n[j] = reinterpret_cast<const float4*>(nw)[64 * j + lane];
  }
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    float4 x = v[j];
    ss += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
    if (nw) {
      x.x *= n[j].x; x.y *= n[j].y; x.z *= n[j].z; x.w *= n[j].w;
    }
    const int e0 = 256 * j + 4 * lane;
    const int c = e0 / G::CH, within = e0 % G::CH;
    const int m = within / G::EPC, q = (within % G::EPC) / 4;
    sm.xs[q * G::PS + c * 64 + m] = x;
  }
  return wave_sum(ss);
}

// ---- control wave: stage the split's K / V^T rows (positions p0 .. p0+127) into LDS ------
// 64 LDS-DMA loads (global_load_lds_dwordx4: no VGPRs, all in flight at once; completion is
// the wave's vmcnt, waited for before the attention reads them).  Instruction j fills 1 KB of
// LDS linearly (lane i -> slot 16 j... + i); the XOR swizzle is applied on the SOURCE side:
// LDS slot s of row r holds global granule s ^ (r & 15).
typedef __attribute__((address_space(3))) void lds_void;
__device__ __forceinline__ void stage_kv(Smem& sm, const uint16_t* kc, const uint16_t* vc,
                                         int max_pos, int lane) {
  // kc: K rows of (slot, kv head) starting at position p0 (contiguous 256 B per position);
  // vc: V^T of (slot, kv head) at position p0 (row d at vc + d * max_pos).
  // z: opaque zero, so LICM cannot hoist 64 loop-invariant addresses out of the layer loop
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  const uint4* k4 = reinterpret_cast<const uint4*>(kc) + z;
  const uint16_t* v2 = vc + z;
  char* ksb = reinterpret_cast<char*>(sm.ks) + z;
  char* vsb = reinterpret_cast<char*>(sm.vs) + z;
  const int rsub = lane >> 4, sl = lane & 15;
#pragma unroll
  for (int j = 0; j < SPL / 4; ++j) {
    const int p = 4 * j + rsub;
    __builtin_amdgcn_global_load_lds(k4 + (size_t)p * 16 + (sl ^ (p & 15)),
                                     (lds_void*)(ksb + 1024 * j), 16, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const int d = 4 * j + rsub;
    __builtin_amdgcn_global_load_lds(v2 + (size_t)d * max_pos + 8 * (sl ^ (d & 15)),
                                     (lds_void*)(vsb + 1024 * j), 16, 0, 0);
  }
}

// ---- control wave: attention of one (kv head, split) -------------------------------------
// qkv: this layer's qkv vector (q[24][128] | k[8][128] | v[8][128], k / v bf16-exact fp32)
__device__ __forceinline__ void attention(Smem& sm, const MegaArgs& a, int l, int kvh, int split,
                                          int nsplit, int L, const float* qkv, int lane,
                                          bool& dead) {
  const int pos = L - 1, p0 = split * SPL;
  drain();  // the LDS-DMA K / V staging of this split has landed
  // the new position's k / v into LDS (bf16, like the cache)
  if (pos >= p0 && pos < p0 + SPL) {
    const int pn = pos - p0;
    const float k0 = ld_sc1(qkv + QD + kvh * 128 + 2 * lane);
    const float k1 = ld_sc1(qkv + QD + kvh * 128 + 2 * lane + 1);
    const float v0 = ld_sc1(qkv + QD + KVH * 128 + kvh * 128 + lane);
    const float v1 = ld_sc1(qkv + QD + KVH * 128 + kvh * 128 + lane + 64);
    uint32_t* krow = reinterpret_cast<uint32_t*>(&sm.ks[pn * 16]);
    krow[(((2 * lane) >> 3) ^ (pn & 15)) * 4 + ((2 * lane) & 7) / 2] = pack2_bf16(k0, k1);
    uint16_t* vrow0 = reinterpret_cast<uint16_t*>(&sm.vs[lane * 16]);
    uint16_t* vrow1 = reinterpret_cast<uint16_t*>(&sm.vs[(lane + 64) * 16]);
    vrow0[((pn >> 3) ^ (lane & 15)) * 8 + (pn & 7)] = f32_to_bf16(v0);
    vrow1[((pn >> 3) ^ ((lane + 64) & 15)) * 8 + (pn & 7)] = f32_to_bf16(v1);
  }
  const int c = lane & 15, g = lane >> 4, rr = lane & 15;
  // Q^T fragments: lane (head c, group g) holds q[c][32 st + 8 g + j] in 3 bf16 parts
  bf16x8 qf[3][4];
  {
    const int hq = c < GRP ? c : 0;
    const float* qb = qkv + (kvh * GRP + hq) * 128 + 8 * g;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const int i4 = (int)((qb + 32 * st) - qkv) / 4;
      const float4 lo = ld4_sc1(qkv, i4), hi = ld4_sc1(qkv, i4 + 1);
      float x[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
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
#pragma unroll
  for (int ch = 0; ch < SPL / 32; ++ch) {
    const int lb = 32 * ch, base = p0 + lb;
    if (base >= L) break;  // wave-uniform
    f32x4 sc[2];
#pragma unroll
    for (int T = 0; T < 2; ++T) {
      const int pl = lb + 8 * (rr >> 2) + 4 * T + (rr & 3);
      sc[T] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const bf16x8 kb = __builtin_bit_cast(bf16x8, sm.ks[pl * 16 + ((4 * st + g) ^ (pl & 15))]);
#pragma unroll
        for (int pt = 0; pt < 3; ++pt)
          sc[T] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kb, qf[pt][st], sc[T], 0, 0, 0);
      }
    }
    float sv[8];
    float mc = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int p = base + 8 * g + j;
      sv[j] = p < L ? sc[j >> 2][j & 3] * a.att_scale : -INFINITY;
      mc = fmaxf(mc, sv[j]);
    }
    mc = fmaxf(mc, __shfl_xor(mc, 16, 64));
    mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
    const float Mn = fmaxf(M, mc);
    const float alpha = expf(M - Mn);
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
      const int d = 16 * t + c;
      const bf16x8 vb = __builtin_bit_cast(bf16x8, sm.vs[d * 16 + (((lb >> 3) + g) ^ (d & 15))]);
#pragma unroll
      for (int pt = 0; pt < 3; ++pt)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf[pt], vb, acc[t], 0, 0, 0);
    }
  }
  // lanes g == 0 hold O^T rows (head i) at dims 16 t + c; (M, lsum) of head c in lane c
  float* att = a.ws + (size_t)l * MEGA_WS_LAYER + MEGA_OFF_ATT + kvh * GRP * 128;
  int* sync = a.sync + l * MEGA_SYNC_LAYER;
  if (nsplit == 1) {
    float inv[GRP];
#pragma unroll
    for (int i = 0; i < GRP; ++i) inv[i] = 1.0f / __shfl(lsum, i, 64);
    if (g == 0) {
#pragma unroll
      for (int i = 0; i < GRP; ++i)
#pragma unroll
        for (int t = 0; t < 8; ++t) st_sc1(att + i * 128 + 16 * t + c, acc[t][i] * inv[i]);
    }
    signal(sync + MEGA_SYNC_DONE);
    return;
  }
  float* part = a.part + ((size_t)(l * KVH + kvh) * a.nsplit_cap) * PART;
  float* mine = part + (size_t)split * PART;
  if (g == 0) {
#pragma unroll
    for (int i = 0; i < GRP; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t) st_sc1(mine + i * 128 + 16 * t + c, acc[t][i]);
  }
  if (lane < GRP) {
    st_sc1(mine + 3 * 128 + lane, M);
    st_sc1(mine + 3 * 128 + GRP + lane, lsum);
  }
  drain();
  int t = 0;
  if (lane == 0)
    t = __hip_atomic_fetch_add(sync + MEGA_SYNC_TICK + kvh, 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
  t = __builtin_amdgcn_readfirstlane(t);
  if (t != nsplit - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // last arriver: merge every split in batches of 8 (online rescale across batches).
  // lane owns outputs o = lane + 64 k (k < 6): head o >> 7, dim o & 127
  constexpr int MB = 4;
  float Mr[GRP], den[GRP], num[6];
#pragma unroll
  for (int i = 0; i < GRP; ++i) { Mr[i] = -INFINITY; den[i] = 0.f; }
#pragma unroll
  for (int k = 0; k < 6; ++k) num[k] = 0.f;
  for (int s0 = 0; s0 < nsplit; s0 += MB) {
    const int nb = min(MB, nsplit - s0);
    // (m, l) of split s0 + (lane / 6), entry lane % 6, in lanes < 6 nb
    const float ml = lane < 6 * nb ? ld_sc1(part + (size_t)(s0 + lane / 6) * PART + 384 + lane % 6) : 0.f;
    float av[MB][6];
#pragma unroll
    for (int s = 0; s < MB; ++s)
#pragma unroll
      for (int k = 0; k < 6; ++k)
        av[s][k] = ld_sc1(part + (size_t)(s0 + min(s, nb - 1)) * PART + lane + 64 * k);
    float Ms[MB][GRP], Ls[MB][GRP];
#pragma unroll
    for (int s = 0; s < MB; ++s)
#pragma unroll
      for (int i = 0; i < GRP; ++i) {
        Ms[s][i] = __shfl(ml, 6 * s + i, 64);
        Ls[s][i] = __shfl(ml, 6 * s + GRP + i, 64);
      }
    float Mn[GRP], f_old[GRP];
#pragma unroll
    for (int i = 0; i < GRP; ++i) {
      Mn[i] = Mr[i];
#pragma unroll
      for (int s = 0; s < MB; ++s)
        if (s < nb) Mn[i] = fmaxf(Mn[i], Ms[s][i]);
      f_old[i] = Mr[i] == -INFINITY ? 0.f : expf(Mr[i] - Mn[i]);
      den[i] *= f_old[i];
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) num[k] *= f_old[k >> 1];  // output lane + 64 k is head k / 2
#pragma unroll
    for (int s = 0; s < MB; ++s) {
      if (s >= nb) break;
      float f[GRP];
#pragma unroll
      for (int i = 0; i < GRP; ++i) {
        f[i] = expf(Ms[s][i] - Mn[i]);
        den[i] = fmaf(f[i], Ls[s][i], den[i]);
      }
#pragma unroll
      for (int k = 0; k < 6; ++k) num[k] = fmaf(f[k >> 1], av[s][k], num[k]);
    }
#pragma unroll
    for (int i = 0; i < GRP; ++i) Mr[i] = Mn[i];
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) st_sc1(att + lane + 64 * k, num[k] / den[k >> 1]);
  signal(sync + MEGA_SYNC_DONE);
}

// ---- the kernel ---------------------------------------------------------------------------
template <bool F8, int D>
__global__ __launch_bounds__(NTH, 1) void mega_kernel(MegaArgs a) {
  using G = Geo<F8>;
  static_assert(D <= G::U && D <= G::UQ + G::UO + G::UG, "ring deeper than a layer");
  __shared__ Smem sm;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int layers = a.layers;

  if (w < WPB) {
    // ===================== compute waves: the weight ring =====================
    // wave-uniform phase bases of the current layer (buffer descriptors in SGPRs; every unit
    // load is base + 16 lane (one VGPR) + a constant soffset: no per-unit address registers)
    const char* bq = static_cast<const char*>(a.wqkv) + (size_t)(b * BQ + w * RQ) * G::RBH;
    const char* bo = static_cast<const char*>(a.wo) + (size_t)(b * BO + w * RO) * G::RBH;
    const char* bg = static_cast<const char*>(a.wgu) + (size_t)(b * BG + w * RG) * G::RBH;
    const char* bd = static_cast<const char*>(a.wd) + (size_t)(b * BD + w * RD) * G::RBF;
    constexpr size_t SQ = (size_t)QKVR * G::RBH, SO = (size_t)H * G::RBH;
    constexpr size_t SG = (size_t)2 * FF * G::RBH, SD = (size_t)H * G::RBF;
    const char* dummy = reinterpret_cast<const char*>(a.dummy);
    const int voff = 16 * lane;
    auto rsrc = [](const char* p) {
      return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(p), 0, 0x7fffffff, 0x00020000);
    };
    __amdgpu_buffer_rsrc_t rq = rsrc(bq), ro = rsrc(bo), rg = rsrc(bg), rd = rsrc(bd);
    __amdgpu_buffer_rsrc_t nrq, nro, nrg, nrd;  // next layer (or the dummy)
    uint4 ring[D];
    // unit v (0 .. U-1) of the layer whose phase descriptors are (q, o, g, d)
    // z: an opaque zero (asm) added to every constant offset, so LICM cannot hoist 192
    // distinct soffset constants out of the layer loop into (spilled) SGPRs
    auto uload = [&](int v, __amdgpu_buffer_rsrc_t q, __amdgpu_buffer_rsrc_t o,
                     __amdgpu_buffer_rsrc_t g, __amdgpu_buffer_rsrc_t d, int z) -> uint4 {
      __amdgpu_buffer_rsrc_t r;
      int off;
      if (v < G::OO) { r = q; off = (v / G::KH) * (int)G::RBH + (v % G::KH) * 1024; }
      else if (v < G::OG) { r = o; off = ((v - G::OO) / G::KH) * (int)G::RBH + ((v - G::OO) % G::KH) * 1024; }
      else if (v < G::OD) { r = g; off = ((v - G::OG) / G::KH) * (int)G::RBH + ((v - G::OG) % G::KH) * 1024; }
      else { r = d; off = ((v - G::OD) / G::KF) * (int)G::RBF + ((v - G::OD) % G::KF) * 1024; }
      const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, voff, off + z, 2 /* nt */);
      return make_uint4(x.x, x.y, x.z, x.w);
    };
    // activations of chunk ch (PL float4 planes)
    auto xread = [&](int ch, float4 (&x)[G::PL]) {
#pragma unroll
      for (int q = 0; q < G::PL; ++q) x[q] = sm.xs[q * G::PS + ch * 64 + lane];
    };
    // One phase: N units at layer offset OFF, KCH units per row, RPW rows.  Per unit: refill
    // its ring slot with unit u + D, read the next unit's activations, FMA this unit into its
    // row's accumulator; an empty asm pins that order (loads ahead, no hoisted LDS reads).
    // Rows are reduced across the wave once, at the end of the phase.
    auto phase = [&](auto OFFc, auto Nc, auto KCHc, auto RPWc) {
      constexpr int OFF = decltype(OFFc)::value, N = decltype(Nc)::value;
      constexpr int KCH = decltype(KCHc)::value, RPW = decltype(RPWc)::value;
      float acc[RPW];
#pragma unroll
      for (int r = 0; r < RPW; ++r) acc[r] = 0.f;
      float4 xc[G::PL], xn[G::PL];
      int z;
      asm volatile("s_mov_b32 %0, 0" : "=s"(z));
      xread(0, xc);
#pragma unroll
      for (int k = 0; k < N; ++k) {
        const int u = OFF + k, row = k / KCH;
        const uint4 wv = ring[u % D];
        const int v = u + D;
        ring[u % D] = v < G::U ? uload(v, rq, ro, rg, rd, z) : uload(v - G::U, nrq, nro, nrg, nrd, z);
        if (k + 1 < N) xread((k + 1) % KCH, xn);
        float t = acc[row];
        if (F8) {
          const uint32_t wd[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x2_t lo = __builtin_amdgcn_cvt_pk_f32_fp8(wd[q], false);
            const f32x2_t hi = __builtin_amdgcn_cvt_pk_f32_fp8(wd[q], true);
            t = fmaf(lo.x, xc[q].x, t);
            t = fmaf(lo.y, xc[q].y, t);
            t = fmaf(hi.x, xc[q].z, t);
            t = fmaf(hi.y, xc[q].w, t);
          }
        } else {
          t = dot8(wv, xc[0], xc[G::PL - 1], t);
        }
        acc[row] = t;
        asm volatile("" : "+v"(acc[row]) :: "memory");
#pragma unroll
        for (int q = 0; q < G::PL; ++q) xc[q] = xn[q];
      }
      // rows -> LDS: lane r ends up holding the total of row r
      float mine = 0.f;
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        const float s = wave_sum(acc[r]);
        mine = lane == r ? s : mine;
      }
      if (lane < RPW) sm.rowres[w * RPW + lane] = mine;
      lds_barrier();  // A: row results in LDS
      lds_barrier();  // B: next activation vector staged
    };
#pragma unroll
    for (int v = 0; v < D; ++v) ring[v] = uload(v, rq, ro, rg, rd, 0);
    lds_barrier();  // initial activation staged
    for (int l = 0; l < layers; ++l) {
      const bool more = l + 1 < layers;
      if (more) { bq += SQ; bo += SO; bg += SG; bd += SD; }
      nrq = rsrc(more ? bq : dummy); nro = rsrc(more ? bo : dummy);
      nrg = rsrc(more ? bg : dummy); nrd = rsrc(more ? bd : dummy);
      phase(std::integral_constant<int, 0>{}, std::integral_constant<int, G::UQ>{},
            std::integral_constant<int, G::KH>{}, std::integral_constant<int, RQ>{});
      phase(std::integral_constant<int, G::OO>{}, std::integral_constant<int, G::UO>{},
            std::integral_constant<int, G::KH>{}, std::integral_constant<int, RO>{});
      phase(std::integral_constant<int, G::OG>{}, std::integral_constant<int, G::UG>{},
            std::integral_constant<int, G::KH>{}, std::integral_constant<int, RG>{});
      phase(std::integral_constant<int, G::OD>{}, std::integral_constant<int, G::UD>{},
            std::integral_constant<int, G::KF>{}, std::integral_constant<int, RD>{});
      rq = nrq; ro = nro; rg = nrg; rd = nrd;
    }
    return;
  }

  // ===================== control wave =====================
  // optional event trace (wall clock, 100 MHz): trace[b][l][ev]
  long long* tr = a.trace ? a.trace + (size_t)b * layers * MEGA_TRACE_EV : nullptr;
#define MEGA_EV(l_, ev_)                                                      \
  if (tr && lane == 0) tr[(size_t)(l_) * MEGA_TRACE_EV + (ev_)] = wall_clock64();
  bool dead = false;
  int* status = a.sync + layers * MEGA_SYNC_LAYER;
  const int slot = a.row_slot[0];
  const int L = a.row_pos[0] + 1, pos = L - 1;
  const int nsplit = (L + SPL - 1) / SPL;
  const bool att_blk = b < KVH * nsplit;
  const int kvh = b % KVH, split = b / KVH;
  const size_t kv_head = ((size_t)slot * KVH + kvh);
  auto kv_src = [&](int l, const uint16_t** kc, const uint16_t** vc) {
    *kc = a.kcache + (size_t)l * a.kv_layer_elems + (kv_head * a.max_pos + split * SPL) * 128;
    *vc = a.vcache + (size_t)l * a.kv_layer_elems + kv_head * 128 * a.max_pos + split * SPL;
  };
  // residual rows of this block (o / down rows: 12 b .. 12 b + 11) live in lanes 0..11
  float hres = lane < BO ? a.h_in[b * BO + lane] : 0.f;
  float ssq = stage_x<F8, H>(sm, a.h_in, a.attn_norm, lane);
  lds_barrier();  // compute waves start on layer 0's qkv rows
  if (att_blk) {  // layer 0's K / V of this split, under the qkv stream
    const uint16_t *kc, *vc;
    kv_src(0, &kc, &vc);
    stage_kv(sm, kc, vc, a.max_pos, lane);
  }
  for (int l = 0; l < layers; ++l) {
    // an opaque zero folded into the lane index: nothing lane-dependent is loop-invariant,
    // so LICM cannot hoist (and spill, then reload behind vmcnt(0)) per-lane addresses
    int zl;
    asm volatile("s_mov_b32 %0, 0" : "=s"(zl));
    const int lane = (tid & 63) + zl;
    float* ws = a.ws + (size_t)l * MEGA_WS_LAYER;
    int* sync = a.sync + l * MEGA_SYNC_LAYER;
    const bool last = l + 1 == layers;
    // ---------------- qkv ----------------
    lds_barrier();  // A
    MEGA_EV(l, 0);
    {
      const float sQ = 1.0f / sqrtf(ssq / (float)H + a.eps);
      float* qkv = ws + MEGA_OFF_QKV;
      if (lane < BQ / 2) {
        const int n0 = b * BQ + 2 * lane;  // packed rows n0, n0 + 1
        float x1 = sm.rowres[2 * lane] * sQ, x2 = sm.rowres[2 * lane + 1] * sQ;
        if (F8) {
          x1 *= a.sqkv[(size_t)l * QKVR + n0];
          x2 *= a.sqkv[(size_t)l * QKVR + n0 + 1];
        }
        const int hh = n0 >> 7, within = n0 & 127;
        if (hh < (QD >> 7) + KVH) {
          const int p = within >> 1;
          const float cs = a.rope_cos[(size_t)pos * 64 + p], sn = a.rope_sin[(size_t)pos * 64 + p];
          const float o1 = x1 * cs - x2 * sn, o2 = x2 * cs + x1 * sn;
          if (hh < (QD >> 7)) {
            st_sc1(qkv + hh * 128 + p, o1);
            st_sc1(qkv + hh * 128 + p + 64, o2);
          } else {
            const int kh = hh - (QD >> 7);
            const uint16_t k1 = f32_to_bf16(o1), k2 = f32_to_bf16(o2);
            st_sc1(qkv + QD + kh * 128 + p, bf16_to_f32(k1));
            st_sc1(qkv + QD + kh * 128 + p + 64, bf16_to_f32(k2));
            uint16_t* kc = a.kcache + (size_t)l * a.kv_layer_elems +
                           (((size_t)slot * KVH + kh) * a.max_pos + pos) * 128;
            kc[p] = k1;
            kc[p + 64] = k2;
          }
        } else {
          const int vh = hh - (QD >> 7) - KVH;
          const uint16_t v1 = f32_to_bf16(x1), v2 = f32_to_bf16(x2);
          st_sc1(qkv + QD + KVH * 128 + vh * 128 + within, bf16_to_f32(v1));
          st_sc1(qkv + QD + KVH * 128 + vh * 128 + within + 1, bf16_to_f32(v2));
          uint16_t* vc = a.vcache + (size_t)l * a.kv_layer_elems +
                         ((size_t)slot * KVH + vh) * 128 * a.max_pos;
          vc[(size_t)within * a.max_pos + pos] = v1;
          vc[(size_t)(within + 1) * a.max_pos + pos] = v2;
        }
      }
      set_flag(a.flags + (l * 4 + 0) * NB + b);
      MEGA_EV(l, 1);
      if (att_blk) {
        wait_flags(a.flags + (l * 4 + 0) * NB, status, 1, dead);
        MEGA_EV(l, 2);
        attention(sm, a, l, kvh, split, nsplit, L, qkv, lane, dead);
        MEGA_EV(l, 3);
      }
      wait_ge(sync + MEGA_SYNC_DONE, KVH, status, 2, dead);
      MEGA_EV(l, 4);
      stage_x<F8, QD>(sm, ws + MEGA_OFF_ATT, nullptr, lane);
    }
    MEGA_EV(l, 5);
    lds_barrier();  // B
    // ---------------- o-proj + residual ----------------
    lds_barrier();  // A
    MEGA_EV(l, 6);
    {
      if (lane < BO) {
        const int n = b * BO + lane;
        float y = sm.rowres[lane];
        if (F8) y *= a.so[(size_t)l * H + n];
        hres += y;
        st_sc1(ws + MEGA_OFF_HA + n, hres);
      }
      set_flag(a.flags + (l * 4 + 1) * NB + b);
      wait_flags(a.flags + (l * 4 + 1) * NB, status, 3, dead);
      MEGA_EV(l, 7);
      ssq = stage_x<F8, H>(sm, ws + MEGA_OFF_HA, a.mlp_norm + (size_t)l * H, lane);
    }
    MEGA_EV(l, 8);
    lds_barrier();  // B
    if (att_blk && !last) {  // next layer's K / V of this split, under the gate/up stream
      const uint16_t *kc, *vc;
      kv_src(l + 1, &kc, &vc);
      stage_kv(sm, kc, vc, a.max_pos, lane);
    }
    MEGA_EV(l, 9);
    // ---------------- gate/up + SiLU*up ----------------
    lds_barrier();  // A
    MEGA_EV(l, 10);
    {
      const float sG = 1.0f / sqrtf(ssq / (float)H + a.eps);
      if (lane < BG / 2) {
        const int n0 = b * BG + 2 * lane;
        float gt = sm.rowres[2 * lane] * sG, up = sm.rowres[2 * lane + 1] * sG;
        if (F8) {
          gt *= a.sgu[(size_t)l * 2 * FF + n0];
          up *= a.sgu[(size_t)l * 2 * FF + n0 + 1];
        }
        st_sc1(ws + MEGA_OFF_ACT + (n0 >> 1), gt / (1.0f + expf(-gt)) * up);
      }
      set_flag(a.flags + (l * 4 + 2) * NB + b);
      wait_flags(a.flags + (l * 4 + 2) * NB, status, 4, dead);
      MEGA_EV(l, 11);
      stage_x<F8, FF>(sm, ws + MEGA_OFF_ACT, nullptr, lane);
    }
    MEGA_EV(l, 12);
    lds_barrier();  // B
    // ---------------- down + residual ----------------
    lds_barrier();  // A
    MEGA_EV(l, 13);
    {
      float* hout = last ? a.h_out : ws + MEGA_OFF_HB;
      if (lane < BD) {
        const int n = b * BD + lane;
        float y = sm.rowres[lane];
        if (F8) y *= a.sd[(size_t)l * H + n];
        hres += y;
        st_sc1(hout + n, hres);
      }
      set_flag(a.flags + (l * 4 + 3) * NB + b);
      if (!last) {
        wait_flags(a.flags + (l * 4 + 3) * NB, status, 5, dead);
        MEGA_EV(l, 14);
        ssq = stage_x<F8, H>(sm, hout, a.attn_norm + (size_t)(l + 1) * H, lane);
      }
    }
    MEGA_EV(l, 15);
    lds_barrier();  // B
  }
}

#undef MEGA_EV
}  // namespace mega

// Host side ----------------------------------------------------------------------------------
template <int D>
static const void* mega_fn(int f8) {
  return f8 ? reinterpret_cast<const void*>(&mega::mega_kernel<true, D>)
            : reinterpret_cast<const void*>(&mega::mega_kernel<false, D>);
}
static const void* mega_pick(int f8, int ring) {
  switch (ring) {
    case 8: return mega_fn<8>(f8);
    case 16: return mega_fn<16>(f8);
    case 32: return mega_fn<32>(f8);
    case 48: return mega_fn<48>(f8);
    default: return nullptr;
  }
}

hipError_t launch_mega(const MegaArgs& a, hipStream_t st) {
  const void* fn = mega_pick(a.f8, a.ring);
  if (!fn) return hipErrorInvalidValue;
  void* args[] = {const_cast<MegaArgs*>(&a)};
  return hipLaunchKernel(fn, dim3(mega::NB), dim3(mega::NTH), args, 0, st);
}

// 1 if every block of the launch can be resident at once on this device
hipError_t mega_resident(int device, int f8, int ring, int* ok) {
  *ok = 0;
  const void* fn = mega_pick(f8, ring);
  if (!fn) return hipErrorInvalidValue;
  int cus = 0, nblk = 0;
  hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess) return e;
  e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nblk, fn, mega::NTH, 0);
  if (e != hipSuccess) return e;
  *ok = (long)cus * nblk >= mega::NB ? 1 : 0;
  return hipSuccess;
}

}  // namespace mx
