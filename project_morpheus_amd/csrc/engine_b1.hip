// Persistent one-row decode engine (option b1_engine): every layer of one B = 1 decode step
// in ONE launch, so the HBM weight stream never stops at a layer's dependency edges.
//
// Replaces the per-kernel hipGraph step (qkv -> attention -> o-proj -> gate/up -> down, 140
// launches per step) for the single-stream decode of vLLM's engine
// (Orpheus-TTS/orpheus_tts_pypi/orpheus_tts/engine_class.py:117, CUDA-graph decode) and
// llama.cpp (Morpheus_Client/tts_engine/llama_local.py:77).  Design: MI355X_MICROARCH.md
// "Persistent kernels" price list, rows ldsdma-fill / nt-weights / engine-vs-launches.
//
// One workgroup per CU (grid = CU count, all co-resident), 5 waves:
//   * wave 0 = LOADER: walks the CU's static weight schedule (every layer: its rows of wqkv,
//     wo, wgu, wd, contiguous row ranges) and streams it into an LDS ring of 16 KB slots with
//     LDS-DMA (global_load_lds_dwordx4 nt: one 1 KB wave instruction per 64 lanes x 16 B),
//     two slots in flight, publishing a slot (LDS word = sequence number) once its loads have
//     landed (counted vmcnt).  It never waits on data, only on a free ring slot, so the
//     stream runs on across every dependency edge of the layer.
//   * waves 1..4 = CONSUMERS: gather each phase's input vector, compute their slots (slot k
//     -> wave k mod 4) from LDS, and publish outputs.
// Cross-CU hand-offs are 8-byte granules {fp32 value, u32 tag}, one write-through (sc1) store
// each, read back with sc1 loads until every tag matches (MI355X_MICROARCH.md granule rows; no
// counters, no fences).  tag = epoch << 8 | layer << 3 | phase; the epoch advances once per
// launch (the last workgroup to finish bumps it), so a granule of an earlier step never
// matches.
//
// Phases per layer (each CU owns a contiguous row range of every matrix):
//   QKV  : gather h (layer input), RMSNorm folded (y = W(x*w) * rsqrt(mean x^2 + eps)); rows of
//          the packed wqkv -> RoPE -> q / k / v granules (+ the bf16 K/V cache at pos).
//   ATTN : items (kv head, split of 128 positions) on spread CUs: the cached positions [0, L-1)
//          on bf16 MFMA exactly as attn_kernel (three bf16 parts of q and p), position L-1 from
//          the k / v granules (bf16-rounded, as the cache will hold it); split partials merged
//          by the last arriving split (ticket), which publishes the attention output granules.
//   O    : gather att; rows of wo; h1 = h + y granules.
//   GU   : gather h1 (RMSNorm); rows of wgu (gate/up interleaved); silu(g) u granules.
//   DOWN : gather act; rows of wd; h2 = h1 + y granules (the next layer's input); the last
//          layer also stores h2 to the decode row's hidden state for the lm_head launch.
// Every wait is bounded (100 MHz realtime clock): a stuck hand-off sets *status and every wave
// leaves, so a launch always drains.
#include "mx_common.h"
#include "mx_llm_kernels.h"
#include "mx_engine.h"

#include <algorithm>

namespace mx {
namespace eng {

constexpr int NC = 4;                // consumer waves (after the NL loader waves)
constexpr int SLOT = 16384;          // ring slot bytes
constexpr int SL = 128;              // attention split length (positions; 4 waves x 32)
constexpr int RING_MAX = 7;          // ring slots (LDS: 112 KB)
constexpr int XA_MAX = 3072;         // staged hidden-width activation (floats)
constexpr int XB_MAX = 8192;         // staged ffn-width activation / attention scratch (floats)
enum { PH_QKV = 0, PH_ATT = 1, PH_H1 = 2, PH_ACT = 3, PH_H2 = 4 };

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_cvoid;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

// ---- granules (8 bytes: value, tag), write-through stores / loads -------------------------
__device__ __forceinline__ void gput(uint2* g, int i, float v, uint32_t tag) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(g, 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(v), tag}, r, i * 8, 0, 16);
}
__device__ __forceinline__ u32x4v gget2(const uint2* g, int i) {  // granules i, i + 1
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint2*>(g), 0, 0x7fffffff, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b128(r, i * 8, 0, 16);
}
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- LDS words shared by the waves of the workgroup ------------------------------------
__device__ __forceinline__ int lds_ld(const int* p) {
  return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Ring flags: relaxed LDS accesses with compiler-only fences.  A release / acquire at
// workgroup scope makes the compiler wait for EVERY outstanding vector-memory operation of the
// wave (vmcnt(0)), which would drain the loader's in-flight LDS-DMA at each publish; the
// ordering is explicit instead: the loader publishes a slot after a counted vmcnt wait (its
// DMA has landed), and LDS instructions of one wave execute in order.
__device__ __forceinline__ int ring_ld(const int* p) {
  const int v = __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  asm volatile("" ::: "memory");
  return v;
}
__device__ __forceinline__ void ring_st(int* p, int v) {
  asm volatile("" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// The loader's own flag accesses, as inline asm: with LDS-DMA in flight the compiler puts a
// vmcnt(0) in front of any LDS instruction it emits (it cannot tell the flag from the DMA
// target), which would drain the weight stream at every publish.  The loader's DMA targets are
// the ring slots only, never these words.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(size_t)((const __attribute__((address_space(3))) char*)p);
}
__device__ __forceinline__ int loader_ld(const int* p) {
  int v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}
__device__ __forceinline__ void loader_st(int* p, int v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}

struct Ctl {           // LDS control block
  int ready[8];        // ring position -> sequence number of the slot it holds (k + 1)
  int freed[8];        // ring position -> sequence number of the slot consumed from it
  int bar;             // consumer barrier arrivals (monotonic)
  int abort_;          // a wave of this workgroup gave up
  int last;            // attention ticket: this CU merges
  int pad;
  float ss[NC];        // per-wave partial sums of squares
  float res1[32], res2[32];  // this CU's residual slice (o-proj / down rows)
  float rope[32][2];   // cos / sin at the step's position for this CU's qkv row pairs
  float scl[2][160];   // e4m3 row scales of this CU's rows, by layer parity:
                       // [0, 32) qkv, [32, 64) o, [64, 128) gate/up, [128, 160) down
};
constexpr int SC_QKV = 0, SC_O = 32, SC_GU = 64, SC_D = 128;

struct Clock {
  uint64_t deadline;
  __device__ bool expired() const { return __builtin_amdgcn_s_memrealtime() > deadline; }
};

// one matrix phase of the static weight schedule, for this CU
struct Ph {
  const uint8_t* W;    // layer 0 base
  size_t layer_bytes;  // bytes per layer
  int r0, r1;          // this CU's rows
  int rps, ips;        // rows per slot, 1 KB instructions per slot
  int rowbytes, nslots;
  int N;
};

__device__ __forceinline__ Ph make_ph(const void* W, int N, int K, int esz, int G, int c,
                                      bool pair) {
  Ph p;
  p.W = static_cast<const uint8_t*>(W);
  p.N = N;
  p.rowbytes = K * esz;
  p.layer_bytes = (size_t)N * p.rowbytes;
  int per = (N + G - 1) / G;
  if (pair) per = (per + 1) & ~1;
  p.r0 = min(N, c * per);
  p.r1 = min(N, p.r0 + per);
  p.rps = min(SLOT / p.rowbytes, 4);  // (the consumers' slot_dot handles up to 4 rows)
  if (pair) p.rps &= ~1;
  p.ips = p.rps * p.rowbytes / 1024;
  p.nslots = (p.r1 - p.r0 + p.rps - 1) / p.rps;
  return p;
}

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// vmcnt <= n, for the in-flight counts the schedule produces (slots of 12 / 16 instructions,
// DEPTH newer slots); any other n waits for the largest listed count below it
__device__ __forceinline__ void wait_vm_n(int n) {
  if (n >= 48) wait_vm<48>();
  else if (n >= 44) wait_vm<44>();
  else if (n >= 40) wait_vm<40>();
  else if (n >= 36) wait_vm<36>();
  else if (n >= 32) wait_vm<32>();
  else if (n >= 28) wait_vm<28>();
  else if (n >= 24) wait_vm<24>();
  else if (n >= 16) wait_vm<16>();
  else if (n >= 12) wait_vm<12>();
  else wait_vm<0>();
}

// ---------------------------------------------------------------------------------------
// consumer helpers
// ---------------------------------------------------------------------------------------
// consumer-only barrier (the loader never joins): monotonic arrival count in LDS
__device__ __forceinline__ bool cbar(Ctl* ctl, int& gen, const Clock& clk, int* status) {
  gen += NC;
  asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_fetch_add(&ctl->bar, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  int spins = 0;
  while (lds_ld(&ctl->bar) < gen) {
    __builtin_amdgcn_s_sleep(1);
    if ((spins++ & 255) == 0 && (lds_ld(&ctl->abort_) || clk.expired())) {
      lds_st(&ctl->abort_, 1);
      if ((threadIdx.x & 63) == 0) __hip_atomic_store(status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
  }
  return true;
}

// Gather n granules of `tag` (cooperatively: consumer thread ct of 256 takes pairs ct, ct+256,
// ...) into the staged-activation planes X (gemv1 layout: element k -> plane (k % EPC) / 4,
// chunk k / EPC), optionally multiplied by w[k]; returns this thread's sum of squares of the
// RAW values.  Values in [rs0, rs0 + nres) are also saved to res[].
template <int EPC>
__device__ __forceinline__ bool gather(const uint2* g, int n, uint32_t tag, float* X, int KC,
                                       const float* w, float* res, int rs0, int nres, int ct,
                                       float& ss, Ctl* ctl, const Clock& clk, int* status,
                                       bool skip = false) {
  ss = 0.f;
  if (skip) return true;  // timing experiment (EngineArgs::dbg & 1): no hand-off waits
  constexpr int B = 8;  // granule pairs in flight per thread (n <= 4096 in one round)
  for (int base = 2 * ct; base < n; base += 2 * 256 * B) {
    u32x4v v[B];
    bool ok[B];
    float2 wv[B];
#pragma unroll
    for (int j = 0; j < B; ++j) {
      const int i = base + 2 * 256 * j;
      v[j] = i < n ? gget2(g, i) : u32x4v{0u, tag, 0u, tag};
      // the norm weights go out with the granules (not after the wait)
      wv[j] = (w && i < n) ? *reinterpret_cast<const float2*>(w + i) : make_float2(1.f, 1.f);
    }
#pragma unroll
    for (int j = 0; j < B; ++j) ok[j] = v[j].y == tag && v[j].w == tag;
    int spins = 0;
    while (true) {
      bool all = true;
#pragma unroll
      for (int j = 0; j < B; ++j) all &= ok[j];
      if (all) break;
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int j = 0; j < B; ++j) {
        if (!ok[j]) {
          v[j] = gget2(g, base + 2 * 256 * j);
          ok[j] = v[j].y == tag && v[j].w == tag;
        }
      }
      if ((spins++ & 63) == 0 && (lds_ld(&ctl->abort_) || clk.expired())) {
        lds_st(&ctl->abort_, 1);
        __hip_atomic_store(status, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
      }
    }
#pragma unroll
    for (int j = 0; j < B; ++j) {
      const int i = base + 2 * 256 * j;
      if (i >= n) continue;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int k = i + e;
        const float x = __uint_as_float(e ? v[j].z : v[j].x);
        ss = fmaf(x, x, ss);
        if (k >= rs0 && k < rs0 + nres) res[k - rs0] = x;
        const float xw = x * (e ? wv[j].y : wv[j].x);
        const int m = k / EPC, q = (k % EPC) >> 2;
        X[(q * KC + m) * 4 + (k & 3)] = xw;
      }
    }
  }
  return true;
}

// Before a gather: poll one WITNESS granule per producer (the last of its contiguous range of
// `per` outputs) instead of sweeping the whole vector, so 256 CUs waiting on an edge put ~4 KB
// each per poll round on the fabric, not the vector (24-64 KB); then join the consumer barrier.
// The sweep that follows is then almost always one pass.
__device__ __forceinline__ bool witness(const uint2* g, int n, int per, uint32_t tag, int ct,
                                        Ctl* ctl, int& gen, const Clock& clk, int* status,
                                        bool skip);

// 64-lane sum: the four in-row steps on DPP (quad_perm [1,0,3,2], [2,3,0,1], row_ror 4, 8:
// VALU, no LDS round trip), the two cross-row steps as lane shuffles
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_sum_fast(float v) {
  v += dpp<0xb1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4e>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x124>(v);  // row_ror:4
  v += dpp<0x128>(v);  // row_ror:8
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// Dot products of the rows of one ring slot with the staged activation: rows j < nr of the
// slot (RPS per slot, KCL 16-byte chunks per lane per row; row j's chunk m at slot[j KC + m],
// lane takes m = lane + 64 i).  Every LDS read of a batch of CH chunks is issued before any
// FMA (one LDS round trip per batch, not per chunk); rows past nr re-read row nr - 1 and are
// ignored by the caller.
// largest divisor of kcl that is <= lim (chunks per batch of LDS reads)
constexpr int batch_of(int kcl, int lim) {
  for (int c = lim; c > 1; --c)
    if (kcl % c == 0) return c;
  return 1;
}

template <bool F8, int RPS, int KCL>
__device__ __forceinline__ float4 slot_dot_t(const uint4* slot, const float4* X, int KC, int nr,
                                             int lane) {
  constexpr int PL = F8 ? 4 : 2;
  constexpr int CH = batch_of(KCL, F8 ? 2 : 4);
  static_assert(KCL % CH == 0, "chunk batches");
  float acc[RPS];
#pragma unroll
  for (int j = 0; j < RPS; ++j) acc[j] = 0.f;
#pragma unroll
  for (int c0 = 0; c0 < KCL; c0 += CH) {
    float4 xq[CH][PL];
    uint4 w[CH][RPS];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int m = lane + 64 * (c0 + i);
#pragma unroll
      for (int q = 0; q < PL; ++q) xq[i][q] = X[q * KC + m];
#pragma unroll
      for (int j = 0; j < RPS; ++j) w[i][j] = slot[min(j, nr - 1) * KC + m];
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) {
#pragma unroll
      for (int j = 0; j < RPS; ++j) {
        if (F8) {
          const uint32_t wd[4] = {w[i][j].x, w[i][j].y, w[i][j].z, w[i][j].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x2_t lo = __builtin_amdgcn_cvt_pk_f32_fp8(wd[q], false);
            const f32x2_t hi = __builtin_amdgcn_cvt_pk_f32_fp8(wd[q], true);
            acc[j] = fmaf(lo.x, xq[i][q].x, acc[j]);
            acc[j] = fmaf(lo.y, xq[i][q].y, acc[j]);
            acc[j] = fmaf(hi.x, xq[i][q].z, acc[j]);
            acc[j] = fmaf(hi.y, xq[i][q].w, acc[j]);
          }
        } else {
          acc[j] = dot8(w[i][j], xq[i][0], xq[i][1], acc[j]);
        }
      }
    }
  }
  float out[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < RPS; ++j) out[j] = wave_sum_fast(acc[j]);
  return make_float4(out[0], out[1], out[2], out[3]);
}

// the (rows per slot, chunks per lane) pairs of the engine's shapes: bf16 K 3072 / 8192 and
// fp8 K 3072 / 8192 (Orpheus-3B), bf16 / fp8 K 1024 / 2048 (the small parity shape)
// (inlined: an out-of-line call reads LDS through flat pointers and, by the calling
// convention, waits at entry for every outstanding memory operation of the wave -- the previous
// slot's write-through granule stores -- measured 1.6 us per slot)
template <bool F8>
__device__ __forceinline__ float4 slot_dot(const uint4* slot, const float4* X, int KC, int nr,
                                        int rps, int lane) {
  const int kcl = KC / 64;
#define MX_SD(R_, K_) \
  if (rps == R_ && kcl == K_) return slot_dot_t<F8, R_, K_>(slot, X, KC, nr, lane);
  if constexpr (!F8) {
    MX_SD(2, 6) MX_SD(1, 16) MX_SD(4, 2) MX_SD(4, 4)
  } else {
    MX_SD(4, 3) MX_SD(2, 8) MX_SD(4, 1) MX_SD(4, 2)
  }
#undef MX_SD
  return make_float4(0.f, 0.f, 0.f, 0.f);  // (no other shape passes the host-side check)
}

__device__ __forceinline__ bool witness(const uint2* g, int n, int per, uint32_t tag, int ct,
                                        Ctl* ctl, int& gen, const Clock& clk, int* status,
                                        bool skip) {
  if (skip) return cbar(ctl, gen, clk, status);
  const int nw = (n + per - 1) / per;
  for (int i = ct; i < nw; i += 256) {
    const int wi = min((i + 1) * per, n) - 1;
    int spins = 0;
    while (true) {
      const u32x4v v = gget2(g, wi & ~1);
      if ((wi & 1 ? v.w : v.y) == tag) break;
      __builtin_amdgcn_s_sleep(2);
      if ((spins++ & 63) == 0 && (lds_ld(&ctl->abort_) || clk.expired())) {
        lds_st(&ctl->abort_, 1);
        __hip_atomic_store(status, 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
      }
    }
  }
  return cbar(ctl, gen, clk, status);
}

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

// ---------------------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------------------
// NL loader waves (slot k streamed by loader k mod NL), each keeping a.depth slots in flight
// beyond the one it waits for: one wave's 63-instruction vmcnt window (~63 KB) is below the
// bytes in flight a CU needs at the loaded-chip latency
template <bool F8, int GRP, int NL>
__global__ __launch_bounds__(64 * (NC + NL), 1) void engine_kernel(EngineArgs a) {
  // Separate LDS objects (not one dynamic array): the compiler then knows the ring flags and
  // the staged activations do not alias the LDS-DMA target, and does not drain the loader's
  // in-flight DMA (vmcnt(0)) before every flag write.
  __shared__ __attribute__((aligned(16))) uint8_t ring[RING_MAX * SLOT];
  __shared__ __attribute__((aligned(16))) float Xa[XA_MAX];
  __shared__ __attribute__((aligned(16))) float Xb[XB_MAX];
  __shared__ Ctl ctl_s;
  Ctl* ctl = &ctl_s;
  const int NS = a.ring_slots;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int G = gridDim.x, c = blockIdx.x;
  constexpr int esz = F8 ? 1 : 2;
  constexpr int EPC = F8 ? 16 : 8;
  const int H = a.H, QD = a.heads * 128, KVD = a.kv_heads * 128, F = a.F;
  const int QKVN = QD + 2 * KVD;
  const int L = a.row_pos[0] + 1;  // attention span of this step (new token at L - 1)
  const int slot_id = a.row_slot[0];
  const uint32_t epoch = __hip_atomic_load(a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  Clock clk{__builtin_amdgcn_s_memrealtime() + (uint64_t)a.timeout_ticks};

  // optional timeline (option engine_trace): 12 stamps of the 100 MHz clock per (CU, layer)
  auto stamp = [&](int l, int idx) {
    if (a.trace) a.trace[((size_t)c * a.layers + l) * 12 + idx] = __builtin_amdgcn_s_memrealtime();
  };
  if (tid < 8) {
    ctl->ready[tid] = 0;
    ctl->freed[tid] = 0;
  }
  if (tid == 0) {
    ctl->bar = 0;
    ctl->abort_ = 0;
    ctl->last = 0;
  }
  __syncthreads();

  const Ph ph0 = make_ph(a.wqkv, QKVN, H, esz, G, c, true), ph1 = make_ph(a.wo, H, QD, esz, G, c, false),
           ph2 = make_ph(a.wgu, 2 * F, H, esz, G, c, true), ph3 = make_ph(a.wd, H, F, esz, G, c, false);

  if (wid < NL) {
    // ================================ LOADER ================================
    const int DEPTH = a.depth;
    int k = 0;
    int kq[4], iq[4], qh = 0, qn = 0;  // this loader's issued, unpublished slots (oldest first)
    int spins = 0;
    bool dead = false;
    auto publish_all = [&]() {
      wait_vm<0>();
      for (; qn > 0; --qn, qh = (qh + 1) & 3) loader_st(&ctl->ready[kq[qh] % NS], kq[qh] + 1);
    };
    auto stream_phase = [&](const Ph& P, int l) {
      const uint8_t* Wl = P.W + (size_t)l * P.layer_bytes;
      const size_t lim = P.layer_bytes - 16;
      for (int s = 0; s < P.nslots; ++s, ++k) {
        if (k % NL != wid) continue;
        const int pos = k % NS;
        if (k >= NS && loader_ld(&ctl->freed[pos]) != k - NS + 1) {
          publish_all();
          while (loader_ld(&ctl->freed[pos]) != k - NS + 1) {
            __builtin_amdgcn_s_sleep(2);
            if ((spins++ & 255) == 0 && (loader_ld(&ctl->abort_) || clk.expired())) {
              dead = true;
              return;
            }
          }
        }
        const size_t off0 = (size_t)(P.r0 + s * P.rps) * P.rowbytes + (size_t)lane * 16;
        uint8_t* dst = ring + (size_t)pos * SLOT;
        if (!(a.dbg & 2)) {
          for (int i = 0; i < P.ips; ++i) {
            const size_t off = min(off0 + (size_t)i * 1024, lim);
            __builtin_amdgcn_global_load_lds((gbl_cvoid*)(Wl + off), (lds_void*)(dst + i * 1024), 16, 0, 2);
          }
        }
        const int qt = (qh + qn) & 3;
        kq[qt] = k;
        iq[qt] = P.ips;
        ++qn;
        if (qn > DEPTH) {  // the oldest has landed once only the DEPTH newer are outstanding
          int newer = 0;
          for (int j = 1; j < qn; ++j) newer += iq[(qh + j) & 3];
          wait_vm_n(newer);
          loader_st(&ctl->ready[kq[qh] % NS], kq[qh] + 1);
          qh = (qh + 1) & 3;
          --qn;
        }
      }
    };
    for (int l = 0; l < a.layers && !dead; ++l) {
      if (wid == 0 && lane == 0) stamp(l, 10);
      stream_phase(ph0, l);
      if (!dead) stream_phase(ph1, l);
      if (!dead) stream_phase(ph2, l);
      if (!dead) stream_phase(ph3, l);
      if (wid == 0 && lane == 0) stamp(l, 11);
    }
    publish_all();
    if (dead) lds_st(&ctl->abort_, 1);
  } else {
    // =============================== CONSUMERS ===============================
    const int cw = wid - NL, ct = tid - 64 * NL;
    int gen = 0;
    bool ok = true;
    int k = 0;  // global slot index, same walk as the loader
    const float4* Xa4 = reinterpret_cast<const float4*>(Xa);
    const float4* Xb4 = reinterpret_cast<const float4*>(Xb);
    const int KC_H = H / EPC, KC_Q = QD / EPC, KC_F = F / EPC;
    // attention items: S splits x kv heads, item i on CU i * G / items
    const int S = (L + SL - 1) / SL;
    const int items = S * a.kv_heads;
    const float att_scale = 1.0f / sqrtf(128.0f);
    const bool nodeps = a.dbg & 1;  // timing experiment: stream only, no hand-off waits
    // outputs per producer CU of the o / down projections (h1, h2) and of gate/up (act)
    const int per_h = (H + G - 1) / G;                             // make_ph(.., pair = false)
    const int per_act = ((((2 * F + G - 1) / G) + 1) & ~1) / 2;    // make_ph(.., pair = true) / 2

    // wait for ring slot k; returns its LDS base (nullptr on abort)
    auto take = [&](int kk) -> const uint4* {
      const int pos = kk % NS;
      int spins = 0;
      while (ring_ld(&ctl->ready[pos]) != kk + 1) {
        __builtin_amdgcn_s_sleep(1);
        if ((spins++ & 255) == 0 && (lds_ld(&ctl->abort_) || clk.expired())) {
          lds_st(&ctl->abort_, 1);
          if (lane == 0) __hip_atomic_store(a.status, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          return nullptr;
        }
      }
      return reinterpret_cast<const uint4*>(ring + (size_t)pos * SLOT);
    };
    // (slot_dot's LDS reads have returned: their values are in the reduced sums)
    auto give = [&](int kk) { ring_st(&ctl->freed[kk % NS], kk + 1); };

    for (int l = 0; l < a.layers && ok; ++l) {
      const uint32_t tg = (epoch << 8) | ((uint32_t)l << 3);
      uint16_t* kc = a.kcache + a.kv_layer_elems * l;
      uint16_t* vc = a.vcache + a.kv_layer_elems * l;
      const bool st0 = ct == 0;
      if (st0) stamp(l, 0);
      // ---------------- QKV ----------------
      {
        // this layer's e4m3 row scales and (once) the rope factors of the step's position, to
        // LDS: read in the slot epilogues, visible after the gather's barrier below (the
        // scales are double-buffered by layer parity: a wave may still be in the previous
        // layer's down-projection epilogue)
        if (l == 0) {
          for (int j = ct; 2 * j < ph0.r1 - ph0.r0; j += 256) {
            const int p = ((ph0.r0 + 2 * j) & 127) >> 1;
            ctl->rope[j][0] = a.rope_cos[(size_t)(L - 1) * 64 + p];
            ctl->rope[j][1] = a.rope_sin[(size_t)(L - 1) * 64 + p];
          }
        }
        if (F8) {
          float* sc = ctl->scl[l & 1];
          for (int j = ct; j < 160; j += 256) {
            const float* src = nullptr;
            int r = 0;
            if (j < SC_O) { r = ph0.r0 + j; src = r < ph0.r1 ? a.sqkv + (size_t)l * QKVN + r : nullptr; }
            else if (j < SC_GU) { r = ph1.r0 + j - SC_O; src = r < ph1.r1 ? a.so + (size_t)l * H + r : nullptr; }
            else if (j < SC_D) { r = ph2.r0 + j - SC_GU; src = r < ph2.r1 ? a.sgu + (size_t)l * 2 * F + r : nullptr; }
            else { r = ph3.r0 + j - SC_D; src = r < ph3.r1 ? a.sd + (size_t)l * H + r : nullptr; }
            sc[j] = src ? *src : 0.f;
          }
        }
        float ss = 0.f;
        const float* nw = a.attn_norm + (size_t)l * H;
        if (l == 0) {  // the decode row's hidden state (previous launch: plain loads)
          for (int kk = ct; kk < H; kk += 256) {
            const float x = a.h[kk];
            ss = fmaf(x, x, ss);
            if (kk >= ph1.r0 && kk < ph1.r1) ctl->res1[kk - ph1.r0] = x;
            Xa[((((kk % EPC) >> 2) * KC_H) + kk / EPC) * 4 + (kk & 3)] = x * nw[kk];
          }
        } else {
          ok = witness(a.g_h2, H, per_h, tg - 8 + PH_H2, ct, ctl, gen, clk, a.status, nodeps) &&
               gather<EPC>(a.g_h2, H, tg - 8 + PH_H2, Xa, KC_H, nw, ctl->res1, ph1.r0,
                           ph1.r1 - ph1.r0, ct, ss, ctl, clk, a.status, nodeps);
          if (!ok) break;
        }
        ss = wave_sum(ss);
        if (lane == 0) ctl->ss[cw] = ss;
        if (!(ok = cbar(ctl, gen, clk, a.status))) break;
        if (st0) stamp(l, 1);
        const float scale = 1.0f / sqrtf((ctl->ss[0] + ctl->ss[1] + ctl->ss[2] + ctl->ss[3]) / H + a.eps);
        const Ph& P = ph0;
        const int pos = L - 1;
        for (int s = 0; s < P.nslots; ++s, ++k) {
          if (k % NC != cw) continue;
          const uint4* sl = take(k);
          if (!sl) { ok = false; break; }
          const int n0 = P.r0 + s * P.rps, nr = min(P.rps, P.r1 - n0);
          float acc[4];
          {
            const float4 r4 = slot_dot<F8>(sl, Xa4, KC_H, nr, P.rps, lane);
            acc[0] = r4.x; acc[1] = r4.y; acc[2] = r4.z; acc[3] = r4.w;
          }
          give(k);
          if (lane == 0) {
            for (int j = 0; j + 1 < nr; j += 2) {
              const int n = n0 + j;
              float x1 = acc[j] * scale, x2 = acc[j + 1] * scale;
              if (F8) {
                x1 *= ctl->scl[l & 1][SC_QKV + n - P.r0];
                x2 *= ctl->scl[l & 1][SC_QKV + n + 1 - P.r0];
              }
              const int hh = n >> 7, within = n & 127, p = within >> 1;
              if (hh < a.heads + a.kv_heads) {
                const float cs = ctl->rope[(n - P.r0) >> 1][0], sn = ctl->rope[(n - P.r0) >> 1][1];
                const float o1 = x1 * cs - x2 * sn, o2 = x2 * cs + x1 * sn;
                if (hh < a.heads) {
                  gput(a.g_qkv, hh * 128 + p, o1, tg + PH_QKV);
                  gput(a.g_qkv, hh * 128 + p + 64, o2, tg + PH_QKV);
                } else {
                  const int kh = hh - a.heads;
                  const uint16_t b1 = f32_to_bf16(o1), b2 = f32_to_bf16(o2);
                  uint16_t* kk2 = kc + ((size_t)slot_id * a.kv_heads + kh) * a.max_pos * 128;
                  kk2[kv_k_off(pos, p)] = b1;
                  kk2[kv_k_off(pos, p + 64)] = b2;
                  gput(a.g_qkv, QD + kh * 128 + p, bf16_to_f32(b1), tg + PH_QKV);
                  gput(a.g_qkv, QD + kh * 128 + p + 64, bf16_to_f32(b2), tg + PH_QKV);
                }
              } else {
                const int vh = hh - a.heads - a.kv_heads;
                const uint16_t b1 = f32_to_bf16(x1), b2 = f32_to_bf16(x2);
                uint16_t* vv = vc + ((size_t)slot_id * a.kv_heads + vh) * 128 * a.max_pos;
                vv[kv_v_off(pos, within)] = b1;
                vv[kv_v_off(pos, within + 1)] = b2;
                gput(a.g_qkv, QD + KVD + vh * 128 + within, bf16_to_f32(b1), tg + PH_QKV);
                gput(a.g_qkv, QD + KVD + vh * 128 + within + 1, bf16_to_f32(b2), tg + PH_QKV);
              }
            }
          }
        }
        if (!ok) break;
        if (st0) stamp(l, 2);
      }
      // ---------------- ATTENTION ----------------
      for (int it = 0; it < (nodeps ? 0 : items); ++it) {
        // item it = (kv head, split) runs on CU it * G / items (spread over the grid)
        if (it * G / items != c) continue;
        const int kvh = it % a.kv_heads, sp = it / a.kv_heads;
        const int p0 = sp * SL, p1 = min(p0 + SL, L);  // positions [p0, p1) of this split
        const bool has_new = p1 == L;                  // holds position L - 1 (granules)
        const int Lc = L - 1;                          // cached positions
        // scratch in Xb: q [GRP][128], k/v of the new position, wave partials
        float* qs = Xb;
        float* kn = qs + GRP * 128;
        float* vn = kn + 128;
        float* wacc = vn + 128;                        // [NC + 1][GRP][128]
        float* wml = wacc + (NC + 1) * GRP * 128;      // [NC + 1][GRP][2]
        const size_t head = (size_t)slot_id * a.kv_heads + kvh;
        const uint4* Kf = reinterpret_cast<const uint4*>(kc) + head * a.max_pos * 16;
        const uint4* Vf = reinterpret_cast<const uint4*>(vc) + head * a.max_pos * 16;
        const int base = p0 + 32 * cw;                 // this wave's chunk
        const bool live = base < min(p1, Lc);
        uint4 kf[2][4], vf[8];
        if (live) {  // cached K / V chunk loads go out before the q wait
          const uint4* kcp = Kf + (size_t)(base >> 5) * 512 + lane;
          const uint4* vcp = Vf + (size_t)(base >> 5) * 512 + lane;
#pragma unroll
          for (int T = 0; T < 2; ++T)
#pragma unroll
            for (int st = 0; st < 4; ++st) kf[T][st] = kcp[(T * 4 + st) * 64];
#pragma unroll
          for (int t = 0; t < 8; ++t) vf[t] = vcp[t * 64];
        }
        // gather q (GRP heads) and, for the last split, the new k / v
        {
          float dummy;
          ok = gather<4>(a.g_qkv + (size_t)kvh * GRP * 128, GRP * 128, tg + PH_QKV, qs, GRP * 32,
                         nullptr, nullptr, 0, 0, ct, dummy, ctl, clk, a.status, nodeps);
          // (EPC 4: plane 0 only, i.e. qs[k] in natural order)
          if (ok && has_new) {
            ok = gather<4>(a.g_qkv + QD + kvh * 128, 128, tg + PH_QKV, kn, 32, nullptr, nullptr, 0, 0,
                           ct, dummy, ctl, clk, a.status, nodeps);
            if (ok)
              ok = gather<4>(a.g_qkv + QD + KVD + kvh * 128, 128, tg + PH_QKV, vn, 32, nullptr, nullptr,
                             0, 0, ct, dummy, ctl, clk, a.status, nodeps);
          }
          if (!ok || !(ok = cbar(ctl, gen, clk, a.status))) break;
        }
        const int cc = lane & 15, g = lane >> 4;
        float M = -INFINITY, lsum = 0.f;
        f32x4 acc[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (live) {
          bf16x8 qf[3][4];
          {
            const int hq = cc < GRP ? cc : 0;
#pragma unroll
            for (int st = 0; st < 4; ++st) {
              float x[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) x[j] = cc < GRP ? qs[hq * 128 + 32 * st + 8 * g + j] : 0.f;
              split3(x, qf[0][st], qf[1][st], qf[2][st]);
            }
          }
          f32x4 sc[2];
#pragma unroll
          for (int T = 0; T < 2; ++T) {
            sc[T] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int st = 0; st < 4; ++st) {
              const bf16x8 kb = __builtin_bit_cast(bf16x8, kf[T][st]);
#pragma unroll
              for (int pt = 0; pt < 3; ++pt)
                sc[T] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kb, qf[pt][st], sc[T], 0, 0, 0);
            }
          }
          const int lim = min(p1, Lc);
          float sv[8], mc = -INFINITY;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int p = base + 8 * g + j;
            sv[j] = p < lim ? sc[j >> 2][j & 3] * att_scale : -INFINITY;
            mc = fmaxf(mc, sv[j]);
          }
          mc = fmaxf(mc, __shfl_xor(mc, 16, 64));
          mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
          M = mc;
          float pv[8], ps = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            pv[j] = expf(sv[j] - M);
            ps += pv[j];
          }
          ps += __shfl_xor(ps, 16, 64);
          ps += __shfl_xor(ps, 32, 64);
          lsum = ps;
          bf16x8 pf[3];
          split3(pv, pf[0], pf[1], pf[2]);
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const bf16x8 vb = __builtin_bit_cast(bf16x8, vf[t]);
#pragma unroll
            for (int pt = 0; pt < 3; ++pt)
              acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf[pt], vb, acc[t], 0, 0, 0);
          }
        }
        // wave partial -> LDS (head c's (M, l) in lanes c; O rows: lane (c, g = 0) holds heads i)
        if (g == 0 && cc < GRP) {
          wml[(cw * GRP + cc) * 2] = M;
          wml[(cw * GRP + cc) * 2 + 1] = lsum;
        }
        if (g == 0) {
#pragma unroll
          for (int i = 0; i < GRP; ++i)
#pragma unroll
            for (int t = 0; t < 8; ++t) wacc[(cw * GRP + i) * 128 + 16 * t + cc] = acc[t][i];
        }
        // the new position: one more "wave" partial per head (score, 1, v)
        if (has_new && cw == 0 && lane < GRP) {
          float sdot = 0.f;
          for (int d = 0; d < 128; ++d) sdot = fmaf(qs[lane * 128 + d], kn[d], sdot);
          wml[(NC * GRP + lane) * 2] = sdot * att_scale;
          wml[(NC * GRP + lane) * 2 + 1] = 1.f;
        }
        if (has_new && cw == 1) {
          for (int i = lane; i < GRP * 128; i += 64) wacc[NC * GRP * 128 + i] = vn[i & 127];
        }
        if (!(ok = cbar(ctl, gen, clk, a.status))) break;
        // merge the NC (+1) wave partials: consumer thread ct -> outputs idx = ct, ct + 256, ...
        const int nparts = has_new ? NC + 1 : NC;
        float* part = a.part + (size_t)kvh * a.smax * GRP * 130;
        const bool single = S == 1;
        for (int idx = ct; idx < GRP * 128; idx += 256) {
          const int h = idx >> 7, td = idx & 127;
          float Mb = -INFINITY;
          for (int w = 0; w < nparts; ++w) Mb = fmaxf(Mb, wml[(w * GRP + h) * 2]);
          float num = 0.f, den = 0.f;
          for (int w = 0; w < nparts; ++w) {
            const float mw = wml[(w * GRP + h) * 2];
            const float f = mw == -INFINITY ? 0.f : expf(mw - Mb);
            num = fmaf(f, wacc[(w * GRP + h) * 128 + td], num);
            den = fmaf(f, wml[(w * GRP + h) * 2 + 1], den);
          }
          if (single) {
            gput(a.g_att, (kvh * GRP + h) * 128 + td, num / den, tg + PH_ATT);
          } else {
            float* pp = part + ((size_t)sp * GRP + h) * 130;
            st_wt(pp + td, num);
            if (td == 0) {
              st_wt(pp + 128, Mb);
              st_wt(pp + 129, den);
            }
          }
        }
        if (!single) {
          if (!(ok = cbar(ctl, gen, clk, a.status))) break;  // (cbar waits vmcnt(0): partials landed)
          if (ct == 0) {
            int* tk = a.tickets + l * a.kv_heads + kvh;
            const int t = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = t == S - 1;
            if (last) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lds_st(&ctl->last, last);
          }
          if (!(ok = cbar(ctl, gen, clk, a.status))) break;
          if (lds_ld(&ctl->last)) {  // the last split of this kv head merges all S
            // MC splits' (m, l, acc) loads in flight per round (one round up to L = 1,024),
            // merged online in split order
            constexpr int MC = 8;
            for (int idx = ct; idx < GRP * 128; idx += 256) {
              const int h = idx >> 7, td = idx & 127;
              float Mb = -INFINITY, num = 0.f, den = 0.f;
              for (int s0 = 0; s0 < S; s0 += MC) {
                float mv[MC], lv[MC], av[MC];
#pragma unroll
                for (int j = 0; j < MC; ++j) {
                  const float* pp = part + ((size_t)min(s0 + j, S - 1) * GRP + h) * 130;
                  mv[j] = ld_wt(pp + 128);
                  lv[j] = ld_wt(pp + 129);
                  av[j] = ld_wt(pp + td);
                }
                float mn = Mb;
#pragma unroll
                for (int j = 0; j < MC; ++j)
                  if (s0 + j < S) mn = fmaxf(mn, mv[j]);
                const float r = Mb == -INFINITY ? 0.f : expf(Mb - mn);
                num *= r;
                den *= r;
#pragma unroll
                for (int j = 0; j < MC; ++j) {
                  if (s0 + j < S) {
                    const float f = mv[j] == -INFINITY ? 0.f : expf(mv[j] - mn);
                    num = fmaf(f, av[j], num);
                    den = fmaf(f, lv[j], den);
                  }
                }
                Mb = mn;
              }
              gput(a.g_att, (kvh * GRP + h) * 128 + td, num / den, tg + PH_ATT);
            }
          }
        }
        if (!(ok = cbar(ctl, gen, clk, a.status))) break;  // scratch reused by the next item
      }
      if (!ok) break;
      if (st0) stamp(l, 3);
      // ---------------- O-PROJ ----------------
      {
        float ss;
        ok = witness(a.g_att, QD, GRP * 128, tg + PH_ATT, ct, ctl, gen, clk, a.status, nodeps) &&
             gather<EPC>(a.g_att, QD, tg + PH_ATT, Xb, KC_Q, nullptr, nullptr, 0, 0, ct, ss, ctl,
                         clk, a.status, nodeps);
        if (!ok || !(ok = cbar(ctl, gen, clk, a.status))) break;
        if (st0) stamp(l, 4);
        const Ph& P = ph1;
        for (int s = 0; s < P.nslots; ++s, ++k) {
          if (k % NC != cw) continue;
          const uint4* sl = take(k);
          if (!sl) { ok = false; break; }
          const int n0 = P.r0 + s * P.rps, nr = min(P.rps, P.r1 - n0);
          float acc[4];
          {
            const float4 r4 = slot_dot<F8>(sl, Xb4, KC_Q, nr, P.rps, lane);
            acc[0] = r4.x; acc[1] = r4.y; acc[2] = r4.z; acc[3] = r4.w;
          }
          give(k);
          if (lane < nr) {
            float y = acc[0];
#pragma unroll
            for (int j = 1; j < 4; ++j) y = lane == j ? acc[j] : y;
            const int n = n0 + lane;
            if (F8) y *= ctl->scl[l & 1][SC_O + n - P.r0];
            gput(a.g_h1, n, ctl->res1[n - P.r0] + y, tg + PH_H1);
          }
        }
        if (!ok) break;
        if (st0) stamp(l, 5);
      }
      // ---------------- GATE / UP ----------------
      {
        float ss;
        ok = witness(a.g_h1, H, per_h, tg + PH_H1, ct, ctl, gen, clk, a.status, nodeps) &&
             gather<EPC>(a.g_h1, H, tg + PH_H1, Xa, KC_H, a.mlp_norm + (size_t)l * H, ctl->res2,
                         ph3.r0, ph3.r1 - ph3.r0, ct, ss, ctl, clk, a.status, nodeps);
        if (!ok) break;
        ss = wave_sum(ss);
        if (lane == 0) ctl->ss[cw] = ss;
        if (!(ok = cbar(ctl, gen, clk, a.status))) break;
        if (st0) stamp(l, 6);
        const float scale = 1.0f / sqrtf((ctl->ss[0] + ctl->ss[1] + ctl->ss[2] + ctl->ss[3]) / H + a.eps);
        const Ph& P = ph2;
        for (int s = 0; s < P.nslots; ++s, ++k) {
          if (k % NC != cw) continue;
          const uint4* sl = take(k);
          if (!sl) { ok = false; break; }
          const int n0 = P.r0 + s * P.rps, nr = min(P.rps, P.r1 - n0);
          float acc[4];
          {
            const float4 r4 = slot_dot<F8>(sl, Xa4, KC_H, nr, P.rps, lane);
            acc[0] = r4.x; acc[1] = r4.y; acc[2] = r4.z; acc[3] = r4.w;
          }
          give(k);
          // pair j (rows n0 + 2j, n0 + 2j + 1) -> lane j
          if (2 * lane + 1 < nr) {
            float gt = acc[0] * scale, up = acc[1] * scale;
            if (lane == 1) { gt = acc[2] * scale; up = acc[3] * scale; }
            const int n = n0 + 2 * lane;
            if (F8) {
              gt *= ctl->scl[l & 1][SC_GU + n - P.r0];
              up *= ctl->scl[l & 1][SC_GU + n + 1 - P.r0];
            }
            gput(a.g_act, n >> 1, gt / (1.0f + expf(-gt)) * up, tg + PH_ACT);
          }
        }
        if (!ok) break;
        if (st0) stamp(l, 7);
      }
      // ---------------- DOWN ----------------
      {
        float ss;
        ok = witness(a.g_act, F, per_act, tg + PH_ACT, ct, ctl, gen, clk, a.status, nodeps) &&
             gather<EPC>(a.g_act, F, tg + PH_ACT, Xb, KC_F, nullptr, nullptr, 0, 0, ct, ss, ctl, clk,
                         a.status, nodeps);
        if (!ok || !(ok = cbar(ctl, gen, clk, a.status))) break;
        if (st0) stamp(l, 8);
        const Ph& P = ph3;
        const bool last_layer = l == a.layers - 1;
        for (int s = 0; s < P.nslots; ++s, ++k) {
          if (k % NC != cw) continue;
          const uint4* sl = take(k);
          if (!sl) { ok = false; break; }
          const int n0 = P.r0 + s * P.rps, nr = min(P.rps, P.r1 - n0);
          float acc[4];
          {
            const float4 r4 = slot_dot<F8>(sl, Xb4, KC_F, nr, P.rps, lane);
            acc[0] = r4.x; acc[1] = r4.y; acc[2] = r4.z; acc[3] = r4.w;
          }
          give(k);
          if (lane < nr) {
            float y = acc[0];
#pragma unroll
            for (int j = 1; j < 4; ++j) y = lane == j ? acc[j] : y;
            const int n = n0 + lane;
            if (F8) y *= ctl->scl[l & 1][SC_D + n - P.r0];
            const float v = ctl->res2[n - P.r0] + y;
            if (last_layer) a.h[n] = v;
            else gput(a.g_h2, n, v, tg + PH_H2);
          }
        }
        if (!ok) break;
        if (st0) stamp(l, 9);
      }
    }
    if (!ok) lds_st(&ctl->abort_, 1);
  }
  __syncthreads();
  // the last workgroup to finish advances the epoch (every workgroup read it at entry: none
  // can finish before all have started, since every phase needs every CU's outputs)
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add(a.epoch + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (unsigned)G - 1) {
      __hip_atomic_store(a.epoch + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint32_t e = epoch + 1;
      if ((e & 0xffffffu) == 0) e += 1;  // tag 0 is never a valid epoch (zeroed buffers)
      __hip_atomic_store(a.epoch, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace eng

// Xb holds the o-proj input (heads x 128), the down-proj input (ffn) and the attention scratch
int engine_xb_floats(int heads, int kv_heads, int F) {
  const int grp = heads / kv_heads;
  const int att = grp * 128 + 256 + (eng::NC + 1) * grp * 130;
  return std::max(std::max(F, heads * 128), att);
}
int engine_ring_max() { return eng::RING_MAX; }
// the engine's LDS is static (eng::RING_MAX slots, XA_MAX / XB_MAX floats): shapes must fit it
size_t engine_lds_bytes(int ring_slots, int H, int xb_floats) {
  if (ring_slots > eng::RING_MAX || H > eng::XA_MAX || xb_floats > eng::XB_MAX) return ~(size_t)0;
  return (size_t)eng::RING_MAX * eng::SLOT + (size_t)(eng::XA_MAX + eng::XB_MAX) * 4 + sizeof(eng::Ctl);
}

// Workgroups of the engine one CU holds at once (it needs exactly one per CU, all co-resident)
static const void* engine_fn(const EngineArgs& a) {
  const int grp = a.heads / a.kv_heads;
  const void* fn = nullptr;
#define MX_ENGF(F8_, G_, L_)                                                  \
  if (a.f8 == F8_ && grp == G_ && a.loaders == L_)                            \
    fn = reinterpret_cast<const void*>(&eng::engine_kernel<F8_, G_, L_>);
  MX_ENGF(false, 3, 1) MX_ENGF(true, 3, 1) MX_ENGF(false, 4, 1) MX_ENGF(true, 4, 1)
  MX_ENGF(false, 3, 2) MX_ENGF(true, 3, 2) MX_ENGF(false, 4, 2) MX_ENGF(true, 4, 2)
#undef MX_ENGF
  return fn;
}

hipError_t engine_per_cu(const EngineArgs& a, int* per_cu) {
  const size_t lds = engine_lds_bytes(a.ring_slots, a.H, a.xb);
  const void* fn = engine_fn(a);
  if (!fn) return hipErrorNotSupported;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, fn, 64 * (eng::NC + a.loaders), 0);
}

hipError_t launch_engine_b1(const EngineArgs& a, int grid, hipStream_t st) {
  const size_t lds = engine_lds_bytes(a.ring_slots, a.H, a.xb);
  if (a.ring_slots < 3 || a.ring_slots > eng::RING_MAX || a.ring_slots <= a.depth ||
      lds > 160 * 1024 || a.layers > 31)
    return hipErrorInvalidValue;
  // Xb must hold the attention scratch: before 5129db2 it was sized by the ffn width alone, and
  // on the small test shape (GQA 4, ffn 2,048 < 3,368 scratch floats) the attention items wrote
  // past it into the control block (ring flags, barrier count), so a CU stopped publishing and
  // its consumers' gathers timed out (status 3, gpurun_out/r05_eng1/tests.log).  Assert it here.
  if (a.xb < engine_xb_floats(a.heads, a.kv_heads, a.F) || a.xb > eng::XB_MAX) return hipErrorInvalidValue;
  if (a.H % 1024 || a.F % 1024 || a.heads * 128 != a.H) return hipErrorNotSupported;
  const void* fn = engine_fn(a);
  if (!fn) return hipErrorNotSupported;
  void* args[] = {const_cast<EngineArgs*>(&a)};
  return hipLaunchKernel(fn, dim3(grid), dim3(64 * (eng::NC + a.loaders)), args, 0, st);
}

}  // namespace mx
