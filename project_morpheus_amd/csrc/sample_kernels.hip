// Temperature + top-p sampling of the next token (BASELINE P2).
//
// Replaces the sampler behind vLLM SamplingParams(temperature, top_p, repetition_penalty)
// (Orpheus-TTS/orpheus_tts_pypi/orpheus_tts/engine_class.py:106-112) and the llama.cpp
// sampler the reference drives with the same three knobs (Morpheus_Client/tts_engine/
// inference.py:75-105, llama_local.py:77).  Greedy decoding stays the parity mode: rows whose
// KV slot has temperature <= 0 keep the argmax key of the lm_head epilogue and this kernel
// returns at once.
//
// Definition (restated by oracle/sampling_ref.py, which the GPU tests compare against):
//   l_i   penalised logits (the lm_head epilogue keeps them for sampling rows)
//   e_i   = exp((l_i - max l) / T)                        in (0, 1]
//   f_i   = floor(e_i * 2^40)                             integer mass (uint64, exact sums)
//   Z     = sum f_i;   thr = max(1, floor(top_p * Z)) in float64 (top_p >= 1: thr = Z)
//   keep i  iff  sum_{j : e_j > e_i} f_j < thr            (nucleus; ties kept together)
//   u_i   = ((philox(seed, (i, pos)).x >> 9) + 0.5) * 2^-23,   q_i = -log(u_i)
//           (23 bits: u + 0.5 is exact in fp32, so u is strictly inside (0, 1))
//   token = argmax_{kept i} e_i / q_i  (smallest index on ties)   -- the exponential race,
//           an exact draw from the renormalised kept distribution.
// Integer masses make the nucleus cut order-independent (deterministic under atomics); the
// cut is found by a 3-pass radix select over the bit pattern of e_i (12 + 12 + 8 bits) with
// per-bin masses in LDS, one 1024-thread block per row.
#include "mx_common.h"
#include "mx_llm_kernels.h"

namespace mx {

// Philox4x32-10 (Salmon et al., SC'11): word 0 of the block for counter (c0, c1, 0, 0).
__device__ __forceinline__ uint32_t philox_x0(uint32_t c0, uint32_t c1, uint32_t k0,
                                              uint32_t k1) {
  uint32_t x0 = c0, x1 = c1, x2 = 0u, x3 = 0u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, x0), lo0 = 0xD2511F53u * x0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, x2), lo1 = 0xCD9E8D57u * x2;
    x0 = hi1 ^ x1 ^ k0;
    x1 = lo1;
    x2 = hi0 ^ x3 ^ k1;
    x3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return x0;
}

constexpr int SMP_T = 1024;  // threads per row block
constexpr float SMP_FX = 1099511627776.0f;  // 2^40

__device__ __forceinline__ unsigned long long u64_wave_sum(unsigned long long v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, MX_WAVE);
  return v;
}

// Bins [0, 1024*PER) of `hist` hold integer masses; `base` is the mass of everything above
// bin NB-1.  Finds the unique bin b with C_b < thr <= C_b + hist[b], where C_b = base + mass
// of bins above b, and publishes (b, C_b) to *cut_bin / *cut_base.
template <int PER>
__device__ void find_cut(const unsigned long long* hist, unsigned long long base,
                         unsigned long long thr, int* cut_bin, unsigned long long* cut_base,
                         unsigned long long* wsum) {
  constexpr int NB = SMP_T * PER;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) {  // (always overwritten: thr <= base + the mass of these bins)
    *cut_bin = 0;
    *cut_base = base;
  }
  unsigned long long v[PER], tot = 0ull;
#pragma unroll
  for (int k = 0; k < PER; ++k) {  // thread t owns bins NB-1-t*PER .. NB-PER-t*PER (descending)
    v[k] = hist[NB - 1 - (t * PER + k)];
    tot += v[k];
  }
  unsigned long long inc = tot;  // inclusive scan over the descending order
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long o = __shfl_up(inc, d, MX_WAVE);
    if (lane >= d) inc += o;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  unsigned long long c = base + inc - tot;
  for (int i = 0; i < w; ++i) c += wsum[i];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (c < thr && c + v[k] >= thr) {
      *cut_bin = NB - 1 - (t * PER + k);
      *cut_base = c;
    }
    c += v[k];
  }
  __syncthreads();
}

__global__ __launch_bounds__(SMP_T) void sample_kernel(SampleArgs a) {
  const int r = blockIdx.x;
  const int slot = a.row_slot[r];
  const float T = a.temp[slot];
  if (!(T > 0.f)) return;  // greedy row: the epilogue's argmax key stands
  const float top_p = a.top_p[slot];
  const uint32_t k0 = a.seed[2 * slot], k1 = a.seed[2 * slot + 1];
  const uint32_t ctr1 = (uint32_t)a.row_pos[r];
  const float* lg = a.logits + (size_t)r * a.V;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int V = a.V;

  __shared__ unsigned long long hist[4096];
  __shared__ unsigned long long wsum[SMP_T / 64];
  __shared__ float fred[SMP_T / 64];
  __shared__ int cut_bin;
  __shared__ unsigned long long cut_base;

  // pass 1: max logit
  float m = -INFINITY;
  for (int i = t; i < V; i += SMP_T) m = fmaxf(m, lg[i]);
  m = wave_max(m);
  if (lane == 0) fred[w] = m;
  for (int i = t; i < 4096; i += SMP_T) hist[i] = 0ull;
  __syncthreads();
  m = fred[0];
  for (int i = 1; i < SMP_T / 64; ++i) m = fmaxf(m, fred[i]);
  auto e_of = [&](int i) { return expf((lg[i] - m) / T); };
  auto f_of = [&](float e) { return (unsigned long long)(e * SMP_FX); };

  // pass 2: total integer mass Z and the first radix histogram (bits 31..20 of e)
  unsigned long long z = 0ull;
  for (int i = t; i < V; i += SMP_T) {
    const float e = e_of(i);
    const unsigned long long f = f_of(e);
    z += f;
    if (f) atomicAdd(&hist[__float_as_uint(e) >> 20], f);
  }
  z = u64_wave_sum(z);
  if (lane == 0) wsum[w] = z;
  __syncthreads();
  unsigned long long Z = 0ull;
  for (int i = 0; i < SMP_T / 64; ++i) Z += wsum[i];
  unsigned long long thr = Z;
  if (top_p < 1.f) {
    thr = (unsigned long long)((double)Z * (double)top_p);
    if (thr < 1ull) thr = 1ull;
  }
  __syncthreads();  // every thread has read wsum
  find_cut<1>(hist, 0ull, thr, &cut_bin, &cut_base, wsum);
  const uint32_t b1 = (uint32_t)cut_bin;
  const unsigned long long c1 = cut_base;

  // pass 3: bits 19..8 inside bin b1
  for (int i = t; i < 4096; i += SMP_T) hist[i] = 0ull;
  __syncthreads();
  for (int i = t; i < V; i += SMP_T) {
    const float e = e_of(i);
    const uint32_t bits = __float_as_uint(e);
    if ((bits >> 20) == b1) {
      const unsigned long long f = f_of(e);
      if (f) atomicAdd(&hist[(bits >> 8) & 0xFFFu], f);
    }
  }
  __syncthreads();
  find_cut<4>(hist, c1, thr, &cut_bin, &cut_base, wsum);
  const uint32_t b12 = (b1 << 12) | (uint32_t)cut_bin;
  const unsigned long long c2 = cut_base;

  // pass 4: bits 7..0 inside (b1, b2)
  for (int i = t; i < 4096; i += SMP_T) hist[i] = 0ull;
  __syncthreads();
  for (int i = t; i < V; i += SMP_T) {
    const float e = e_of(i);
    const uint32_t bits = __float_as_uint(e);
    if ((bits >> 8) == b12) {
      const unsigned long long f = f_of(e);
      if (f) atomicAdd(&hist[bits & 0xFFu], f);
    }
  }
  __syncthreads();
  find_cut<1>(hist, c2, thr, &cut_bin, &cut_base, wsum);
  const uint32_t tcut = (b12 << 8) | (uint32_t)cut_bin;

  // pass 5: exponential race over the kept tokens
  unsigned long long best = 0ull;
  for (int i = t; i < V; i += SMP_T) {
    const float e = e_of(i);
    if (__float_as_uint(e) >= tcut) {
      const uint32_t x = philox_x0((uint32_t)i, ctr1, k0, k1);
      const float u = ((float)(x >> 9) + 0.5f) * 1.1920928955078125e-07f;  // 2^-23, u < 1 exactly
      const float s = e / -logf(u);
      const unsigned long long key = argmax_key(s, (uint32_t)i);
      best = key > best ? key : best;
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const unsigned long long o = __shfl_xor(best, d, MX_WAVE);
    best = o > best ? o : best;
  }
  if (lane == 0) wsum[w] = best;
  __syncthreads();
  if (t == 0) {
    unsigned long long k = wsum[0];
    for (int i = 1; i < SMP_T / 64; ++i) k = wsum[i] > k ? wsum[i] : k;
    a.best[r] = k;
  }
}

__global__ void set_slot_params_kernel(float* penalty, float* temp, float* top_p,
                                       uint32_t* seed, int slot, float pen, float t, float p,
                                       uint32_t s0, uint32_t s1) {
  penalty[slot] = pen;
  temp[slot] = t;
  top_p[slot] = p;
  seed[2 * slot] = s0;
  seed[2 * slot + 1] = s1;
}

hipError_t launch_sample(const SampleArgs& a, int R, hipStream_t st) {
  hipLaunchKernelGGL(sample_kernel, dim3(R), dim3(SMP_T), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_set_slot_params(float* penalty, float* temp, float* top_p, uint32_t* seed,
                                  int slot, float pen, float t, float p, uint64_t s,
                                  hipStream_t st) {
  hipLaunchKernelGGL(set_slot_params_kernel, dim3(1), dim3(1), 0, st, penalty, temp, top_p,
                     seed, slot, pen, t, p, (uint32_t)s, (uint32_t)(s >> 32));
  return hipGetLastError();
}

}  // namespace mx
