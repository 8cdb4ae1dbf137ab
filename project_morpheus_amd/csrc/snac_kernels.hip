// SNAC 24 kHz codec decoder on MI355X (gfx950), fp32 arithmetic.
//
// Replaces snac.SNAC.decode (third-party snac 1.2.x; call site
// Morpheus_Client/tts_engine/speechpipe.py:118) plus the slice / PCM16 epilogue
// (speechpipe.py:122-129).  Every dense contraction (1x1 convs, NoiseBlock linear,
// polyphase ConvTranspose1d) runs as one "segmented conv-GEMM" on the bf16 MFMA with both
// fp32 operands split into three bf16 parts (fp32-accurate products), the Snake activation
// of the next consumer and bias / residual / noise fused into the epilogue.  Depthwise
// dilated k7 convs stage a haloed, Snake-activated tile in LDS.
#include "mx_common.h"
#include "mx_snac_kernels.h"
#include "mx_rows_common.h"

namespace mx {


__device__ __forceinline__ float snake(float x, float a) {
  // layers.py snake(): x + (alpha + 1e-9).reciprocal() * sin(alpha * x)^2.  The sine is the
  // hardware v_sin_f32 (8 cycles) on the fp32 argument reduced to [0, 1) revolutions: the
  // library sinf (~30 instructions) made the Snake stages VALU-bound.  CPU emulation of this
  // reduction: audio RMS 6e-7 vs torch.sin (scripts/snac_fastsin_emulation.py).
  const float rev = (a * x) * 0.15915494309189535f;
  const float s = __builtin_amdgcn_sinf(rev - floorf(rev));
  return x + (1.0f / (a + 1e-9f)) * (s * s);
}

// ---------------------------------------------------------------------------------
// RVQ from_codes (vq.py): z[c][t] = sum_i out_proj_i(codebook_i[code_i[t / stride_i]])
// frames: [B][7N] codes in speechpipe order; de-interleave per speechpipe.py:84-98.
// z is channels-last [B][4N][768].  Grid (4N, B), block 256.
// ---------------------------------------------------------------------------------
struct EmbedPtrs {
  const float* cb[3];
  const float* w[3];
  const float* b[3];
};

__global__ __launch_bounds__(256) void snac_embed_kernel(const int32_t* frames, int n_frames,
                                                         EmbedPtrs p, float* z,
                                                         const SnacIO* io) {
  if (io) frames = io->frames;
  const int t = blockIdx.x, bt = blockIdx.y;
  const int T = 4 * n_frames;
  const int32_t* fr = frames + (size_t)bt * 7 * n_frames;
  __shared__ float e[3][8];
  if (threadIdx.x < 3) {
    const int i = threadIdx.x;
    int code;
    if (i == 0) {
      code = fr[7 * (t >> 2)];
    } else if (i == 1) {
      const int j = t >> 1;  // index into c1 [2N]: {t1, t4} per frame
      code = fr[7 * (j >> 1) + ((j & 1) ? 4 : 1)];
    } else {
      const int f = t >> 2, q = t & 3;  // c2 [4N]: {t2, t3, t5, t6}
      const int off[4] = {2, 3, 5, 6};
      code = fr[7 * f + off[q]];
    }
    code = code < 0 ? 0 : (code > 4095 ? 4095 : code);  // host rejects 4096 / negatives
#pragma unroll
    for (int k = 0; k < 8; ++k) e[i][k] = p.cb[i][code * 8 + k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 768; c += 256) {
    float zc = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      float v = p.b[i][c];
#pragma unroll
      for (int k = 0; k < 8; ++k) v = fmaf(p.w[i][c * 8 + k], e[i][k], v);
      zc += v;
    }
    z[((size_t)bt * T + t) * 768 + c] = zc;
  }
}

// ---------------------------------------------------------------------------------
// Depthwise k7 dilated conv, "same" padding 3*dil, optional Snake on input and output, on
// channels-last activations [B][T][C] (every SNAC activation is channels-last, so a conv-GEMM
// B fragment -- 8 consecutive channels at one time step -- is two 16-byte loads).
// Block = 64 channels x 16 time rows, 4 channels (one 16-byte piece) per lane, so a wave's
// load or store instruction moves 4 rows x 256 B = 1 KB (with one channel per lane it moved
// 256 B: dwconv_kernel<64> ran at 4.1 TB/s on the 32-window shapes).  The TT-step output tile
// reads a haloed Snake(x) tile staged once in LDS (Snake evaluated once per input).  Grid
// (ceil(T/TT), C/64, B): TT = 64 for the batched shapes, 16 for single windows.
// ---------------------------------------------------------------------------------
template <int TT>
__global__ __launch_bounds__(256) void dwconv_kernel(const float* x, float* y, const float* w,
                                                     const float* b, const float* ain,
                                                     const float* aout, int C, int T, int dil) {
  const int cq = threadIdx.x & 15, tr = threadIdx.x >> 4;  // channel quad, row group (16)
  const int c = blockIdx.y * 64 + 4 * cq, t0 = blockIdx.x * TT, bt = blockIdx.z;
  const int halo = 3 * dil;
  __shared__ float4 tile[TT + 54][16];
  const float* xb = x + (size_t)bt * T * C + c;
  const float4 a_in = ain ? *reinterpret_cast<const float4*>(ain + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  // every global load of the haloed tile is issued before any is consumed (a runtime-count
  // loop of load -> Snake -> LDS store paid one memory latency per row)
  constexpr int NI = (TT + 54 + 15) / 16;
  const int rows = TT + 2 * halo;
  float4 v[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int i = tr + 16 * j, t = t0 - halo + i;
    v[j] = (i < rows && t >= 0 && t < T) ? *reinterpret_cast<const float4*>(xb + (size_t)t * C)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int i = tr + 16 * j;
    if (i < rows) {
      float4 u = v[j];
      if (ain) {
        u.x = snake(u.x, a_in.x); u.y = snake(u.y, a_in.y);
        u.z = snake(u.z, a_in.z); u.w = snake(u.w, a_in.w);
      }
      tile[i][cq] = u;
    }
  }
  __syncthreads();
  float wk[7][4];
#pragma unroll
  for (int k = 0; k < 7; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) wk[k][e] = w[(c + e) * 7 + k];
  const float4 bias = *reinterpret_cast<const float4*>(b + c);
  const float4 a_out = aout ? *reinterpret_cast<const float4*>(aout + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  float* yb = y + (size_t)bt * T * C + c;
  for (int i = tr; i < TT; i += 16) {
    const int t = t0 + i;
    if (t >= T) break;
    float4 acc = bias;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const float4 u = tile[i + k * dil][cq];
      acc.x = fmaf(wk[k][0], u.x, acc.x);
      acc.y = fmaf(wk[k][1], u.y, acc.y);
      acc.z = fmaf(wk[k][2], u.z, acc.z);
      acc.w = fmaf(wk[k][3], u.w, acc.w);
    }
    if (aout) {
      acc.x = snake(acc.x, a_out.x); acc.y = snake(acc.y, a_out.y);
      acc.z = snake(acc.z, a_out.z); acc.w = snake(acc.w, a_out.w);
    }
    *reinterpret_cast<float4*>(yb + (size_t)t * C) = acc;
  }
}

// ---------------------------------------------------------------------------------
// Segmented conv-GEMM on the bf16 MFMA (v_mfma_f32_16x16x32_bf16) with fp32 operands split
// into three bf16 parts each (x = x0 + x1 + x2, w = w0 + w1 + w2, exact to fp32 rounding).
// The six products whose part indices sum to <= 2 are kept; the dropped ones are below
// 2^-24 relative, i.e. fp32 rounding.  Six 16x16x32 MFMAs (96 cycles) replace
// eight 16x16x4 f32 MFMAs (256 cycles) per 32-deep k step of a 16x16 tile.
//   out[b][col_stride*n + ph][m] = epi( sum_seg sum_ci A_ph[m][seg*Cin+ci] X[b][n+d_ph,seg][ci] )
// Weights are pre-split at finalize into three bf16 planes [3][M][nseg*Cin]; a lane's A
// fragment (row c, k = 8g..8g+7) is one 16-byte load per plane.  The B fragment (column n,
// the same 8 k) is two 16-byte loads from channels-last X [t][ci], split in registers.
// One block = one 32 x (16*NSUB) output tile of one (phase, window); its WK waves split K
// and their partial tiles are summed in LDS in a fixed order (deterministic, no atomics).
// Grid (ceil(Tin / (16*NSUB)), M / 32, nphase * B).
// ---------------------------------------------------------------------------------
using rows::bf16x8;
using rows::f32x4;

template <int NSUB>
__device__ __forceinline__ void conv_gemm_tile(const ConvGemmArgs& a, int k_begin, int k_end,
                                               int n0, int m0, int ph, int bt, int lane,
                                               f32x4 (&acc)[2][NSUB]) {
  const int c = lane & 15, g = lane >> 4;
  const uint16_t* A = a.Abf[ph];
  const int d0 = a.dph[ph][0], d1 = a.dph[ph][1];
  const int Ktot = a.nseg * a.Cin;
  const size_t plane = (size_t)a.M * Ktot;
  const float* X = a.X + (size_t)bt * a.Cin * a.Tin;  // [Tin][Cin]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NSUB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int tn[NSUB];
  bool nok[NSUB];
#pragma unroll
  for (int j = 0; j < NSUB; ++j) {
    tn[j] = n0 + 16 * j + c;
    nok[j] = tn[j] < a.Tin;
  }
  const uint16_t* Ar0 = A + (size_t)(m0 + c) * Ktot + 8 * g;
  const uint16_t* Ar1 = A + (size_t)(m0 + 16 + c) * Ktot + 8 * g;
  // two-stage pipeline: the next 32-deep step's A planes and X pieces are in flight while
  // this step splits X and runs its MFMAs (k ranges are multiples of 64: launch_conv_gemm)
  uint4 ab[2][2][3];
  float4 xb[2][NSUB][2];
  auto load = [&](int kc, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      ab[buf][0][p] = *reinterpret_cast<const uint4*>(Ar0 + p * plane + kc);
      ab[buf][1][p] = *reinterpret_cast<const uint4*>(Ar1 + p * plane + kc);
    }
    const int seg = kc >= a.Cin ? 1 : 0;  // a 32-chunk never straddles segments (Cin % 32 == 0)
    const int ci0 = kc + 8 * g - seg * a.Cin;
    const int d = seg ? d1 : d0;
#pragma unroll
    for (int j = 0; j < NSUB; ++j) {
      const int tc = min(max(tn[j] + d, 0), a.Tin - 1);
      const float4* xp = reinterpret_cast<const float4*>(X + (size_t)tc * a.Cin + ci0);
      xb[buf][j][0] = xp[0];
      xb[buf][j][1] = xp[1];
    }
  };
  auto step = [&](int kc, int buf) __attribute__((always_inline)) {
    const int d = kc >= a.Cin ? d1 : d0;
    bf16x8 xf[NSUB][3];
#pragma unroll
    for (int j = 0; j < NSUB; ++j) {
      const int t = tn[j] + d;
      const bool ok = nok[j] && t >= 0 && t < a.Tin;
      const float4 lo = xb[buf][j][0], hi = xb[buf][j][1];
      float x[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      if (!ok) {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = 0.f;
      }
      rows::split_parts<3>(x, xf[j]);
    }
    // six products, smallest first; 2 x NSUB independent accumulator chains per product
    constexpr int PA[6] = {1, 0, 2, 0, 1, 0}, PB[6] = {1, 2, 0, 1, 0, 0};
#pragma unroll
    for (int q = 0; q < 6; ++q)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NSUB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, ab[buf][i][PA[q]]), xf[j][PB[q]], acc[i][j], 0, 0, 0);
  };
  load(k_begin, 0);
  for (int kc = k_begin; kc < k_end; kc += 64) {
    load(kc + 32, 1);
    step(kc, 0);
    if (kc + 64 < k_end) load(kc + 64, 0);
    step(kc + 32, 1);
  }
}

__device__ __forceinline__ void conv_gemm_store(const ConvGemmArgs& a, float v, int m, int n,
                                                int ph, int bt) {
  const int col = a.col_stride * n + ph;
  if (a.bias) v += a.bias[m];
  const size_t o = ((size_t)bt * a.Tout + col) * a.M + m;
  if (a.epi == CG_RESID) v = a.R[o] + v;
  else if (a.epi == CG_NOISE) v = a.R[o] + a.noise[(size_t)bt * a.noise_stride + col] * v;
  a.out[o] = v;
  if (a.out2) a.out2[o] = snake(v, a.alpha2[m]);
}

// 4 consecutive channels m .. m+3 of one column: 16-byte accesses in the channels-last layout
__device__ __forceinline__ void conv_gemm_store4(const ConvGemmArgs& a, f32x4 v, int m, int n,
                                                 int ph, int bt) {
  const int col = a.col_stride * n + ph;
  if (a.bias) v += *reinterpret_cast<const f32x4*>(a.bias + m);
  const size_t o = ((size_t)bt * a.Tout + col) * a.M + m;
  if (a.epi == CG_RESID) {
    v += *reinterpret_cast<const f32x4*>(a.R + o);
  } else if (a.epi == CG_NOISE) {
    const float nz = a.noise[(size_t)bt * a.noise_stride + col];
    v = *reinterpret_cast<const f32x4*>(a.R + o) + nz * v;
  }
  *reinterpret_cast<f32x4*>(a.out + o) = v;
  if (a.out2) {
    f32x4 s2;
#pragma unroll
    for (int r = 0; r < 4; ++r) s2[r] = snake(v[r], a.alpha2[m + r]);
    *reinterpret_cast<f32x4*>(a.out2 + o) = s2;
  }
}

// Epilogue operands gathered before any output is stored.  In the residual units R and out
// are the same buffer, so the compiler may not move a later element's R (or bias / noise /
// alpha) load above an earlier element's store: every element of the epilogue paid its own
// dependent memory round trip.  Loading them all first keeps each element's read-before-write
// (the elements of a thread are distinct) and the arithmetic of conv_gemm_store(4).
struct CgOps4 {
  f32x4 bias, r, a2;
  float nz;
};
__device__ __forceinline__ CgOps4 conv_gemm_ops4(const ConvGemmArgs& a, int m, int n, int ph,
                                                 int bt) {
  CgOps4 p;
  p.bias = a.bias ? *reinterpret_cast<const f32x4*>(a.bias + m) : f32x4{0.f, 0.f, 0.f, 0.f};
  const int col = a.col_stride * n + ph;
  const size_t o = ((size_t)bt * a.Tout + col) * a.M + m;
  p.r = (a.epi == CG_RESID || a.epi == CG_NOISE) ? *reinterpret_cast<const f32x4*>(a.R + o)
                                                   : f32x4{0.f, 0.f, 0.f, 0.f};
  p.nz = a.epi == CG_NOISE ? a.noise[(size_t)bt * a.noise_stride + col] : 0.f;
  p.a2 = a.out2 ? *reinterpret_cast<const f32x4*>(a.alpha2 + m) : f32x4{0.f, 0.f, 0.f, 0.f};
  return p;
}
__device__ __forceinline__ void conv_gemm_store4p(const ConvGemmArgs& a, f32x4 v, int m, int n,
                                                  int ph, int bt, const CgOps4& p) {
  const int col = a.col_stride * n + ph;
  if (a.bias) v += p.bias;
  const size_t o = ((size_t)bt * a.Tout + col) * a.M + m;
  if (a.epi == CG_RESID) v += p.r;
  else if (a.epi == CG_NOISE) v = p.r + p.nz * v;
  *reinterpret_cast<f32x4*>(a.out + o) = v;
  if (a.out2) {
    f32x4 s2;
#pragma unroll
    for (int r = 0; r < 4; ++r) s2[r] = snake(v[r], p.a2[r]);
    *reinterpret_cast<f32x4*>(a.out2 + o) = s2;
  }
}

template <int WK, int NSUB>
__global__ __launch_bounds__(WK * 64) void conv_gemm_kernel(ConvGemmArgs a) {
  constexpr int BM = 32, BN = 16 * NSUB;
  const int lane = threadIdx.x & 63, wk = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int ph = blockIdx.z / a.B, bt = blockIdx.z - ph * a.B;
  const int Kw = a.nseg * a.Cin / WK;
  f32x4 acc[2][NSUB];
  conv_gemm_tile<NSUB>(a, wk * Kw, (wk + 1) * Kw, n0, m0, ph, bt, lane, acc);
  // deterministic cross-wave K reduction through LDS: tile [BM][BN] per wave
  __shared__ float red[WK][BM * BN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NSUB; ++j)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) red[wk][(16 * i + 4 * g + rg) * BN + 16 * j + c] = acc[i][j][rg];
  __syncthreads();
  // element e = tid + WK 64 it: consecutive threads take consecutive channels; operands of
  // every element first, then the stores (see conv_gemm_ops4)
  constexpr int IT = BM * BN / (WK * 64);
  static_assert(IT * WK * 64 == BM * BN, "epilogue tiling");
  float ob[IT], orr[IT], onz[IT], oa2[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int e = threadIdx.x + WK * 64 * it;
    const int nn = e / BM, mm = e - nn * BM, m = m0 + mm;
    const int n = min(n0 + nn, a.Tin - 1);
    const int col = a.col_stride * n + ph;
    const size_t o = ((size_t)bt * a.Tout + col) * a.M + m;
    ob[it] = a.bias ? a.bias[m] : 0.f;
    orr[it] = (a.epi == CG_RESID || a.epi == CG_NOISE) ? a.R[o] : 0.f;
    onz[it] = a.epi == CG_NOISE ? a.noise[(size_t)bt * a.noise_stride + col] : 0.f;
    oa2[it] = a.out2 ? a.alpha2[m] : 0.f;
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int e = threadIdx.x + WK * 64 * it;
    const int nn = e / BM, mm = e - nn * BM;
    const int n = n0 + nn;
    if (n >= a.Tin) continue;
    const int ei = mm * BN + nn;
    float v = red[0][ei];
#pragma unroll
    for (int w = 1; w < WK; ++w) v += red[w][ei];
    // conv_gemm_store with the gathered operands
    const int col = a.col_stride * n + ph;
    if (a.bias) v += ob[it];
    const size_t o = ((size_t)bt * a.Tout + col) * a.M + m0 + mm;
    if (a.epi == CG_RESID) v = orr[it] + v;
    else if (a.epi == CG_NOISE) v = orr[it] + onz[it] * v;
    a.out[o] = v;
    if (a.out2) a.out2[o] = snake(v, oa2[it]);
  }
}

// WK == 1: one wave per tile, the epilogue straight from registers.
template <int NSUB>
__global__ __launch_bounds__(64) void conv_gemm1_kernel(ConvGemmArgs a) {
  constexpr int BM = 32, BN = 16 * NSUB;
  const int lane = threadIdx.x & 63;
  const int c = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int ph = blockIdx.z / a.B, bt = blockIdx.z - ph * a.B;
  f32x4 acc[2][NSUB];
  conv_gemm_tile<NSUB>(a, 0, a.nseg * a.Cin, n0, m0, ph, bt, lane, acc);
  CgOps4 ops[2][NSUB];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NSUB; ++j)
      ops[i][j] = conv_gemm_ops4(a, m0 + 16 * i + 4 * g, min(n0 + 16 * j + c, a.Tin - 1), ph, bt);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NSUB; ++j) {
      const int n = n0 + 16 * j + c;
      if (n >= a.Tin) continue;
      conv_gemm_store4p(a, acc[i][j], m0 + 16 * i + 4 * g, n, ph, bt, ops[i][j]);
    }
}

// ---------------------------------------------------------------------------------
// Block-tiled conv-GEMM for batched windows (the serving shapes): the B windows' columns are
// concatenated (column = window * Tin + t), and a 256-thread block computes a (64 BMT) x 128
// tile: BMT = 1 over 2 x 2 waves (32 x 64 each), BMT = 2 over 4 x 1 waves (32 x 128 each:
// the staged X tile feeds twice the MFMAs).  Per 32-deep k step the block stages A (64 BMT
// rows x 3 bf16 planes) and X (128 columns x 32 channels, split into 3 bf16 parts) ONCE in
// LDS in MFMA fragment order, so every operand byte fetched from L2 feeds 4-16x more MFMAs
// than the one-wave kernels above (whose A / X re-fetches made them vector-memory bound:
// 50-70 TF/s).  The next step's global loads are in flight (registers) while this step's
// MFMAs run.  Grid (M / (64 BMT) * nphase, ceil(B*Tin / 128)): (M tile, phase) fastest, so
// the blocks reading one X column tile are dispatched together and share it through L2.
// ---------------------------------------------------------------------------------
template <int BMT>
__global__ __launch_bounds__(256) void conv_gemm_tiled_kernel(ConvGemmArgs a) {
  constexpr int WMN = 2 * BMT, NJ = 2 * WMN;  // waves along M (of 4); n-tiles per wave (of 8)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int wm = w % WMN, wn = w / WMN;
  // XCD-aware tile order: the dispatcher deals consecutive block ids round-robin over the 8
  // XCDs, each with its own L2, so the gridDim.x blocks of one X column tile would land on
  // different XCDs and each fetch the tile from HBM.  Logical id = XCD-major over the first
  // 8 * (nb / 8) ids (a bijection; the tail keeps its id): one XCD runs consecutive logical
  // ids, i.e. all (M tile, phase) blocks of a column tile, and the tile is read once.
  const int nb = gridDim.x * gridDim.y;
  int bid = blockIdx.x + blockIdx.y * gridDim.x;
  const int per = nb >> 3;
  if (bid < per * 8) bid = (bid & 7) * per + (bid >> 3);
  const int bx = bid % gridDim.x, by = bid / gridDim.x;
  const int mtiles = a.M / (64 * BMT);
  const int ph = bx / mtiles;
  const int m0 = (bx - ph * mtiles) * 64 * BMT;
  const int ncol = a.B * a.Tin;
  const int col0 = by * 128;
  const uint16_t* A = a.Abf[ph];
  const int Ktot = a.nseg * a.Cin;
  const size_t plane = (size_t)a.M * Ktot;
  const int d0 = a.dph[ph][0], d1 = a.dph[ph][1];
  __shared__ uint4 As[3][4 * BMT][64];  // [plane][m-tile][lane]: A fragments
  __shared__ uint4 Bs[3][8][64];        // [part][n-tile][lane]: B fragments

  // staging roles: A — rows ar + 64 r, k quarter aq (8 k, 16 B per plane);
  // X — column xn = tid / 2, channel half xh = tid % 2 (16 channels, 4 x float4)
  const int ar = tid >> 2, aq = tid & 3;
  const uint16_t* Arow = A + (size_t)(m0 + ar) * Ktot + 8 * aq;
  const int xn = tid >> 1, xh = tid & 1;
  const int xcol = col0 + xn;
  const bool xin = xcol < ncol;
  const int xbt = xin ? xcol / a.Tin : 0, xt = xin ? xcol - xbt * a.Tin : 0;
  const float* Xw = a.X + (size_t)xbt * a.Tin * a.Cin;
  // (native vector types: as HIP's uint4 struct the copies global -> ra -> LDS were lowered
  // to memcpy and ra lived in scratch memory, a store + reload per k step behind vmcnt waits)
  typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
  u32x4v ra[BMT][3];
  float4 rx[4];
  bool xok = false;
  // (macros, not lambdas: with the staging registers captured by reference the compiler kept
  // ra in scratch memory -- a store and a reload per k step behind a vmcnt wait)
#define MX_TILED_GLOAD(KC)                                                                     \
  do {                                                                                         \
    const int kc_ = (KC);                                                                      \
    _Pragma("unroll") for (int r = 0; r < BMT; ++r)                                            \
    _Pragma("unroll") for (int p = 0; p < 3; ++p)                                              \
      ra[r][p] = *reinterpret_cast<const u32x4v*>(Arow + (size_t)64 * r * Ktot + p * plane + kc_); \
    const int seg_ = kc_ >= a.Cin ? 1 : 0;                                                     \
    const int t_ = xt + (seg_ ? d1 : d0);                                                      \
    xok = xin && t_ >= 0 && t_ < a.Tin;                                                        \
    /* unconditional loads (the address is clamped in range), zeroed in MX_TILED_LSTORE */     \
    const float4* xp_ = reinterpret_cast<const float4*>(                                       \
        Xw + (size_t)min(max(t_, 0), a.Tin - 1) * a.Cin + (kc_ - seg_ * a.Cin) + 16 * xh);     \
    _Pragma("unroll") for (int q = 0; q < 4; ++q) rx[q] = xp_[q];                              \
  } while (0)
#define MX_TILED_LSTORE()                                                                      \
  do {                                                                                         \
    _Pragma("unroll") for (int r = 0; r < BMT; ++r)                                            \
    _Pragma("unroll") for (int p = 0; p < 3; ++p)                                              \
      As[p][4 * r + (ar >> 4)][aq * 16 + (ar & 15)] = __builtin_bit_cast(uint4, ra[r][p]);     \
    _Pragma("unroll") for (int h = 0; h < 2; ++h) { /* channels 8 (2 xh + h) .. of column xn */ \
      float x_[8] = {rx[2 * h].x, rx[2 * h].y, rx[2 * h].z, rx[2 * h].w,                       \
                     rx[2 * h + 1].x, rx[2 * h + 1].y, rx[2 * h + 1].z, rx[2 * h + 1].w};      \
      _Pragma("unroll") for (int e = 0; e < 8; ++e) x_[e] = xok ? x_[e] : 0.f;                \
      bf16x8 xf_[3];                                                                           \
      rows::split_parts<3>(x_, xf_);                                                           \
      const int gg_ = 2 * xh + h;                                                              \
      _Pragma("unroll") for (int p = 0; p < 3; ++p)                                            \
        Bs[p][xn >> 4][gg_ * 16 + (xn & 15)] = __builtin_bit_cast(uint4, xf_[p]);              \
    }                                                                                          \
  } while (0)

  f32x4 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  MX_TILED_GLOAD(0);
  for (int kc = 0; kc < Ktot; kc += 32) {
    __syncthreads();  // the previous step's fragments are consumed
    MX_TILED_LSTORE();
    __syncthreads();
    if (kc + 32 < Ktot) MX_TILED_GLOAD(kc + 32);
    bf16x8 af[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int p = 0; p < 3; ++p) af[i][p] = __builtin_bit_cast(bf16x8, As[p][2 * wm + i][lane]);
    constexpr int PA[6] = {1, 0, 2, 0, 1, 0}, PB[6] = {1, 2, 0, 1, 0, 0};
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      bf16x8 bfr[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) bfr[p] = __builtin_bit_cast(bf16x8, Bs[p][NJ * wn + j][lane]);
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][PA[q]], bfr[PB[q]], acc[i][j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = col0 + 16 * (NJ * wn + j) + c;
    if (col >= ncol) continue;
    const int bt = col / a.Tin, t = col - bt * a.Tin;
#pragma unroll
    for (int i = 0; i < 2; ++i) conv_gemm_store4(a, acc[i][j], m0 + 32 * wm + 16 * i + 4 * g, t, ph, bt);
  }
}

#undef MX_TILED_GLOAD
#undef MX_TILED_LSTORE

// fp32 [n] -> three bf16 planes [3][n] (x = p0 + p1 + p2), for the conv-GEMM weights.
__global__ void split_planes_kernel(const float* src, uint16_t* dst, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float r = src[i];
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    const uint32_t pk = pack2_bf16(r, 0.f);
    dst[p * n + i] = (uint16_t)(pk & 0xffffu);
    r -= bf16_lo(pk);
  }
}

hipError_t launch_split_planes(const float* src, uint16_t* dst, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src,
                     dst, n);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// Output stage: conv 64->1 k7 pad 3 (+bias) -> tanh on the Snake-activated input (the
// last ResidualUnit's epilogue wrote Snake(x, out.alpha)), then the PCM16 epilogue on the
// [lo, hi) slice: (x * 32767) truncated toward zero, as (audio_slice*32767).to(int16).
// Grid (ceil(T / OUT_T), B), block 256.  The block stages its input rows [t0 - 3, t0 + OUT_T
// + 3) (channels-last, 256 B per row) in LDS with coalesced 16-byte loads, then 16 lanes share
// one output sample: lane j holds channels 4j .. 4j+3 of the 7 taps' weights in registers, reads
// one 16-byte piece per tap (a row is 256 contiguous bytes: conflict-free), and the 16 partial
// sums meet by butterfly.  (One thread per sample straight from global memory touched 16-64
// cache lines per load instruction: 139 us for 32 windows, against ~20 us of HBM bytes.)
// ---------------------------------------------------------------------------------
constexpr int OUT_T = 256;
__global__ __launch_bounds__(256) void snac_out_kernel(const float* xs, const float* w,
                                                       const float* b, int T, int lo, int hi,
                                                       float* audio, int16_t* pcm,
                                                       const SnacIO* io) {
  if (io) {
    audio = io->audio;
    pcm = io->pcm;
  }
  __shared__ float4 xt[OUT_T + 6][16];  // rows t0 - 3 .. t0 + OUT_T + 2, 64 channels each
  const int bt = blockIdx.y, t0 = blockIdx.x * OUT_T;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float4* xb = reinterpret_cast<const float4*>(xs + (size_t)bt * T * 64);
  // every staging load issued before any is stored (a load -> store loop waits one memory
  // round trip per iteration)
  constexpr int NL = ((OUT_T + 6) * 16 + 255) / 256;
  float4 xv[NL];
#pragma unroll
  for (int n = 0; n < NL; ++n) {
    const int i = tid + 256 * n, r = i >> 4, q = i & 15, tt = t0 - 3 + r;
    xv[n] = (i < (OUT_T + 6) * 16 && tt >= 0 && tt < T) ? xb[(size_t)tt * 16 + q]
                                                        : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int n = 0; n < NL; ++n) {
    const int i = tid + 256 * n;
    if (i < (OUT_T + 6) * 16) xt[i >> 4][i & 15] = xv[n];
  }
  const int j = lane & 15, sub = lane >> 4;  // channel quad j; 4 samples per wave instruction
  float wk[7][4];
#pragma unroll
  for (int k = 0; k < 7; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) wk[k][e] = w[(4 * j + e) * 7 + k];
  const float bias = b[0];
  __syncthreads();
  // wave wid: samples t0 + 64 wid + 4 it + sub, it = 0..15
  for (int it = 0; it < OUT_T / 16; ++it) {
    const int tl = 64 * wid + 4 * it + sub;  // local sample; its taps are rows tl .. tl + 6
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const float4 v = xt[tl + k][j];
      acc = fmaf(wk[k][0], v.x, acc);
      acc = fmaf(wk[k][1], v.y, acc);
      acc = fmaf(wk[k][2], v.z, acc);
      acc = fmaf(wk[k][3], v.w, acc);
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    acc += __shfl_xor(acc, 4, 64);
    acc += __shfl_xor(acc, 8, 64);
    const int t = t0 + tl;
    if (j != 0 || t >= T) continue;
    const float v = tanhf(acc + bias);
    if (audio) audio[(size_t)bt * T + t] = v;
    if (pcm && t >= lo && t < hi) {
      const float s = v * 32767.0f;
      pcm[(size_t)bt * (hi - lo) + (t - lo)] = (int16_t)truncf(s);
    }
  }
}

// Counter-based Gaussian noise (Box-Muller over a 64-bit mix hash) for NoiseBlock when the
// caller does not pass explicit noise (the reference draws torch.randn per call).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// N(0,1) noise.  seeds == null: element i of the whole batch from `seed`; otherwise item
// b = i / per draws element j = i % per from seeds[b], so a window's noise depends only on
// its own seed (batching-invariant streams).
__global__ void gauss_kernel(float* out, int64_t n, uint64_t seed, const uint64_t* seeds,
                             int64_t per, const SnacIO* io) {
  if (io) {
    seed = io->seed;
    seeds = io->seeds;
  }
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t j = seeds ? (uint64_t)(i % per) : (uint64_t)i;
  const uint64_t h = mix64((seeds ? seeds[i / per] : seed) ^ mix64(j));
  const float u1 = ((float)(h >> 40) + 1.0f) * (1.0f / 16777217.0f);
  const float u2 = (float)((h >> 16) & 0xffffff) * (1.0f / 16777216.0f);
  out[i] = sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}

// ---------------------------------------------------------------------------------
__global__ void set_io_kernel(SnacIO* dst, SnacIO v) { *dst = v; }

hipError_t launch_set_io(SnacIO* dst, const SnacIO& v, hipStream_t st) {
  hipLaunchKernelGGL(set_io_kernel, dim3(1), dim3(1), 0, st, dst, v);
  return hipGetLastError();
}

hipError_t launch_snac_embed(const int32_t* frames, int n_frames, int B,
                             const float* const* codebooks, const float* const* proj_w,
                             const float* const* proj_b, float* z, hipStream_t st,
                             const SnacIO* io) {
  EmbedPtrs p;
  for (int i = 0; i < 3; ++i) {
    p.cb[i] = codebooks[i];
    p.w[i] = proj_w[i];
    p.b[i] = proj_b[i];
  }
  hipLaunchKernelGGL(snac_embed_kernel, dim3(4 * n_frames, B), dim3(256), 0, st, frames,
                     n_frames, p, z, io);
  return hipGetLastError();
}

hipError_t launch_dwconv(const float* x, float* y, const float* w, const float* b,
                         const float* alpha_in, const float* alpha_out, int B, int C, int T,
                         int dil, hipStream_t st) {
  if (dil > 9 || C % 64) return hipErrorInvalidValue;
  // 64-step tiles once there are enough of them (16-step tiles re-read the dil-9 halo 4.4x;
  // with 16-byte lanes the 64-step tile wins from B * T = 16K: 32 windows at T = 1792)
  if ((int64_t)B * T >= 16384)
    hipLaunchKernelGGL(dwconv_kernel<64>, dim3((T + 63) / 64, C / 64, B), dim3(256), 0, st, x, y,
                       w, b, alpha_in, alpha_out, C, T, dil);
  else
    hipLaunchKernelGGL(dwconv_kernel<16>, dim3((T + 15) / 16, C / 64, B), dim3(256), 0, st, x, y,
                       w, b, alpha_in, alpha_out, C, T, dil);
  return hipGetLastError();
}

hipError_t launch_conv_gemm(const ConvGemmArgs& a, int nphase, hipStream_t st) {
  const int Ktot = a.nseg * a.Cin;
  if (a.tiled) {
    if (a.M % 64 || a.Cin % 32) return hipErrorInvalidValue;
    const int ctiles = (a.B * a.Tin + 127) / 128;
    if (ctiles > 65535) return hipErrorInvalidValue;
    // BMT = 2 (128 x 128 blocks) is parity-green but slower: 0.101 vs 0.098 ms per window at
    // x32, 0.164 vs 0.138 at x8 (occupancy 2 vs 4; profiles/r02_snac_tile_bm.log)
    hipLaunchKernelGGL(conv_gemm_tiled_kernel<1>, dim3(a.M / 64 * nphase, ctiles), dim3(256), 0, st, a);
    return hipGetLastError();
  }
  if (a.M % 32 || a.Cin % 32 || Ktot % (64 * a.wk)) return hipErrorInvalidValue;
  const int bn = 16 * a.nsub;
  const dim3 grid((a.Tin + bn - 1) / bn, a.M / 32, nphase * a.B);
#define MX_CG(WK_, NS_)                                                                   \
  if (a.wk == WK_ && a.nsub == NS_) {                                                     \
    if (WK_ == 1)                                                                         \
      hipLaunchKernelGGL((conv_gemm1_kernel<NS_>), grid, dim3(64), 0, st, a);             \
    else                                                                                  \
      hipLaunchKernelGGL((conv_gemm_kernel<WK_, NS_>), grid, dim3(WK_ * 64), 0, st, a);   \
    return hipGetLastError();                                                             \
  }
  MX_CG(1, 2) MX_CG(1, 4) MX_CG(2, 2) MX_CG(2, 4) MX_CG(4, 2) MX_CG(4, 4) MX_CG(8, 2)
  MX_CG(8, 4)
#undef MX_CG
  return hipErrorInvalidValue;
}

hipError_t launch_snac_out(const float* xs, const float* w, const float* b, int B, int T,
                           int lo, int hi, float* audio, int16_t* pcm, hipStream_t st,
                           const SnacIO* io) {
  hipLaunchKernelGGL(snac_out_kernel, dim3((T + OUT_T - 1) / OUT_T, B), dim3(256), 0, st, xs, w, b, T, lo,
                     hi, audio, pcm, io);
  return hipGetLastError();
}

hipError_t launch_gauss(float* out, int64_t n, uint64_t seed, const uint64_t* seeds, int64_t per,
                        hipStream_t st, const SnacIO* io) {
  hipLaunchKernelGGL(gauss_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, n,
                     seed, seeds, per, io);
  return hipGetLastError();
}

}  // namespace mx
