// SNAC 24 kHz codec decoder on MI355X (gfx950), fp32 end to end.
//
// Replaces snac.SNAC.decode (third-party snac 1.2.x; call site
// Morpheus_Client/tts_engine/speechpipe.py:118) plus the slice / PCM16 epilogue
// (speechpipe.py:122-129).  Every dense contraction (1x1 convs, NoiseBlock linear,
// polyphase ConvTranspose1d) runs as one "segmented conv-GEMM" on the exact-f32 MFMA
// (v_mfma_f32_16x16x4_f32: bit-for-bit a k-ordered fmaf chain), with the Snake
// activation fused into the B-operand loader and bias / residual / noise fused into the
// epilogue.  Depthwise dilated k7 convs stage a haloed, Snake-activated tile in LDS.
#include "mx_common.h"
#include "mx_snac_kernels.h"

namespace mx {

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float snake(float x, float a) {
  // layers.py snake(): x + (alpha + 1e-9).reciprocal() * sin(alpha * x)^2
  const float s = sinf(a * x);
  return x + (1.0f / (a + 1e-9f)) * (s * s);
}

// ---------------------------------------------------------------------------------
// RVQ from_codes (vq.py): z[c][t] = sum_i out_proj_i(codebook_i[code_i[t / stride_i]])
// frames: [B][7N] codes in speechpipe order; de-interleave per speechpipe.py:84-98.
// Grid (4N, B), block 256.
// ---------------------------------------------------------------------------------
struct EmbedPtrs {
  const float* cb[3];
  const float* w[3];
  const float* b[3];
};

__global__ __launch_bounds__(256) void snac_embed_kernel(const int32_t* frames, int n_frames,
                                                         EmbedPtrs p, float* z) {
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
    z[((size_t)bt * 768 + c) * T + t] = zc;
  }
}

// ---------------------------------------------------------------------------------
// Depthwise k7 dilated conv, "same" padding 3*dil, optional Snake on input and output.
// Grid (ceil(T/256), C, B), block 256; haloed Snake(x) tile in LDS.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dwconv_kernel(const float* x, float* y, const float* w,
                                                     const float* b, const float* ain,
                                                     const float* aout, int C, int T, int dil) {
  const int c = blockIdx.y, bt = blockIdx.z;
  const int t0 = blockIdx.x * 256;
  const int halo = 3 * dil;
  __shared__ float tile[256 + 2 * 27];
  const float* xr = x + ((size_t)bt * C + c) * T;
  const float a_in = ain ? ain[c] : 0.f;
  for (int i = threadIdx.x; i < 256 + 2 * halo; i += 256) {
    const int t = t0 - halo + i;
    float v = 0.f;
    if (t >= 0 && t < T) {
      v = xr[t];
      if (ain) v = snake(v, a_in);
    }
    tile[i] = v;
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= T) return;
  float acc = b[c];
#pragma unroll
  for (int k = 0; k < 7; ++k) acc = fmaf(w[c * 7 + k], tile[threadIdx.x + k * dil], acc);
  if (aout) acc = snake(acc, aout[c]);
  y[((size_t)bt * C + c) * T + t] = acc;
}

// ---------------------------------------------------------------------------------
// Segmented conv-GEMM on f32 MFMA 16x16x4.
//   out[b][m][col_stride*n + col_off] = epi( sum_seg sum_ci A[m][seg*Cin+ci]
//                                            * f(X[b][ci][n + delta_seg]) )
// Tile 64 (M) x 64 (n) x 16 (k); 4 waves, each a 32x32 sub-tile of 2x2 MFMA tiles.
// Grid (ceil(Tin/64), M/64, B).
// ---------------------------------------------------------------------------------
constexpr int CG_BM = 64, CG_BN = 64, CG_BK = 16;

__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvGemmArgs a) {
  __shared__ float As[CG_BK][CG_BM + 4];
  __shared__ float Bs[CG_BK][CG_BN + 4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n0 = blockIdx.x * CG_BN, m0 = blockIdx.y * CG_BM, bt = blockIdx.z;
  const int Ktot = a.nseg * a.Cin;
  const float* X = a.X + (size_t)bt * a.Cin * a.Tin;
  const int wm = (wid >> 1) * 32, wn = (wid & 1) * 32;
  floatx4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // loader mapping: A: thread -> (row m = tid/4, k quad = (tid%4)*4); B: (k = tid/16, n quad)
  const int am = tid >> 2, ak = (tid & 3) * 4;
  const int bk = tid >> 4, bn = (tid & 15) * 4;
  for (int k0 = 0; k0 < Ktot; k0 += CG_BK) {
    {
      const float4 v = *reinterpret_cast<const float4*>(a.A + (size_t)(m0 + am) * Ktot + k0 + ak);
      As[ak + 0][am] = v.x;
      As[ak + 1][am] = v.y;
      As[ak + 2][am] = v.z;
      As[ak + 3][am] = v.w;
    }
    {
      const int kk = k0 + bk;
      const int seg = kk / a.Cin, ci = kk - seg * a.Cin;
      const int d = seg == 0 ? a.delta[0] : a.delta[1];
      const float* xr = X + (size_t)ci * a.Tin;
      const float al = a.alpha ? a.alpha[ci] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int t = n0 + bn + q + d;
        float v = 0.f;
        if (n0 + bn + q < a.Tin && t >= 0 && t < a.Tin) {
          v = xr[t];
          if (a.alpha) v = snake(v, al);
        }
        Bs[bk][bn + q] = v;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k4 = 0; k4 < CG_BK; k4 += 4) {
      const int kr = k4 + (lane >> 4);
      const float a0 = As[kr][wm + (lane & 15)];
      const float a1 = As[kr][wm + 16 + (lane & 15)];
      const float b0 = Bs[kr][wn + (lane & 15)];
      const float b1 = Bs[kr][wn + 16 + (lane & 15)];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }
  // epilogue: C/D map for 16x16: col = lane & 15, row = (lane >> 4) * 4 + reg
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int m = m0 + wm + i * 16 + (lane >> 4) * 4 + reg;
        const int n = n0 + wn + j * 16 + (lane & 15);
        if (n >= a.Tin) continue;
        const int col = a.col_stride * n + a.col_off;
        float v = acc[i][j][reg];
        if (a.bias) v += a.bias[m];
        const size_t o = ((size_t)bt * a.M + m) * a.Tout + col;
        if (a.epi == CG_RESID) v = a.R[o] + v;
        else if (a.epi == CG_NOISE) v = a.R[o] + a.noise[(size_t)bt * a.noise_stride + col] * v;
        a.out[o] = v;
      }
}

// ---------------------------------------------------------------------------------
// Output stage: Snake(64) -> conv 64->1 k7 pad 3 (+bias) -> tanh; PCM16 epilogue on the
// [lo, hi) slice: (x * 32767) truncated toward zero, as (audio_slice*32767).to(int16).
// Grid (ceil(T/256), B), block 256.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void snac_out_kernel(const float* x, const float* alpha,
                                                       const float* w, const float* b, int T,
                                                       int lo, int hi, float* audio,
                                                       int16_t* pcm) {
  const int bt = blockIdx.y;
  const int t0 = blockIdx.x * 256;
  __shared__ float tile[64][256 + 6];
  const float* xb = x + (size_t)bt * 64 * T;
  for (int i = threadIdx.x; i < 64 * 262; i += 256) {
    const int c = i / 262, j = i - c * 262;
    const int t = t0 - 3 + j;
    float v = 0.f;
    if (t >= 0 && t < T) v = snake(xb[(size_t)c * T + t], alpha[c]);
    tile[c][j] = v;
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= T) return;
  float acc = b[0];
  for (int c = 0; c < 64; ++c)
#pragma unroll
    for (int k = 0; k < 7; ++k) acc = fmaf(w[c * 7 + k], tile[c][threadIdx.x + k], acc);
  const float v = tanhf(acc);
  if (audio) audio[(size_t)bt * T + t] = v;
  if (pcm && t >= lo && t < hi) {
    const float s = v * 32767.0f;
    pcm[(size_t)bt * (hi - lo) + (t - lo)] = (int16_t)truncf(s);
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
__global__ void gauss_kernel(float* out, int64_t n, uint64_t seed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = mix64(seed ^ mix64((uint64_t)i));
  const float u1 = ((float)(h >> 40) + 1.0f) * (1.0f / 16777217.0f);
  const float u2 = (float)((h >> 16) & 0xffffff) * (1.0f / 16777216.0f);
  out[i] = sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}

// ---------------------------------------------------------------------------------
hipError_t launch_snac_embed(const int32_t* frames, int n_frames, int B,
                             const float* const* codebooks, const float* const* proj_w,
                             const float* const* proj_b, float* z, hipStream_t st) {
  EmbedPtrs p;
  for (int i = 0; i < 3; ++i) {
    p.cb[i] = codebooks[i];
    p.w[i] = proj_w[i];
    p.b[i] = proj_b[i];
  }
  hipLaunchKernelGGL(snac_embed_kernel, dim3(4 * n_frames, B), dim3(256), 0, st, frames,
                     n_frames, p, z);
  return hipGetLastError();
}

hipError_t launch_dwconv(const float* x, float* y, const float* w, const float* b,
                         const float* alpha_in, const float* alpha_out, int B, int C, int T,
                         int dil, hipStream_t st) {
  if (dil > 9) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dwconv_kernel, dim3((T + 255) / 256, C, B), dim3(256), 0, st, x, y, w, b,
                     alpha_in, alpha_out, C, T, dil);
  return hipGetLastError();
}

hipError_t launch_conv_gemm(const ConvGemmArgs& a, int B, hipStream_t st) {
  if (a.M % CG_BM || (a.nseg * a.Cin) % CG_BK || a.Cin % CG_BK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(conv_gemm_kernel, dim3((a.Tin + CG_BN - 1) / CG_BN, a.M / CG_BM, B),
                     dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_snac_out(const float* x, const float* alpha, const float* w, const float* b,
                           int B, int T, int lo, int hi, float* audio, int16_t* pcm,
                           hipStream_t st) {
  hipLaunchKernelGGL(snac_out_kernel, dim3((T + 255) / 256, B), dim3(256), 0, st, x, alpha, w,
                     b, T, lo, hi, audio, pcm);
  return hipGetLastError();
}

hipError_t launch_gauss(float* out, int64_t n, uint64_t seed, hipStream_t st) {
  hipLaunchKernelGGL(gauss_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, n,
                     seed);
  return hipGetLastError();
}

}  // namespace mx
