// SNAC 24 kHz decoder kernels (snac_kernels.hip).  All fp32 (the reference never casts
// SNAC: speechpipe.py:43-49), activations laid out [batch][channels][time].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mx {

enum { CG_STORE = 0, CG_RESID = 1, CG_NOISE = 2 };

struct ConvGemmArgs {
  const float* A;       // [M][nseg*Cin] row-major (packed per phase for ConvTranspose)
  const float* X;       // [B][Cin][Tin]
  const float* alpha;   // Snake alpha on the input channels, or null
  const float* bias;    // [M] or null
  const float* R;       // residual source [B][M][Tout] (CG_RESID / CG_NOISE)
  const float* noise;   // window b's noise at noise + b * noise_stride (CG_NOISE)
  int noise_stride;
  float* out;           // [B][M][Tout]
  int M, Cin, Tin, Tout;
  int nseg;
  int delta[2];         // time shift per K segment
  int col_stride, col_off;  // output column = col_stride * n + col_off
  int epi;
};

hipError_t launch_snac_embed(const int32_t* frames, int n_frames, int B,
                             const float* const* codebooks, const float* const* proj_w,
                             const float* const* proj_b, float* z, hipStream_t st);
hipError_t launch_dwconv(const float* x, float* y, const float* w, const float* b,
                         const float* alpha_in, const float* alpha_out, int B, int C, int T,
                         int dil, hipStream_t st);
hipError_t launch_conv_gemm(const ConvGemmArgs& a, int B, hipStream_t st);
hipError_t launch_snac_out(const float* x, const float* alpha, const float* w, const float* b,
                           int B, int T, int lo, int hi, float* audio, int16_t* pcm,
                           hipStream_t st);
hipError_t launch_gauss(float* out, int64_t n, uint64_t seed, hipStream_t st);

}  // namespace mx
