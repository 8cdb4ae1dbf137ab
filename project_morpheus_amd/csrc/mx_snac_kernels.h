// SNAC 24 kHz decoder kernels (snac_kernels.hip).  fp32 arithmetic (the reference never casts
// SNAC: speechpipe.py:43-49), activations channels-last [batch][time][channels].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mx {

enum { CG_STORE = 0, CG_RESID = 1, CG_NOISE = 2 };

struct ConvGemmArgs {
  const uint16_t* Abf[8];  // per phase: bf16 planes [3][M][nseg*Cin] (ConvTranspose packed per phase)
  int dph[8][2];        // per phase: time shift of each K segment
  const float* X;       // [B][Tin][Cin]
  const float* bias;    // [M] or null
  const float* R;       // residual source [B][Tout][M] (CG_RESID / CG_NOISE)
  const float* noise;   // window b's noise at noise + b * noise_stride (CG_NOISE)
  int noise_stride;
  float* out;           // [B][Tout][M]
  float* out2;          // optional: Snake(out, alpha2) [B][Tout][M] for the next consumer
  const float* alpha2;
  int M, Cin, Tin, Tout, B;
  int nseg;
  int col_stride;       // output column = col_stride * n + phase
  int epi;
  int wk, nsub;         // waves splitting K; 16-column subtiles per tile
  int tiled;            // 1: block-tiled kernel over the windows' concatenated columns
};

// Per-call I/O of a graph-captured window decode: the captured kernels read these from a
// ctx-owned device copy (written by set_io before each replay), so one graph serves every
// call of its shape.  Eager launches pass io = nullptr and use their direct arguments.
struct SnacIO {
  const int32_t* frames;
  const uint64_t* seeds;
  uint64_t seed;
  int16_t* pcm;
  float* audio;
};
hipError_t launch_set_io(SnacIO* dst, const SnacIO& v, hipStream_t st);

hipError_t launch_snac_embed(const int32_t* frames, int n_frames, int B,
                             const float* const* codebooks, const float* const* proj_w,
                             const float* const* proj_b, float* z, hipStream_t st,
                             const SnacIO* io = nullptr, float* noise = nullptr,
                             int64_t noise_n = 0, int64_t noise_per = 1, uint64_t seed = 0,
                             const uint64_t* seeds = nullptr);
hipError_t launch_dwconv(const float* x, float* y, const float* w, const float* b,
                         const float* alpha_in, const float* alpha_out, int B, int C, int T,
                         int dil, hipStream_t st);
hipError_t launch_conv_gemm(const ConvGemmArgs& a, int nphase, hipStream_t st);
hipError_t launch_split_planes(const float* src, uint16_t* dst, int64_t n, hipStream_t st);
hipError_t launch_snac_out(const float* xs, const float* w, const float* b, int B, int T,
                           int lo, int hi, float* audio, int16_t* pcm, hipStream_t st,
                           const SnacIO* io = nullptr);
hipError_t launch_snac_cut(const float* src, float* dst, int B, int T, int C, int c0, int n,
                           hipStream_t st);

}  // namespace mx
