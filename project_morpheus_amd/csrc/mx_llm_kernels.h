// Argument blocks and launchers for the decode-step kernels (llm_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mx {

enum { EPI_STORE = 0, EPI_RESID = 1, EPI_SILU = 2, EPI_QKV = 3, EPI_ARGMAX = 4 };

constexpr int ATT_CHUNK = 64;  // positions per attention split
constexpr int ATT_MAXG = 4;    // max q-heads per kv-head (one wave each)

struct GemvArgs {
  const uint16_t* W;       // [N][K] bf16, packed row order
  int N, K;
  const float* X;          // activations, row r at X + r * xstride
  int xstride;
  int R;                   // activation rows
  const float* norm_w;     // RMSNorm weight [K] (NORM prologue)
  float eps;
  float* Y;                // STORE [R][N]; RESID [R][ystride] += ; SILU [R][N/2]
  int ystride;
  int max_blocks;          // grid cap (0 = default)
  // EPI_QKV
  const float* rope_cos;   // [max_pos][64]
  const float* rope_sin;
  const int32_t* row_slot;
  const int32_t* row_pos;
  uint16_t* kcache;        // this layer: [slots][kv_heads][max_pos][128]
  uint16_t* vcache;
  int heads, kv_heads, max_pos;
  float* Q;                // [R][heads][128]
  // EPI_ARGMAX
  const uint8_t* seen;     // [slots][N]
  const float* penalty;    // device scalar
  unsigned long long* best;  // [R]
  float* logits;           // optional debug copy of penalised logits [R][N]
};

struct AttnArgs {
  const float* Q;          // [R][heads][128]
  const uint16_t* kcache;  // this layer
  const uint16_t* vcache;
  const int32_t* row_slot;
  const int32_t* row_pos;
  int heads, kv_heads, max_pos, nsplit_max;
  float scale;
  float* part_ml;          // [R][heads][nsplit_max][2]
  float* part_acc;         // [R][heads][nsplit_max][128]
  float* out;              // [R][heads*128]
};

struct CommitArgs {
  unsigned long long* best;  // [R]
  const int32_t* dst_row;    // optional remap
  int32_t* row_slot;
  int32_t* row_pos;
  int32_t* row_token;
  uint8_t* seen;
  int32_t* hist;             // host-mapped [slots][max_pos]
  const uint16_t* embed;
  float* h;
  int hidden, vocab, max_pos, pos_advance;
};

hipError_t gemv_prepare(int kmax);
hipError_t launch_gemv(const GemvArgs& a, int epi, bool norm, hipStream_t st);
hipError_t launch_set_rows(int32_t* slot, int32_t* pos, int n, int slot_val, int pos0,
                           hipStream_t st);
hipError_t launch_set_scalar(float* p, float v, hipStream_t st);
hipError_t launch_attention(const AttnArgs& a, int R, hipStream_t st);
hipError_t launch_commit(const CommitArgs& a, int R, hipStream_t st);
hipError_t launch_embed_rows(const int32_t* ids, int n, int slot, const uint16_t* embed,
                             int hidden, int vocab, uint8_t* seen, float* h, hipStream_t st);
hipError_t launch_pack_rows(uint16_t* dst, const void* src, const int32_t* perm, int rows,
                            int cols, int src_f32, hipStream_t st);
hipError_t launch_to_f32(float* dst, const void* src, int64_t n, int src_bf16, hipStream_t st);

}  // namespace mx
