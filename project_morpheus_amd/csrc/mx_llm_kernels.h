// Argument blocks and launchers for the decode-step kernels (llm_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mx {

enum { EPI_STORE = 0, EPI_RESID = 1, EPI_SILU = 2, EPI_QKV = 3, EPI_ARGMAX = 4 };
enum { WT_BF16 = 0, WT_FP8 = 1 };  // weight storage: bf16, or OCP e4m3 + fp32 scale per row

constexpr int ATT_S_MIN = 128;      // smallest split (positions) = 4 waves x 32 x 1 chunk
constexpr int ATT_MAX_SPLITS = 256; // splits one launch may merge
constexpr int ATT_MAXG = 4;         // max q-heads per kv-head
constexpr int ATT_MERGE_CHUNK = 16; // splits whose partials the merging block prefetches

struct GemvArgs {
  const void* W;           // [N][K] bf16 (WT_BF16) or e4m3 bytes (WT_FP8), packed row order
  const float* wscale;     // WT_FP8: dequant scale per row [N]
  int wdtype;
  int N, K;
  const float* X;          // activations, row r at X + r * xstride
  int xstride;
  int R;                   // activation rows
  const float* norm_w;     // RMSNorm weight [K] (NORM prologue)
  float eps;
  float* Y;                // STORE [R][N]; RESID [R][ystride] += ; SILU [R][N/2]
  int ystride;
  int max_blocks;          // grid cap (0 = default)
  int force_legacy;        // 1: use the grid-stride kernel even for R = 1 (A/B timing)
  int wpb;                 // R = 1 kernel: waves per block (4 or 8; 0 = 8)
  int rpw;                 // R = 1 kernel: weight rows per wave (0 = default per epilogue)
  float* ws;               // R >= 2 kernel: split-K partial tiles (gemm_rows_workspace)
  size_t ws_floats;
  int* tickets;            // R >= 2 kernel: per-tile arrival counters (zero between launches)
  size_t tickets_n;
  int rows_dbg;             // R >= 2 kernel timing experiments (0 = product; results invalid otherwise)
  int rows_npart;          // R >= 2 kernel: activation bf16 parts (2 or 3; 0 = 3)
  int rows_pw;             // generation 4: weight prefetch distance in sub-chunks (1, 2; 0 = 1)
  int rows_pw_f8;          // the same for e4m3 weights
  int rows_target;         // generation 4: blocks the K-range split aims for (0 = per shape)
  int rows_nt_max;         // generation 4: largest batch tile in 16-row units (0 = 4)
  int rows_kernel;         // R >= 2 kernel generation: 4 (default), 7 (falls back to 4 outside its shapes), 5
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
  const uint16_t* vcache;  // TRANSPOSED: [slot][kv_head][128][max_pos]
  const int32_t* row_slot;
  const int32_t* row_pos;
  int heads, kv_heads, max_pos;
  int cpw;                 // 32-position chunks per wave: split = 32 * nw * cpw positions
  int nw;                  // waves per block (4 or 8; 0 = 4)
  int split_stride;        // partial slots per (row, kv-head) >= max_pos / split
  float scale;
  float* part_ml;          // [R][kv_heads][nsplit_max][grp][2]  (m, l) per split
  float* part_acc;         // [R][kv_heads][nsplit_max][grp][128]
  int* counter;            // [R][kv_heads] split arrival tickets (zero between launches)
  float* out;              // [R][heads*128]
  int debug;               // timing experiments only (0 in the product path)
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
  int scratch_slot;          // rows bound to this slot are parked: no advance, no history
};

// ---- persistent single-stream decode step (llm_mega.hip) --------------------------------
// Fixed to the Orpheus-3B / Llama-3.2-3B shapes (hidden 3072, 24/8 heads of 128, FFN 8192).
constexpr int MEGA_BLOCKS = 256;     // one block per CU, all resident
constexpr int MEGA_SPLIT = 128;      // attention positions per split (one control wave)
constexpr int MEGA_PART = 392;       // floats per split partial: acc[3][128], m[3], l[3], pad
constexpr int MEGA_MAX_SPLITS = MEGA_BLOCKS / 8;  // longest fast-path context: 4096 positions
// per-layer activation vectors (floats); each has its own lines, none is rewritten in a launch
constexpr int MEGA_OFF_QKV = 0;      // q[24][128] | k[8][128] | v[8][128] (k, v bf16-exact)
constexpr int MEGA_OFF_ATT = 5120;   // attention output [3072]
constexpr int MEGA_OFF_HA = 8192;    // residual after attention [3072]
constexpr int MEGA_OFF_ACT = 11264;  // SiLU(gate) * up [8192]
constexpr int MEGA_OFF_HB = 19456;   // residual after the MLP [3072]
constexpr int MEGA_WS_LAYER = 22528;
// per-layer sync words (ints), zeroed by a memset node before every launch
constexpr int MEGA_SYNC_Q = 0, MEGA_SYNC_O = 1, MEGA_SYNC_G = 2, MEGA_SYNC_D = 3;
constexpr int MEGA_SYNC_TICK = 4;    // [8] split arrival tickets per kv head
constexpr int MEGA_SYNC_DONE = 12;   // kv heads whose attention output is published
constexpr int MEGA_SYNC_LAYER = 16;  // + one status word after the last layer (0 = ok)
// sync words (+ status, padded to 16 B) are followed by the per-block seam flags
inline size_t mega_sync_ints(int layers) { return ((size_t)layers * MEGA_SYNC_LAYER + 1 + 3) / 4 * 4; }
inline size_t mega_flag_ints(int layers) { return (size_t)layers * 4 * MEGA_BLOCKS; }

struct MegaArgs {
  const void *wqkv, *wo, *wgu, *wd;  // [layers][packed rows][K] contiguous (bf16 or e4m3)
  const float *sqkv, *so, *sgu, *sd; // fp8 row scales [layers][rows] (unused for bf16)
  const float *attn_norm, *mlp_norm; // [layers][3072]
  const float *rope_cos, *rope_sin;  // [max_pos][64]
  const int32_t *row_slot, *row_pos; // decode row 0
  uint16_t *kcache, *vcache;         // [layers][slots][8][max_pos][128], V^T per head
  size_t kv_layer_elems;
  int max_pos, layers, nsplit_cap;   // nsplit_cap: split partial slots per (layer, kv head)
  int f8, ring;                      // e4m3 weights; register ring depth (8, 16, 32 or 48 units)
  const float* h_in;                 // [3072] input embedding row (commit kernel output)
  float* h_out;                      // [3072] residual after the last layer (lm_head input)
  float* ws;                         // [layers][MEGA_WS_LAYER]
  float* part;                       // [layers][8][nsplit_cap][MEGA_PART]
  int* sync;                         // [layers][MEGA_SYNC_LAYER] + status
  int* flags;                        // [layers][4 seams][256 blocks] arrival flags (same memset)
  const void* dummy;                 // >= 128 KB of zeros: the ring's loads past the last layer
  float eps, att_scale;
  long long* trace;                  // diagnostics: [blocks][layers][MEGA_TRACE_EV] wall clocks, or null
};
constexpr int MEGA_TRACE_EV = 16;
hipError_t launch_mega(const MegaArgs& a, hipStream_t st);
hipError_t mega_resident(int device, int f8, int ring, int* ok);

hipError_t gemv_prepare(int kmax);
hipError_t launch_gemv(const GemvArgs& a, int epi, bool norm, hipStream_t st);
// R >= 2 rows on bf16 MFMA (llm_batched.hip); hipErrorNotSupported if the shape is not covered
hipError_t launch_gemm_rows(const GemvArgs& a, int epi, bool norm, hipStream_t st);
void gemm_rows_workspace(int N, int K, int R, int epi, size_t* ws_floats, size_t* tickets);
namespace v4 {  // multi-row GEMM generation 4 (llm_batched_v4.hip): the default product path
hipError_t launch_gemm_rows_v4(const GemvArgs& a, int epi, bool norm, hipStream_t st);
void gemm_rows_workspace_v4(int N, int K, int R, int epi, size_t* ws_floats, size_t* tickets);
}  // namespace v4
// R = 2..32 rows, one block per weight tile, K split over its waves (llm_batched_v7.hip);
// hipErrorNotSupported outside the Orpheus-3B projection shapes
hipError_t launch_gemm_rows_v7(const GemvArgs& a, int epi, bool norm, hipStream_t st);
hipError_t launch_set_rows(int32_t* slot, int32_t* pos, int n, int slot_val, int pos0,
                           hipStream_t st);
hipError_t launch_set_scalar(float* p, float v, hipStream_t st);
hipError_t launch_attention(const AttnArgs& a, int R, int max_len, hipStream_t st);
hipError_t launch_commit(const CommitArgs& a, int R, hipStream_t st);
hipError_t launch_embed_rows(const int32_t* ids, int n, int slot, const uint16_t* embed,
                             int hidden, int vocab, uint8_t* seen, float* h, hipStream_t st);
hipError_t launch_scatter_rows(void* dst, const void* src, const int32_t* dmap, int rows,
                               int cols, int mode, hipStream_t st);
hipError_t launch_to_f32(float* dst, const void* src, int64_t n, int src_bf16, hipStream_t st);

}  // namespace mx
