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
constexpr int ATT_QKV_NKC_MAX = 8;  // qkv K ranges the attention sums (AttnArgs::qkv_parts)

struct GemvArgs {
  const void* W;           // [N][K] bf16 (WT_BF16) or e4m3 bytes (WT_FP8), packed row order
  const void* Wf;          // null, or the same matrix fragment-major (launch_frag_major) for R >= 2
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
  int gemv_cus;            // R = 1 kernel, option gemv_balance: CU count to balance the qkv /
                           // merging o-proj grids over (0 = off)
  int rpw;                 // R = 1 kernel: weight rows per wave (0 = default per epilogue)
  float* ws;               // R >= 2 kernel: split-K partial tiles (gemm_rows_workspace)
  size_t ws_floats;
  int* tickets;            // R >= 2 kernel: per-tile arrival counters (zero between launches)
  size_t tickets_n;
  int rows_lds_pad;        // R >= 2 kernel: extra dynamic LDS KB per block (occupancy probe; 0 = none)
  int rows_pw;             // generation 4: weight prefetch distance in sub-chunks (1, 2; 0 = 1)
  int rows_pw_f8;          // the same for e4m3 weights
  int rows_target;         // generation 4: blocks the K-range split aims for (0 = per shape)
  int rows_nt_max;         // generation 4: largest batch tile in 16-row units (0 = 4)
  int rows_head_target;    // generation 4: K-range target of the lm_head (0 = the default 192)
  int rows_head_mt;        // R >= 2 lm_head: weight rows per wave in 16-row units (1 or 2)
  int rows_atomic;         // generation 4, residual projections split over K: every K range
                           // adds its partial tile into Y with float atomics (no seam)
  float* qkv_parts;        // generation 4 EPI_QKV, decode: null, or [nkc][R][N] -- every K range
  float* qkv_ss;           // stores its raw partial (and [nkc][R] partial sums of squares);
                           // the attention launch sums them, scales, RoPEs and appends K / V
  unsigned long long* trace;  // generation 4 diagnostic: [block][8] phase stamps (null = off)
  int trace_cap;           // blocks the trace buffer holds (stamps of later blocks are dropped)
  int head_b1;             // R = 1 lm_head on the persistent kernel (head_b1.hip; 0 = gemv_kernel)
  // EPI_QKV
  const float* rope_cos;   // [max_pos][64]
  const float* rope_sin;
  const int32_t* row_slot;
  const int32_t* row_pos;
  uint16_t* kcache;        // this layer: [slots][kv_heads][max_pos * 128], 32-position chunks (kv_k_off)
  uint16_t* vcache;
  int heads, kv_heads, max_pos;
  float* Q;                // [R][heads][128]
  // R = 1 o-proj: merge the attention split partials in the prologue (attn no_merge mode)
  const float* att_ml;     // [kv_heads][att_stride][grp][2]  (m, l) per split, row 0
  const float* att_acc;    // [kv_heads][att_stride][grp][128]
  int att_S, att_stride;   // split length (positions) and partial slots per kv head
  int att_nsm;             // splits the launch may have to merge (host bound, <= 8)
  // EPI_ARGMAX
  const uint8_t* seen;     // [slots][N]
  const float* penalty;    // repetition penalty per KV slot [slots]
  const float* samp_temp;  // sampling temperature per KV slot (> 0: the row samples)
  unsigned long long* best;  // [R]
  float* logits;           // penalised logits [R][N], kept for sampling rows (or every row)
  int logits_all;          // 1: keep every row's logits (parity / debug reads)
};

struct AttnArgs {
  const float* Q;          // [R][heads][128]
  const uint16_t* kcache;  // this layer
  const uint16_t* vcache;  // the same, V chunks in P.V fragment order (kv_v_off)
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
  int no_merge;            // 1: every split stores its partial, the consumer merges (R = 1)
  // multi-row decode with the qkv GEMM's K-range partials (GemvArgs::qkv_parts): q / k / v of
  // the new position = RoPE(rsqrt(mean x^2 + eps) x sum of the partials), K / V appended here
  const float* qkv_parts;  // [nkc][R][qkv_n] raw partial sums, packed wqkv row order (null: off)
  const float* qkv_ss;     // [nkc][R] partial sums of squares of the qkv input
  int qkv_nkc, qkv_n, hidden;
  float eps;
  const float* rope_cos;   // [max_pos][64]
  const float* rope_sin;
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
  const int* abort_word;     // null, or the persistent engine's host-mapped status: when set,
                             // nothing is committed and the history entry reads -1
};


hipError_t gemv_prepare(int kmax);
hipError_t launch_gemv(const GemvArgs& a, int epi, bool norm, hipStream_t st);
// R = 1 lm_head + penalty + argmax, persistent (head_b1.hip); hipErrorNotSupported off K = 3072
hipError_t launch_head_b1(const GemvArgs& a, hipStream_t st);
namespace v4 {  // multi-row GEMM generation 4 (mx_rows_v4.inc)
hipError_t launch_gemm_rows_v4(const GemvArgs& a, int epi, bool norm, hipStream_t st);
void gemm_rows_workspace_v4(int N, int K, int R, int epi, size_t* ws_floats, size_t* tickets);
// the multi-row o-projection can merge the attention splits itself (attn no_merge)
bool rows_merge_ok_v4(const GemvArgs& o);
// K ranges the qkv launch (EPI_QKV, NORM) of these arguments splits into
int rows_qkv_nkc_v4(const GemvArgs& a);
}  // namespace v4
struct SampleArgs {
  const float* logits;     // [R][V] penalised logits (kept by the lm_head epilogue)
  const int32_t* row_slot; // [R]
  const int32_t* row_pos;  // [R] position of the row's input token (RNG counter)
  const float* temp;       // per KV slot: temperature (<= 0: greedy, kernel returns)
  const float* top_p;      // per KV slot
  const uint32_t* seed;    // per KV slot: Philox key (lo, hi)
  unsigned long long* best;  // [R] argmax-key encoded token (read by commit)
  int V;
};
hipError_t launch_sample(const SampleArgs& a, int R, hipStream_t st);
hipError_t launch_set_slot_params(float* penalty, float* temp, float* top_p, uint32_t* seed,
                                  int slot, float pen, float t, float p, uint64_t s,
                                  hipStream_t st);
hipError_t launch_set_rows(int32_t* slot, int32_t* pos, int n, int slot_val, int pos0,
                           hipStream_t st);
hipError_t launch_set_scalar(float* p, float v, hipStream_t st);
hipError_t launch_move_row(int32_t* slot, int32_t* pos, int32_t* token, float* h, int hidden,
                           int dst, int src, int scratch, hipStream_t st);
hipError_t launch_attention(const AttnArgs& a, int R, int max_len, hipStream_t st);
hipError_t launch_commit(const CommitArgs& a, int R, hipStream_t st);
hipError_t launch_embed_rows(const int32_t* ids, int n, int slot, const uint16_t* embed,
                             int hidden, int vocab, uint8_t* seen, float* h, hipStream_t st);
hipError_t launch_scatter_rows(void* dst, const void* src, const int32_t* dmap, int rows,
                               int cols, int mode, hipStream_t st);
hipError_t launch_to_f32(float* dst, const void* src, int64_t n, int src_bf16, hipStream_t st);
// [N][K] (esz bytes per element) -> fragment-major copy for the multi-row GEMM (mx_rows_v4.inc)
hipError_t launch_frag_major(const void* src, void* dst, int N, int K, int esz, hipStream_t st);
inline size_t frag_major_bytes(int N, int K, int esz) { return (size_t)((N + 15) / 16) * 16 * K * esz; }

}  // namespace mx
