// One-launch decode step for a single row (B = 1): argument block and launcher
// (step_kernels.hip).  See DESIGN.md §5 "Dataflow step".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mx {

constexpr int STEP_SPLIT = 64;       // attention positions per split block
constexpr int STEP_CS = 32;          // ints between two counters (one 128-byte line each)
constexpr int STEP_LAYER_CNT = 48;   // counters per layer (see step_kernels.hip)
constexpr int STEP_BEST = 64;        // argmax shards of the lm_head stage
constexpr int STEP_PART = 130;       // floats per (split, head) partial: acc[128], m, l

struct StepArgs {
  // weights, every layer's matrix of one kind contiguous (packed row order, capi.hip)
  const void *wqkv, *wo, *wgu, *wd, *lm;
  const float *sqkv, *so, *sgu, *sd, *slm;  // fp8 row scales (null for bf16)
  const float *attn_norm, *mlp_norm, *norm;  // [L][H], [L][H], [H]
  const uint16_t* embed;                     // bf16 [V][H] (next-token gather)
  const float *rope_cos, *rope_sin;          // [max_pos][64]
  uint16_t *kcache, *vcache;                 // [L][slots][kvh][max_pos * 128], fragment-major chunks
  size_t kv_layer_elems;
  // row / slot state (row 0)
  int32_t *row_slot, *row_pos, *row_token;
  uint8_t* seen;                             // [slots][V]
  int32_t* hist;                             // host-mapped [slots][max_pos]
  const float *penalty, *samp_temp;          // per slot
  float* logits;                             // [V] kept for sampling rows (or logits_all)
  int logits_all;
  unsigned long long* best;                  // [1]: argmax key for the sampler (commit = 0)
  unsigned long long* best_sh;               // [STEP_BEST] shards, zero between launches
  float* h;                                  // h_dec [H]: step input; next embedding out
  // hand-off buffers: each element written at most once per launch
  float *hd, *ho;                            // [L][H] residual after the MLP / attention
  float *q, *knew, *vnew;                    // [L][heads*128], [L][kvh*128] (bf16-rounded)
  float* part;                               // [L][kvh][split_max][GRP][STEP_PART]
  float* att;                                // [L][heads*128]
  float* act;                                // [L][F]
  int* cnt;                                  // counters, zero between launches
  int* status;                               // device: first give-up code (sticky)
  int* status_host;                          // host-mapped copy written by the finish block
  int H, F, heads, kvh, V, layers, max_pos, nsplit, split_max, scratch_slot;
  float eps, att_scale;
  int commit;                                // 1: finish commits the argmax (greedy row)
  unsigned long long* trace;                 // diagnostic: [blocks][4] timestamps (null: off)
  int64_t block0;                            // global role index of this launch's block 0
};

// Blocks of the launch: layers * (qkv + attention + o + gate/up + down) + lm_head + 1.
int64_t step_blocks(const StepArgs& a);
size_t step_counter_ints(int layers);
// hipErrorNotSupported when the shape has no instantiation (the caller keeps the per-kernel
// step); the launch itself is asynchronous on `st`.
hipError_t launch_step(const StepArgs& a, bool f8, hipStream_t st);
// The same step cut into several launches (stream-ordered, same roles and counters): a layer's
// stages are qkv 0, attention 1, o-proj 2, gate/up 3, down 4; bit s of `cuts` starts a new
// launch at stage s of every layer (bit 0 is implied), and the lm_head + finish blocks are one
// more launch.  Blocks still wait only on lower role indices, now possibly in an earlier launch.
hipError_t launch_step_cut(const StepArgs& a, bool f8, int cuts, hipStream_t st);
bool step_supported(int H, int F, int heads, int kvh, bool f8);

}  // namespace mx
