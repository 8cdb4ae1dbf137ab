// Persistent one-row decode engine (engine_b1.hip): arguments and launcher.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mx {

struct EngineArgs {
  // weights, every layer contiguous per kind, packed rows as the one-row GEMVs read them
  const void *wqkv, *wo, *wgu, *wd;
  const float *sqkv, *so, *sgu, *sd;       // e4m3 row scales (f8), per layer contiguous
  const float *attn_norm, *mlp_norm;       // [layers][H]
  const float *rope_cos, *rope_sin;        // [max_pos][64]
  uint16_t *kcache, *vcache;               // layer 0; layer l at + l * kv_layer_elems
  size_t kv_layer_elems;
  const int32_t *row_slot, *row_pos;       // decode row 0
  float* h;                                // decode row 0 hidden state: input and output
  uint2 *g_qkv, *g_att, *g_h1, *g_act, *g_h2;  // hand-off granules {f32 bits, tag}
  float* part;                             // attention split partials [kv][smax][grp][130]
  int* tickets;                            // [layers][kv_heads], zero between launches
  uint32_t* epoch;                         // [0] epoch (>= 1), [1] finished-workgroup ticket
  int* status;                             // host-mapped: 0, or why a launch gave up
  int layers, H, heads, kv_heads, F, max_pos, smax, ring_slots, f8;
  int depth;                               // ring slots in flight per loader wave (2 or 3)
  int loaders;                             // loader waves (1 or 2)
  int xb;                                  // floats of the second staging buffer (engine_xb_floats)
  float eps;
  long long timeout_ticks;                 // 100 MHz realtime ticks per launch
  uint64_t* trace;                         // null, or [grid][layers][12] clock stamps
  int dbg;                                 // timing experiments only: 1 no hand-off waits, 2 no weight DMA
};

int engine_xb_floats(int heads, int kv_heads, int F);
int engine_ring_max();  // ring slots the engine's static LDS holds
size_t engine_lds_bytes(int ring_slots, int H, int xb_floats);
// engine workgroups one CU holds (sets the kernel's dynamic-LDS limit; call outside capture)
hipError_t engine_per_cu(const EngineArgs& a, int* per_cu);
hipError_t launch_engine_b1(const EngineArgs& a, int grid, hipStream_t st);

}  // namespace mx
