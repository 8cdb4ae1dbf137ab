// Weight-streaming access-pattern probe (diagnostic, not part of the library).
// Same grid, rows and bytes as the gen-4 gate/up launch at 32 rows (16384 x 3072 bf16,
// 128 row tiles x 2 K ranges, 8 waves x 16 rows per block); only the lane -> address map of
// each 16-byte-per-lane load instruction differs:
//   A: 16 rows x 64 B per instruction (the MFMA A-fragment order gen 4 loads in)
//   B: 4 rows x 256 B per instruction
//   C: 1 row x 1 KB per instruction
// Each wave sums what it loads (no LDS, no MFMA) and stores one word per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int N = 16384, K = 3072, NKC = 2, KR = K / NKC;  // elements
constexpr int ROWB = K * 2;                                 // bytes per row

template <int PAT>
__global__ __launch_bounds__(512) void stream_kernel(const uint4* __restrict__ w, uint32_t* out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 128 + wv * 16;
  const int kb0 = blockIdx.y * KR * 2;  // byte offset of the K range
  const char* base = reinterpret_cast<const char*>(w);
  uint32_t acc = 0;
  constexpr int NI = 16 * KR * 2 / 1024;  // 1 KB instructions per wave (48)
#pragma unroll 8
  for (int i = 0; i < NI; ++i) {
    size_t off;
    if (PAT == 0) {        // instruction i = (sub-chunk s, piece l): row c, 64 B run at 256 s + 64 l + 16 g
      const int c = lane & 15, g = lane >> 4, s = i >> 2, l = i & 3;
      off = (size_t)(n0 + c) * ROWB + kb0 + 256 * s + 64 * l + 16 * g;
    } else if (PAT == 1) { // 4 rows x 256 B: rows 4 (i % 4) + (lane >> 4), 256 B run per row
      const int r = 4 * (i & 3) + (lane >> 4), s = i >> 2;
      off = (size_t)(n0 + r) * ROWB + kb0 + 256 * s + 16 * (lane & 15);
    } else {               // 1 row x 1 KB: row i / 3, KB (i % 3) of the row's range
      const int r = i / 3, q = i % 3;
      off = (size_t)(n0 + r) * ROWB + kb0 + 1024 * q + 16 * lane;
    }
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + off));
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  out[(blockIdx.y * gridDim.x + blockIdx.x) * 512 + threadIdx.x] = acc;
}

template <int PAT>
float run(const uint4* w, uint32_t* out, hipStream_t st) {
  const dim3 grid(N / 128, NKC);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(stream_kernel<PAT>, grid, dim3(512), 0, st, w, out);
  hipEventRecord(e0, st);
  const int reps = 50;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(stream_kernel<PAT>, grid, dim3(512), 0, st, w, out);
  hipEventRecord(e1, st);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.f / reps;
}

int main() {
  // 8 copies so consecutive launches stream different bytes (no Infinity-Cache reuse)
  const size_t bytes = (size_t)N * ROWB;
  const int copies = 8;
  char* w = nullptr;
  uint32_t* out = nullptr;
  if (hipMalloc(&w, bytes * copies) != hipSuccess || hipMalloc(&out, (size_t)N / 128 * NKC * 512 * 4) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(w, 1, bytes * copies);
  hipStream_t st;
  hipStreamCreate(&st);
  for (int round = 0; round < 3; ++round) {
    float us[3];
    // rotate the copy per pattern call through a pointer offset
    us[0] = run<0>(reinterpret_cast<const uint4*>(w + bytes * (round % copies)), out, st);
    us[1] = run<1>(reinterpret_cast<const uint4*>(w + bytes * ((round + 3) % copies)), out, st);
    us[2] = run<2>(reinterpret_cast<const uint4*>(w + bytes * ((round + 5) % copies)), out, st);
    printf("round %d: A 16x64B %.2f us (%.0f GB/s) | B 4x256B %.2f us (%.0f GB/s) | C 1x1KB %.2f us (%.0f GB/s)\n",
           round, us[0], bytes / us[0] / 1e3, us[1], bytes / us[1] / 1e3, us[2], bytes / us[2] / 1e3);
  }
  hipFree(w);
  hipFree(out);
  return 0;
}
