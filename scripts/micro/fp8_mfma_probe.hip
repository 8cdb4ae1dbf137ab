// Probe of the gfx950 scaled fp8 MFMA (v_mfma_scale_f32_16x16x128_f8f6f4) semantics that the
// fp8-MFMA multi-row GEMM relies on: (1) A / B lane layouts are symmetric (lane i + 16 kl holds
// row / column i, 32 k values kl*32 .. +31, byte p <-> k = 32 kl + p), (2) the E8M0 scale
// convention (127 = 2^0; what 0 means), (3) scale_b applies per lane, i.e. per (column, 32-k
// block).  Prints max |gpu - cpu| per case.  Build: hipcc --offload-arch=gfx950 -O2 this -o probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void probe(const uint8_t* A, const uint8_t* B, const int* sa, const int* sb, float* C,
                      int mode) {
  const int lane = threadIdx.x, i = lane & 15, kl = lane >> 4;
  v8i a, b;
  const uint32_t* ap = reinterpret_cast<const uint32_t*>(A + i * 128 + 32 * kl);
  const uint32_t* bp = reinterpret_cast<const uint32_t*>(B + i * 128 + 32 * kl);  // B stored [col][k]
  for (int q = 0; q < 8; ++q) { a[q] = ap[q]; b[q] = bp[q]; }
  v4f c = {0.f, 0.f, 0.f, 0.f};
  if (mode == 0)
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 0, 0, 0);
  else
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa[lane], 0, sb[lane]);
  // D[4 kl + r][i]
  for (int r = 0; r < 4; ++r) C[(4 * kl + r) * 16 + i] = c[r];
}

static float e4m3_to_f(uint8_t v) {
  const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float r;
  if (e == 0) r = std::ldexp((float)m / 8.f, -6);
  else r = std::ldexp(1.f + (float)m / 8.f, e - 7);
  if (e == 15 && m == 7) r = NAN;
  return s ? -r : r;
}

int main() {
  uint8_t hA[16 * 128], hB[16 * 128];
  srand(1);
  for (int n = 0; n < 16 * 128; ++n) {
    uint8_t v;
    do { v = rand() & 0xff; } while (((v >> 3) & 15) == 15 || ((v >> 3) & 15) > 10 || ((v >> 3) & 15) < 4);
    hA[n] = v;
    do { v = rand() & 0xff; } while (((v >> 3) & 15) == 15 || ((v >> 3) & 15) > 10 || ((v >> 3) & 15) < 4);
    hB[n] = v;
  }
  uint8_t *dA, *dB;
  int *dsa, *dsb;
  float* dC;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB);
  hipMalloc(&dsa, 256); hipMalloc(&dsb, 256); hipMalloc(&dC, 16 * 16 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  struct Case { const char* name; int mode; int sa_kind; int sb_kind; };
  // sb_kind: 0 = 127 everywhere, 1 = 127 + (col % 3) - 1 (per column), 2 = 127 + kl - 1
  // (per k block), 3 = constant 0
  const Case cases[] = {{"scales 0/0 (CK unscaled form)", 0, 0, 0},
                        {"scales 127/127", 1, 0, 0},
                        {"scale_b per column 126..128", 1, 0, 1},
                        {"scale_b per k block 126..129", 1, 0, 2},
                        {"scales 0/0 via operands", 1, 3, 3}};
  for (const Case& cs : cases) {
    int hsa[64], hsb[64];
    float wa[64], wb[64];
    for (int l = 0; l < 64; ++l) {
      const int i = l & 15, kl = l >> 4;
      hsa[l] = cs.sa_kind == 3 ? 0 : 127;
      hsb[l] = cs.sb_kind == 3 ? 0 : cs.sb_kind == 1 ? 127 + (i % 3) - 1 : cs.sb_kind == 2 ? 127 + kl - 1 : 127;
      wa[l] = std::ldexp(1.f, hsa[l] - 127);
      wb[l] = std::ldexp(1.f, hsb[l] - 127);
    }
    hipMemcpy(dsa, hsa, 256, hipMemcpyHostToDevice);
    hipMemcpy(dsb, hsb, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC, cs.mode);
    float hC[256];
    hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
    double err_scaled = 0, err_plain = 0, mag = 0;
    for (int r = 0; r < 16; ++r)
      for (int c = 0; c < 16; ++c) {
        double ref = 0, plain = 0;
        for (int k = 0; k < 128; ++k) {
          const int kl = k / 32;
          const double p = (double)e4m3_to_f(hA[r * 128 + k]) * e4m3_to_f(hB[c * 128 + k]);
          plain += p;
          ref += p * wa[r + 16 * kl] * wb[c + 16 * kl];
        }
        err_scaled = fmax(err_scaled, fabs(hC[r * 16 + c] - ref));
        err_plain = fmax(err_plain, fabs(hC[r * 16 + c] - plain));
        mag = fmax(mag, fabs(ref));
      }
    printf("%-34s max|gpu-cpu_scaled| %.3e  max|gpu-cpu_unscaled| %.3e  (max|ref| %.3e)\n", cs.name,
           err_scaled, err_plain, mag);
  }
  return 0;
}
