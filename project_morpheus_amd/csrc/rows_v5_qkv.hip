// Multi-row decode GEMM generation 5, EPI_QKV instantiations (own translation unit).
#include "mx_rows_v5.inc"

namespace mx {
namespace v5 {

// 16-row weight tiles: 320 blocks at Orpheus width (qkv N = 5120)
hipError_t launch_rows5_qkv(const GemvArgs& a, int nt, hipStream_t st) {
  const int wpb = a.rows5_wpb ? a.rows5_wpb : 4;
  if (nt == 1) return launch5<1, 1, EPI_QKV, true>(a, wpb, st);
  if (nt == 2) return launch5<1, 2, EPI_QKV, true>(a, wpb, st);
  return launch5<1, 4, EPI_QKV, true>(a, wpb, st);
}

}  // namespace v5
}  // namespace mx
