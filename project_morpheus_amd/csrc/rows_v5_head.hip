// Multi-row decode GEMM generation 5, EPI_ARGMAX instantiations (own translation unit).
#include "mx_rows_v5.inc"

namespace mx {
namespace v5 {

// lm_head + penalty + argmax: 64 weight rows per block (32 above 32 batch rows)
hipError_t launch_rows5_head(const GemvArgs& a, int nt, hipStream_t st) {
  const int wpb = a.rows5_wpb ? a.rows5_wpb : 8;
  if (nt == 1) return launch5<4, 1, EPI_ARGMAX, true>(a, wpb, st);
  if (nt == 2) return launch5<4, 2, EPI_ARGMAX, true>(a, wpb, st);
  if (a.wdtype == WT_FP8) return launch5<1, 4, EPI_ARGMAX, true>(a, wpb, st);
  return launch5<2, 4, EPI_ARGMAX, true>(a, wpb, st);
}

}  // namespace v5
}  // namespace mx
