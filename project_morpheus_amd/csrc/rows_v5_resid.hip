// Multi-row decode GEMM generation 5, EPI_RESID instantiations (own translation unit).
#include "mx_rows_v5.inc"

namespace mx {
namespace v5 {

// o-proj / down: 16-row weight tiles, 192 blocks of 8 waves at Orpheus width
hipError_t launch_rows5_resid(const GemvArgs& a, int nt, hipStream_t st) {
  const int wpb = a.rows5_wpb ? a.rows5_wpb : 8;
  if (nt == 1) return launch5<1, 1, EPI_RESID, false>(a, wpb, st);
  if (nt == 2) return launch5<1, 2, EPI_RESID, false>(a, wpb, st);
  return launch5<1, 4, EPI_RESID, false>(a, wpb, st);
}

}  // namespace v5
}  // namespace mx
