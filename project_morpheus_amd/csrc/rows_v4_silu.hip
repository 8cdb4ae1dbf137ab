// Multi-row decode GEMM generation 4, EPI_SILU instantiations (own translation unit).
#include "mx_rows_v4.inc"

namespace mx {
namespace v4 {

hipError_t launch_rows_silu(const GemvArgs& a, int nt, hipStream_t st) {
  if (nt == 1) return launch_rows_k<1, 1, EPI_SILU, true>(a, st);
  if (nt == 2) return launch_rows_k<1, 2, EPI_SILU, true>(a, st);
  return launch_rows_k<1, 4, EPI_SILU, true>(a, st);
}

}  // namespace v4
}  // namespace mx
