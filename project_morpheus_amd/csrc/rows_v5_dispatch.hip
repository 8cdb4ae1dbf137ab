// Multi-row decode GEMM generation 5: the dispatcher (mx_rows_v5.inc).
#include "mx_rows_v5.inc"

namespace mx {
namespace v5 {

// 2 <= R <= 64 rows on the fragment-major weights; hipErrorNotSupported otherwise (the caller
// then takes generation 4: prefill rows, shapes whose K does not split over the waves).
hipError_t launch_gemm_rows_v5(const GemvArgs& a, int epi, bool norm, hipStream_t st) {
  if (a.R < 1 || a.R > 64 || !a.Wf) return hipErrorNotSupported;
  const int nt = a.R <= 16 ? 1 : a.R <= 32 ? 2 : 4;
  if (epi == EPI_QKV && norm) return launch_rows5_qkv(a, nt, st);
  if (epi == EPI_RESID && !norm) return launch_rows5_resid(a, nt, st);
  if (epi == EPI_SILU && norm) return launch_rows5_silu(a, nt, st);
  if (epi == EPI_ARGMAX && norm) return launch_rows5_head(a, nt, st);
  return hipErrorNotSupported;
}

}  // namespace v5
}  // namespace mx
