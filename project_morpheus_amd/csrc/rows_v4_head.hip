// Multi-row decode GEMM generation 4, EPI_ARGMAX / EPI_STORE instantiations (own translation unit).
#include "mx_rows_v4.inc"

namespace mx {
namespace v4 {

hipError_t launch_rows_head(const GemvArgs& a, int epi, bool norm, int nt, hipStream_t st) {
#define MX_R(EPI_, NORM_)                                                                 \
  if (epi == EPI_ && norm == NORM_) {                                                     \
    if (nt == 1) return launch_rows_k<1, 1, EPI_, NORM_>(a, st);                          \
    if (nt == 2) return launch_rows_k<1, 2, EPI_, NORM_>(a, st);                          \
    return launch_rows_k<1, 4, EPI_, NORM_>(a, st);                                       \
  }
  // rows_head_mt = 2 (option): 32 weight rows per wave (256 per block), so every staged
  // activation sub-chunk feeds twice the lm_head weights.  It won round 4 (-22 us per 32-row
  // bf16 step) only while every wave took its own argmax atomic; with one atomic per block
  // (rows_epilogue) the 16-row waves at 128 VGPRs (two blocks per CU) stream faster: 8 rows
  // 169 -> 150 us bf16, 91 -> 80 us e4m3; 32 rows 185 -> 154 us (profiles/r05_head_options.log)
  if (epi == EPI_ARGMAX && norm && a.rows_head_mt == 2) {
    if (nt == 1) return launch_rows_k<2, 1, EPI_ARGMAX, true>(a, st);
    if (nt == 2) return launch_rows_k<2, 2, EPI_ARGMAX, true>(a, st);
  }
  MX_R(EPI_ARGMAX, true)
  MX_R(EPI_STORE, false)
  MX_R(EPI_STORE, true)
#undef MX_R
  return hipErrorNotSupported;
}

}  // namespace v4
}  // namespace mx
