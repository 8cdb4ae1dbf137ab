// Multi-row decode GEMM generation 8, EPI_RESID instantiations (own translation unit).
#include "mx_rows_g8.inc"

namespace mx {
namespace g8 {

hipError_t launch_g8_resid(const GemvArgs& a, const Plan& p, hipStream_t st) {
  if (p.nt == 1) return launch_g8<1, EPI_RESID, false>(a, p, st);
  if (p.nt == 2) return launch_g8<2, EPI_RESID, false>(a, p, st);
  return hipErrorNotSupported;
}

// every instantiation may take up to 72 KB of dynamic LDS
hipError_t prepare_g8_resid() {
  hipError_t e = hipSuccess;
#define MX_P(NT_, SUB_, F8_)                                                                   \
  if (e == hipSuccess && SUB_ <= sub_max(NT_))                                                  \
    e = hipFuncSetAttribute(                                                                    \
        reinterpret_cast<const void*>(&rows8_kernel<NT_, EPI_RESID, false, (SUB_ <= sub_max(NT_) ? SUB_ : 2), F8_, 2>), \
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes(NT_, SUB_));
#define MX_PS(SUB_) MX_P(1, SUB_, false) MX_P(2, SUB_, false) MX_P(1, SUB_, true) MX_P(2, SUB_, true)
  MX_PS(2) MX_PS(3) MX_PS(4) MX_PS(6) MX_PS(8)
#undef MX_PS
#undef MX_P
  return e;
}

}  // namespace g8
}  // namespace mx
