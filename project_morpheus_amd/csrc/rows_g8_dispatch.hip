// Multi-row decode GEMM generation 8: planning, workspace sizing, LDS attributes, dispatch.
#include "mx_rows_g8.inc"

namespace mx {
namespace g8 {

hipError_t prepare_g8_qkv();
hipError_t prepare_g8_resid();
hipError_t prepare_g8_silu();

hipError_t prepare() {
  hipError_t e = prepare_g8_qkv();
  if (e == hipSuccess) e = prepare_g8_resid();
  if (e == hipSuccess) e = prepare_g8_silu();
  return e;
}

void workspace(int N, int K, int R, bool f8, size_t* ws_floats, size_t* tickets) {
  *ws_floats = 0;
  *tickets = 0;
  Plan p;
  if (!make_plan(N, K, R, f8, &p)) return;
  const size_t tiles = (size_t)((N + 16 * WPB - 1) / (16 * WPB)) * ((R + 16 * p.nt - 1) / (16 * p.nt));
  if (p.nkc > 1) *ws_floats = tiles * p.nkc * ((size_t)WPB * p.nt * 4 * 64 + 16 * p.nt);
  *tickets = tiles;
}

hipError_t launch(const GemvArgs& a, int epi, bool norm, hipStream_t st) {
  Plan p;
  if (a.R < 2 || !make_plan(a.N, a.K, a.R, a.wdtype == WT_FP8, &p)) return hipErrorNotSupported;
  if (epi == EPI_QKV && norm) return launch_g8_qkv(a, p, st);
  if (epi == EPI_RESID && !norm) return launch_g8_resid(a, p, st);
  if (epi == EPI_SILU && norm) return launch_g8_silu(a, p, st);
  return hipErrorNotSupported;
}

}  // namespace g8
}  // namespace mx
