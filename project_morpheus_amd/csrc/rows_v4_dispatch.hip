// Multi-row decode GEMM generation 4: workspace sizing and the dispatcher.
#include "mx_rows_v4.inc"

namespace mx {
namespace v4 {

// Workspace (floats) and tickets a launch of this shape needs (0 when K is one range).
void gemm_rows_workspace_v4(int N, int K, int R, int epi, size_t* ws_floats, size_t* tickets) {
  *ws_floats = 0;
  *tickets = 0;
  for (int cap : {1, 2, 4}) {  // every batch-tile cap option rows_nt_max may pick
    int mt, nt;
    rows_tiles(epi, R, &mt, &nt, cap);
    // the lm_head also runs 32 weight rows per wave (rows_head_mt = 2, batch tiles of 16 / 32)
    for (int m : {1, 2}) {
      if (m == 2 && (epi != EPI_ARGMAX || nt > 2)) continue;
      // the largest split any rows_target option can ask for (nkc grows with the target)
      const int nkc = K % 128 ? 1 : rows_nkc(N, K, R, m, nt, 4096);
      const size_t tn = (N + 128 * m - 1) / (128 * m), tr = (R + 16 * nt - 1) / (16 * nt);
      *ws_floats = std::max(*ws_floats, nkc > 1 ? tn * tr * nkc * (8 * (size_t)m * nt * 4 * 64 + 16 * nt) : (size_t)0);
      *tickets = std::max(*tickets, tn * tr);
    }
    (void)mt;
  }
}

bool rows_merge_ok_v4(const GemvArgs& o) { return rows_merge_ok(o); }

int rows_qkv_nkc_v4(const GemvArgs& a) {
  int mt, nt;
  rows_tiles(EPI_QKV, a.R, &mt, &nt, a.rows_nt_max);
  return a.K % 128 ? 1 : rows_nkc(a.N, a.K, a.R, mt, nt, rows_target_of<EPI_QKV>(a));
}

// R >= 2 rows.  Returns hipErrorNotSupported for shapes the kernel does not cover.
hipError_t launch_gemm_rows_v4(const GemvArgs& a, int epi, bool norm, hipStream_t st) {
  if (a.R < 1) return hipErrorNotSupported;
  int mt, nt;
  rows_tiles(epi, a.R, &mt, &nt, a.rows_nt_max);
  if (epi == EPI_QKV && norm) return launch_rows_qkv(a, nt, st);
  if (epi == EPI_RESID && !norm) return launch_rows_resid(a, nt, st);
  if (epi == EPI_SILU && norm) return launch_rows_silu(a, nt, st);
  return launch_rows_head(a, epi, norm, nt, st);
}

}  // namespace v4
}  // namespace mx
