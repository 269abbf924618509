// gemm_rows_fwd_kn: one instantiation unit of the layered GEMM templates (gemm_ops.h); the four
// entry points compile as separate units so the build runs them in parallel.
#include "gemm_ops.h"

namespace ppo {

int gemm_rows_fwd_kn(const GemmBatch &gb, int nprob, int rows, int max_n, hipStream_t st) {
  return run_rowwise<B_KN, EPI_FWD>(gb, nprob, rows, max_n, st);
}

}  // namespace ppo
