// The single instantiation of the layered GEMM templates (gemm_ops.h).
#include "gemm_ops.h"

namespace ppo {

int gemm_rows_fwd_nk(const GemmBatch &gb, int nprob, int rows, int max_n, hipStream_t st) {
  return run_rowwise<B_NK, EPI_FWD>(gb, nprob, rows, max_n, st);
}

int gemm_rows_fwd_kn(const GemmBatch &gb, int nprob, int rows, int max_n, hipStream_t st) {
  return run_rowwise<B_KN, EPI_FWD>(gb, nprob, rows, max_n, st);
}

int gemm_rows_dx(const GemmBatch &gb, int nprob, int rows, int max_n, hipStream_t st) {
  return run_rowwise<B_KN, EPI_DX>(gb, nprob, rows, max_n, st);
}

int gemm_wgrad_partial(const GemmBatch &gb, int nprob, int max_m, int max_n, hipStream_t st) {
  return run_partial(gb, nprob, max_m, max_n, st);
}

}  // namespace ppo
