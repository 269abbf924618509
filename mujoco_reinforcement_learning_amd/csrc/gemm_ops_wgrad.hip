// gemm_wgrad_partial: one instantiation unit of the layered GEMM templates (gemm_ops.h); the four
// entry points compile as separate units so the build runs them in parallel.
#include "gemm_ops.h"

namespace ppo {

int gemm_wgrad_partial(const GemmBatch &gb, int nprob, int max_m, int max_n, hipStream_t st) {
  return run_partial(gb, nprob, max_m, max_n, st);
}

}  // namespace ppo
