// Host entry of the wide-path GEMMs (instantiated once, in wide_gemm.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace ppo {
namespace wide {

struct WideBatch;

// kind: WK_FWD / WK_DGRAD / WK_F32 / WK_WGRAD; max_m, max_n: the largest problem's extents (grid
// size); kflops: WGRAD's row count for the timing record's FLOPs (the device count may be lower)
int run(int kind, const WideBatch &wb, int nprob, int max_m, int max_n, int kflops,
        hipStream_t st);
// row-tile height run() uses for this kind and shape (colsum partial rows = ceil(m / row_tile))
int row_tile(int kind, int max_m, int max_n);

}  // namespace wide
}  // namespace ppo
