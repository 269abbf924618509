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
// A layer's WGRAD (wg) and DGRAD (dg) as one wide_pair_kernel launch when both take the default
// 128 x 128 tile and the same problem count, else the two run() launches in that order.  The
// caller guarantees dg writes nothing wg reads.
int run_pair(const WideBatch &wg, int np_w, int max_m_w, int max_n_w, int kflops,
             const WideBatch &dg, int np_d, int rows_d, int max_n_d, hipStream_t st);

}  // namespace wide
}  // namespace ppo
