// The layered engine's GEMMs (gemm.h templates) instantiated ONCE, in gemm_ops.hip, and called
// from the MLP engine, the BiLSTM and the pixel encoder's heads through these plain functions:
// every translation unit that instantiated the templates itself paid minutes of compile time.
#pragma once

#include "gemm.h"

namespace ppo {

// C = act(A B^T + bias), A [rows][k], B [n][k] (torch Linear weights)
int gemm_rows_fwd_nk(const GemmBatch &gb, int nprob, int rows, int max_n, hipStream_t st);
// C = act(A B + bias), B [k][n]
int gemm_rows_fwd_kn(const GemmBatch &gb, int nprob, int rows, int max_n, hipStream_t st);
// C = (A B) * act'(aux), B [k][n]
int gemm_rows_dx(const GemmBatch &gb, int nprob, int rows, int max_n, hipStream_t st);
// slab[split] = A^T B over a row range per split (+ column sums of A)
int gemm_wgrad_partial(const GemmBatch &gb, int nprob, int max_m, int max_n, hipStream_t st);

}  // namespace ppo
