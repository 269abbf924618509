// Per-slice f64 standardisation statistics of one observation row (running_gym_sequential_
// vectorized.py:61-92: mean, unbiased std, std == 0 -> 1), shared by the layered A1 kernel
// (obs_normalize_kernel, O <= 32) and the fused rollout step (policy_fused_kernel), so the two
// produce bit-identical states.  The row sits in 32 registers (slots >= O are zero); each of the
// three sums (x, x - mean, ((x - mean) - cmean)^2) is a fixed pairwise tree over the 32 slots with
// the slots outside the slice zeroed: depth 5 instead of a 32-long dependent f64 chain.  Against
// torch's own (vectorised) summation order the f64 results differ only in rounding, i.e. the f32
// states agree up to rare 1-ulp ties (the bar of test_obs_window_and_normalize).
#pragma once

#include <hip/hip_runtime.h>

namespace ppo {

__device__ __forceinline__ double tree32(double (&v)[32]) {
#pragma unroll
  for (int w = 16; w >= 1; w >>= 1)
#pragma unroll
    for (int i = 0; i < w; ++i) v[i] = v[2 * i] + v[2 * i + 1];
  return v[0];
}

struct SliceStats {
  double mean, sd;
};

// Statistics of slice [lo, hi) (cnt = hi - lo >= 1; cnt == 1 gives sd = NaN, as torch.std).
__device__ __forceinline__ SliceStats slice_stats32(const double (&x)[32], int lo, int hi) {
  const int cnt = hi - lo;
  double t[32];
#pragma unroll
  for (int f = 0; f < 32; ++f) t[f] = (f >= lo && f < hi) ? x[f] : 0.0;
  const double mean = tree32(t) / cnt;
#pragma unroll
  for (int f = 0; f < 32; ++f) t[f] = (f >= lo && f < hi) ? x[f] - mean : 0.0;
  const double cmean = tree32(t) / cnt;
#pragma unroll
  for (int f = 0; f < 32; ++f) {
    const double d = (x[f] - mean) - cmean;
    t[f] = (f >= lo && f < hi) ? d * d : 0.0;
  }
  double sd = sqrt(tree32(t) / (cnt - 1));
  if (sd == 0.0) sd = 1.0;
  return SliceStats{mean, sd};
}

}  // namespace ppo
