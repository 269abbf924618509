// Per-slice f64 standardisation statistics of one observation row (running_gym_sequential_
// vectorized.py:61-92: mean, unbiased std, std == 0 -> 1), shared by the layered A1 kernel
// (obs_normalize_kernel, O <= 32) and the fused rollout step (policy_fused_kernel), so the two
// produce bit-identical states.  The row sits in 32 registers (slots >= O are zero); each of the
// two sums (x, (x - mean)^2) is a fixed pairwise tree over the 32 slots with the slots outside the
// slice zeroed: depth 5 instead of a 32-long dependent f64 chain.  mean = sum * (1/n) and var =
// sum * (1/(n-1)) with the reciprocals taken off the data chain (they depend on the slice width
// only), and no second-pass mean correction: every f64 step stays within ~1 ulp (1e-16) of torch's
// own two-pass f64 std, so the f32 states agree with it up to rare 1-ulp ties (the bar of
// test_obs_window_and_normalize) -- and the rollout step's dependent f64 chain is one butterfly
// and three divides shorter (round 5: 8.8 -> <= 8 us per launch at N = 4096).
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

// Statistics of slice [lo, hi) (cnt = hi - lo >= 1; cnt == 1 gives sd = NaN, as torch.std:
// 0 * (1/0)).
__device__ __forceinline__ SliceStats slice_stats32(const double (&x)[32], int lo, int hi) {
  const int cnt = hi - lo;
  const double inv_n = 1.0 / cnt, inv_n1 = 1.0 / (cnt - 1);
  double t[32];
#pragma unroll
  for (int f = 0; f < 32; ++f) t[f] = (f >= lo && f < hi) ? x[f] : 0.0;
  const double mean = tree32(t) * inv_n;
#pragma unroll
  for (int f = 0; f < 32; ++f) {
    const double d = x[f] - mean;
    t[f] = (f >= lo && f < hi) ? d * d : 0.0;
  }
  double sd = sqrt(tree32(t) * inv_n1);
  if (sd == 0.0) sd = 1.0;
  return SliceStats{mean, sd};
}

// The same statistics with the row spread over 32 lanes (lane = slot, `in` = slot inside the
// slice), two rows per lane interleaved.  tree32's pairwise tree is a butterfly: after level k
// every lane of a 2^k-lane group holds that group's sum (its two halves added in the tree's order
// on the group's first lane, commuted elsewhere: the same value), so any partner lane in the
// sibling group gives the tree's next sum.  Partners on the VALU, no LDS round trips: quad_perm
// xor 1 and xor 2, row_half_mirror (sibling quad), row_ror:8 (sibling 8-lane half of a row), then
// v_permlane16_swap between the 16-lane rows of each 32-lane half (summed as row 0 + row 1: the
// tree's order on every lane).
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(u), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(u >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) |
                                                     static_cast<uint32_t>(lo)));
}
__device__ __forceinline__ double rows16_pair_sum(double v) {  // row0 + row1 of each 32-lane half
  const uint64_t u = __double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane16_swap(static_cast<uint32_t>(u), static_cast<uint32_t>(u), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(static_cast<uint32_t>(u >> 32), static_cast<uint32_t>(u >> 32), false, false);
  const double p0 = __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(hi[0]) << 32) | lo[0]));
  const double p1 = __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(hi[1]) << 32) | lo[1]));
  return p0 + p1;  // row-0 lanes: own + row-1 partner; row-1 lanes: row-0 partner + own
}
__device__ __forceinline__ void butterfly2(double &a, double &b) {
  a = a + dpp_d<0xB1>(a);   // quad_perm [1,0,3,2]
  b = b + dpp_d<0xB1>(b);
  a = a + dpp_d<0x4E>(a);   // quad_perm [2,3,0,1]
  b = b + dpp_d<0x4E>(b);
  a = a + dpp_d<0x141>(a);  // row_half_mirror: the sibling quad
  b = b + dpp_d<0x141>(b);
  a = a + dpp_d<0x128>(a);  // row_ror:8: the other 8 lanes of the row
  b = b + dpp_d<0x128>(b);
  a = rows16_pair_sum(a);
  b = rows16_pair_sum(b);
}

struct SliceStats2 {
  double mean[2], sd[2];
};

__device__ __forceinline__ SliceStats2 slice_stats_lanes(double xa, double xb, bool in, int cnt) {
  SliceStats2 r;
  const double inv_n = 1.0 / cnt, inv_n1 = 1.0 / (cnt - 1);  // off the data chain
  double ta = in ? xa : 0.0, tb = in ? xb : 0.0;
  butterfly2(ta, tb);
  const double ma = ta * inv_n, mb = tb * inv_n;
  const double da = xa - ma, db = xb - mb;
  ta = in ? da * da : 0.0;
  tb = in ? db * db : 0.0;
  butterfly2(ta, tb);
  double sa = sqrt(ta * inv_n1), sb = sqrt(tb * inv_n1);
  if (sa == 0.0) sa = 1.0;
  if (sb == 0.0) sb = 1.0;
  r.mean[0] = ma;
  r.mean[1] = mb;
  r.sd[0] = sa;
  r.sd[1] = sb;
  return r;
}

}  // namespace ppo
