// The single instantiation of the wide-path GEMM templates (wide_gemm.h) and their launch helper,
// plus ppo_wide_gemm: the same launches on caller buffers (kernel-level parity tests, tuning).
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "wide_gemm.h"
#include "wide_ops.h"

namespace ppo {
namespace wide {

template <int TM, int TN, int WM, int WN, int KIND, int NS>
static int launch_cfg(const WideBatch &wb, int nprob, int max_m, int max_n, int kflops,
                      hipStream_t st) {
  using C = WideCfg<TM, TN, WM, WN, KIND, NS>;
  const int tiles = ceil_div(max_m, C::BM) * ceil_div(max_n, C::BN);
  const dim3 grid(KIND == WK_WGRAD ? tiles * wb.splits : tiles, 1, nprob);  // WGRAD: (split, tile)
  TimRec rec{KIND == WK_FWD || KIND == WK_F32 ? KC_GEMM_FWD
                                              : (KIND == WK_DGRAD ? KC_GEMM_DGRAD : KC_GEMM_WGRAD),
             nullptr, 0.0, 0.0};
  if (tim_active()) {
    rec.name = intern_name("wide_gemm_kernel<%d, %d, %d, %d, %d, %d>", TM, TN, WM, WN, KIND, NS);
    for (int i = 0; i < nprob; ++i) {  // algorithmic: bf16 A + B read once, C written once
      const WideProblem &p = wb.p[i];
      const double k = KIND == WK_WGRAD ? kflops : p.k;
      rec.flops += 2.0 * p.m * p.n * k;
      rec.bytes += 2.0 * (static_cast<double>(p.m) * k + static_cast<double>(p.n) * k) +
                   static_cast<double>(p.m) * p.n *
                       (KIND == WK_FWD ? 2.0 : KIND == WK_DGRAD ? 4.0 : 4.0 * (KIND == WK_WGRAD ? wb.splits : 1));
    }
  }
  launch_k(rec, wide_gemm_kernel<TM, TN, WM, WN, KIND, NS>, grid, dim3(C::NT), 0, st, wb);
  PPO_LAUNCHED();
  return 0;
}

// Tile choice: 128 x 128 (4 waves of 64 x 64) for the minibatch GEMMs, 64 x 64 for rollout-sized
// row counts (enough workgroups to cover the chip), 128 x 32 / 32 x 128 for the heads' narrow
// products.  PPO_WIDE_CFG=<n> forces a tile / stage variant (tools/wide_bench.py sweeps).
template <int KIND>
static int run_kind(const WideBatch &wb, int nprob, int max_m, int max_n, int kflops,
                    hipStream_t st) {
  const char *force = getenv("PPO_WIDE_CFG");
  const int f = force ? atoi(force) : -1;
  if (KIND == WK_WGRAD) {
    if (max_m <= 32) return launch_cfg<1, 1, 1, 4, KIND, 3>(wb, nprob, max_m, max_n, kflops, st);
    switch (f) {  // default: 128 x 128 tiles of 8 waves, two stages, two workgroups per CU
      case 1: return launch_cfg<2, 2, 2, 2, KIND, 2>(wb, nprob, max_m, max_n, kflops, st);
      case 2: return launch_cfg<2, 2, 2, 2, KIND, 4>(wb, nprob, max_m, max_n, kflops, st);
      case 3: return launch_cfg<2, 2, 2, 2, KIND, 3>(wb, nprob, max_m, max_n, kflops, st);
      case 10: return launch_cfg<1, 1, 2, 4, KIND, 2>(wb, nprob, max_m, max_n, kflops, st);
      case 12: return launch_cfg<1, 2, 4, 2, KIND, 2>(wb, nprob, max_m, max_n, kflops, st);
      default: return launch_cfg<2, 1, 2, 4, KIND, 2>(wb, nprob, max_m, max_n, kflops, st);
    }
  }
  // F32 outputs wider than the heads (the BiLSTM's input projection, 4H columns): the
  // minibatch tile
  if (KIND == WK_F32 && max_n > 128 && max_m > 4096)
    return launch_cfg<2, 1, 2, 4, KIND, 2>(wb, nprob, max_m, max_n, kflops, st);
  if (KIND == WK_F32 || (KIND == WK_FWD && max_n <= 32))
    return launch_cfg<1, 1, 4, 1, KIND, 8>(wb, nprob, max_m, max_n, kflops, st);
  if (max_m <= 4096) {
    if (f == 5) return launch_cfg<1, 1, 2, 2, KIND, 4>(wb, nprob, max_m, max_n, kflops, st);
    return launch_cfg<1, 1, 2, 2, KIND, 8>(wb, nprob, max_m, max_n, kflops, st);
  }
  // minibatch-sized rows: 256 x 256 tiles, 8 waves of 128 x 64 (2 waves per SIMD), double-buffered
  // LDS (128 KB) -- twice the MFMA work per byte staged of the 128 x 128 tile, whose operand
  // stream co-limits at the per-CU L2 rate; PPO_WIDE_CFG=3 keeps the 128 x 128 tile for A/B
  // minibatch-sized rows (measured, tools/wide_bench.py at B = 65,536): 128 x 128 tiles of 8 waves
  // (64 x 32 each), two LDS stages -- 64 KB + the aliased 68 KB epilogue tile, so two workgroups
  // (16 waves) per CU keep twice the loads in flight of the 4-wave / 3-stage tile (fwd 66 -> 54 us,
  // dgrad 84 -> 64); the 256 x 256 tile (one 8-wave workgroup per CU) measured as slow as the old one
  switch (f) {  // tuning variants
    case 1: return launch_cfg<2, 2, 2, 2, KIND, 2>(wb, nprob, max_m, max_n, kflops, st);
    case 2: return launch_cfg<2, 2, 2, 2, KIND, 4>(wb, nprob, max_m, max_n, kflops, st);
    case 3: return launch_cfg<2, 2, 2, 2, KIND, 3>(wb, nprob, max_m, max_n, kflops, st);
    case 4:
      if constexpr (KIND != WK_WGRAD) return launch_cfg<4, 2, 2, 4, KIND, 2>(wb, nprob, max_m, max_n, kflops, st);
      else return launch_cfg<2, 1, 2, 4, KIND, 2>(wb, nprob, max_m, max_n, kflops, st);
    case 6: return launch_cfg<2, 2, 4, 2, KIND, 3>(wb, nprob, max_m, max_n, kflops, st);
    case 7: return launch_cfg<2, 1, 2, 4, KIND, 3>(wb, nprob, max_m, max_n, kflops, st);
    case 9: return launch_cfg<1, 1, 2, 2, KIND, 2>(wb, nprob, max_m, max_n, kflops, st);
    case 10: return launch_cfg<1, 1, 2, 4, KIND, 2>(wb, nprob, max_m, max_n, kflops, st);
    case 11: return launch_cfg<2, 1, 4, 4, KIND, 2>(wb, nprob, max_m, max_n, kflops, st);
    case 12: return launch_cfg<1, 2, 4, 2, KIND, 2>(wb, nprob, max_m, max_n, kflops, st);
    default: return launch_cfg<2, 1, 2, 4, KIND, 2>(wb, nprob, max_m, max_n, kflops, st);
  }
}

int run(int kind, const WideBatch &wb, int nprob, int max_m, int max_n, int kflops,
        hipStream_t st) {
  switch (kind) {
    case WK_FWD: return run_kind<WK_FWD>(wb, nprob, max_m, max_n, kflops, st);
    case WK_DGRAD: return run_kind<WK_DGRAD>(wb, nprob, max_m, max_n, kflops, st);
    case WK_F32: return run_kind<WK_F32>(wb, nprob, max_m, max_n, kflops, st);
    case WK_WGRAD: return run_kind<WK_WGRAD>(wb, nprob, max_m, max_n, kflops, st);
    default:
      set_error("wide gemm: unknown kind %d", kind);
      return PPO_EINVAL;
  }
}

int run_pair(const WideBatch &wg, int np_w, int max_m_w, int max_n_w, int kflops,
             const WideBatch &dg, int np_d, int rows_d, int max_n_d, hipStream_t st) {
  // the default tiles of both kinds (run_kind): WGRAD with max_m > 32, DGRAD at minibatch rows
  const bool forced = getenv("PPO_WIDE_CFG") != nullptr || getenv("PPO_WIDE_PAIR0") != nullptr;
  if (forced || np_w != np_d || max_m_w <= 32 || rows_d <= 4096) {
    if (int rc = run(WK_WGRAD, wg, np_w, max_m_w, max_n_w, kflops, st)) return rc;
    return run(WK_DGRAD, dg, np_d, rows_d, max_n_d, 0, st);
  }
  using CW = WideCfg<2, 1, 2, 4, WK_WGRAD, 2>;
  using CD = WideCfg<2, 1, 2, 4, WK_DGRAD, 2>;
  static_assert(CW::NT == CD::NT, "one block size");
  const int wg_blocks = ceil_div(max_m_w, CW::BM) * ceil_div(max_n_w, CW::BN) * wg.splits;
  const int dg_blocks = ceil_div(rows_d, CD::BM) * ceil_div(max_n_d, CD::BN);
  PPO_REQUIRE(wg_blocks % 8 == 0 || wg.splits % 8 != 0, "wide pair: WGRAD grid %d", wg_blocks);
  TimRec rec{KC_GEMM_WGRAD, "wide_pair_kernel<2, 1, 2, 4, 2>", 0.0, 0.0};
  if (tim_active()) {  // both kinds' algorithmic work, as their own launches would count it
    for (int i = 0; i < np_w; ++i) {
      const WideProblem &p = wg.p[i];
      rec.flops += 2.0 * p.m * p.n * kflops;
      rec.bytes += 2.0 * (static_cast<double>(p.m) + p.n) * kflops +
                   4.0 * static_cast<double>(p.m) * p.n * wg.splits;
    }
    for (int i = 0; i < np_d; ++i) {
      const WideProblem &p = dg.p[i];
      rec.flops += 2.0 * p.m * p.n * p.k;
      rec.bytes += 2.0 * (static_cast<double>(p.m) + p.n) * p.k + 4.0 * static_cast<double>(p.m) * p.n;
    }
  }
  launch_k(rec, wide_pair_kernel<2, 1, 2, 4, 2>, dim3(wg_blocks + dg_blocks, 1, np_w), dim3(CW::NT),
           0, st, wg, dg, wg_blocks);
  PPO_LAUNCHED();
  return 0;
}

int row_tile(int kind, int max_m, int max_n) {
  if (kind == WK_F32 || (kind == WK_FWD && max_n <= 32)) return 128;
  if (max_m <= 4096) return 64;
  const char *force = getenv("PPO_WIDE_CFG");
  const int f = force ? atoi(force) : -1;
  if (max_n >= 256 && f == 4) return 256;
  if (f == 9 || f == 10) return 64;
  return f == 11 ? 256 : 128;
}

}  // namespace wide
}  // namespace ppo

using namespace ppo;

extern "C" int ppo_wide_gemm(int kind, int m, int n, int k, const void *a_d, int64_t lda,
                             const void *b_d, int64_t ldb, void *c_d, int64_t ldc,
                             const float *bias_d, const void *aux_d, float *colsum_d, int act,
                             int splits, const int32_t *count_d, void *stream) {
  PPO_REQUIRE(kind >= wide::WK_FWD && kind <= wide::WK_WGRAD, "ppo_wide_gemm: kind %d", kind);
  PPO_REQUIRE(a_d && b_d && c_d && m > 0 && n > 0 && k > 0, "ppo_wide_gemm: bad operands");
  PPO_REQUIRE(kind == wide::WK_WGRAD || k % wide::kBK == 0,
              "ppo_wide_gemm: NT reduction length %d must be a multiple of 64", k);
  PPO_REQUIRE(kind == wide::WK_WGRAD || (n % 8 == 0 && ldc % 8 == 0),
              "ppo_wide_gemm: NT outputs need n %% 8 == 0 and ldc %% 8 == 0");
  PPO_REQUIRE(lda % 8 == 0 && ldb % 8 == 0, "ppo_wide_gemm: operand rows must be 16-B aligned");
  PPO_REQUIRE(kind != wide::WK_DGRAD || aux_d, "ppo_wide_gemm: DGRAD needs aux");
  wide::WideBatch wb{};
  wide::WideProblem &p = wb.p[0];
  p.a = static_cast<const __bf16 *>(a_d);
  p.lda = lda;
  p.b = static_cast<const __bf16 *>(b_d);
  p.ldb = ldb;
  p.c = c_d;
  p.ldc = ldc;
  p.bias = bias_d;
  p.aux = static_cast<const __bf16 *>(aux_d);
  p.colsum = colsum_d;
  p.n_colsum = n;
  p.m = m;
  p.n = n;
  p.k = k;
  p.slab_stride = static_cast<int64_t>(m) * ldc;
  wb.rows_n = count_d;
  wb.act = act;
  wb.splits = std::max(1, splits);
  FreeTimingScope ts;
  return wide::run(kind, wb, 1, m, n, k, as_stream(stream));
}
