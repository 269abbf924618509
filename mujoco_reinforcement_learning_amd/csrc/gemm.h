// The f32 / bf16 MFMA GEMM templates of the layered engine (mlp_engine.hip) and their host-side
// launch helpers, shared with the BiLSTM feature extractor (bilstm.hip).
//
//   FWD      C = act(A B^T + bias)            A [rows][k] (A_MK), B [n][k] (B_NK) or [k][n] (B_KN)
//   DX       C = (A B) * act'(aux)            A [rows][k], B [k][n] (B_KN)
//   PARTIAL  slab[split] = A^T B over a k (= row) range, + column sums of A (bias gradients)
// f32: v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulate); bf16 (precision mode
// PPO_PREC_BF16): operands rounded to bf16 as they are staged, v_mfma_f32_32x32x16_bf16.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "timing.h"

namespace ppo {

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { A_MK = 0, A_KM = 1 };
enum { B_NK = 0, B_KN = 1 };
enum { EPI_FWD = 0, EPI_DX = 1, EPI_PARTIAL = 2 };

struct GemmProblem {
  const float *a;
  int64_t lda;
  const float *b;
  int64_t ldb;
  float *c;
  int64_t ldc;
  const float *bias;   // EPI_FWD, nullable
  const float *aux;    // EPI_DX: layer input activations (same layout as c; c may alias it)
  const __bf16 *aux16; // EPI_DX, bf16 kernel, nullable: the activations as bf16 instead of aux
                       // (a ReLU net's: act'(y) depends only on the sign, which RNE keeps)
  float *colsum;       // EPI_PARTIAL: bias-gradient slab base, nullable
  float *colsum2;      // bf16 kernel: a second slab base receiving the same column sums, nullable
  int m, n;
  // bf16 mode: the operand already bf16 in global memory (then a / b are unused), nullable
  const __bf16 *a16, *b16;
};

struct GemmBatch {
  GemmProblem p[2];
  int k;                   // reduction length (EPI_PARTIAL: rows)
  const int32_t *rows_n;   // device row count: M for FWD/DX, K for PARTIAL (nullable)
  int act;
  int splits;              // EPI_PARTIAL
  int64_t slab_stride;     // EPI_PARTIAL: floats between split slabs
  int prec;                // PPO_PREC_F32 / PPO_PREC_BF16 (host-side dispatch only)
};

// XCD-aware tile order (cdna_hip_programming.md T1).  Workgroups are dealt round-robin to the
// 8 XCDs (b % 8 names the XCD group), each with its own L2.  When a problem's tile count is a
// multiple of 8, block b works on logical tile (b % 8) * (tiles / 8) + b / 8 (row-major over
// (tile_m, tile_n)): every XCD owns one contiguous run of row tiles with all their column tiles,
// so an A row panel is fetched into one L2 and reused there, instead of once per XCD.  Other
// tile counts keep the identity order.  Blocks beyond the problem's tiles return.
constexpr int kXcds = 8;
__device__ __forceinline__ bool xcd_tile(int b, int tiles_m, int tiles_n, int &tile_m,
                                         int &tile_n) {
  const int tiles = tiles_m * tiles_n;
  if (b >= tiles) return false;
  const int id = (tiles % kXcds == 0) ? (b % kXcds) * (tiles / kXcds) + b / kXcds : b;
  tile_m = id / tiles_n;
  tile_n = id - tile_m * tiles_n;
  return true;
}

// One operand's share of a k-tile: NV vectors of V floats per thread, staged in registers.
// KC: the stored rows run along k ([rows][k], transposed on the LDS store); otherwise they run
// along the tile dimension ([k][rows]).  load(): bounds-checked, out-of-range elements load as
// zero; load_full(): the tile is known interior, no checks.  V = 4 requires 16-B aligned rows
// (ld % 4 == 0, aligned base).
template <int R, int BK, int NT, int V, bool KC>
struct OperandTile {
  static constexpr int NV = R * BK / (NT * V);
  static_assert((R * BK) % (NT * V) == 0, "tile/thread mismatch");
  float v[NV][V];

  __device__ __forceinline__ static void coords(int e, int &rr, int &kk) {
    if (KC) {
      kk = (e % (BK / V)) * V;
      rr = e / (BK / V);
    } else {
      rr = (e % (R / V)) * V;
      kk = e / (R / V);
    }
  }
  __device__ __forceinline__ static void span(const float *src, int first, int lim,
                                              float (&out)[V]) {
    if (V == 4 && first + 3 < lim) {
      const float4 x = *reinterpret_cast<const float4 *>(src);
      out[0] = x.x;
      out[1 % V] = x.y;
      out[2 % V] = x.z;
      out[3 % V] = x.w;
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) out[j] = (first + j < lim) ? src[j] : 0.f;
    }
  }
  __device__ __forceinline__ void load_full(const float *base, int64_t ld, int r0, int k0,
                                            int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int rr, kk;
      coords(tid + i * NT, rr, kk);
      const float *src = KC ? base + static_cast<int64_t>(r0 + rr) * ld + (k0 + kk)
                            : base + static_cast<int64_t>(k0 + kk) * ld + (r0 + rr);
      if (V == 4) {
        const float4 x = *reinterpret_cast<const float4 *>(src);
        v[i][0] = x.x;
        v[i][1 % V] = x.y;
        v[i][2 % V] = x.z;
        v[i][3 % V] = x.w;
      } else {
        v[i][0] = src[0];
      }
    }
  }
  __device__ __forceinline__ void load(const float *base, int64_t ld, int r0, int rlim, int k0,
                                       int kend, int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int rr, kk;
      coords(tid + i * NT, rr, kk);
      const int gr = r0 + rr, gk = k0 + kk;
      const bool ok = KC ? (gr < rlim) : (gk < kend);
      if (ok) {
        const int64_t row = KC ? gr : gk;
        if (KC) span(base + row * ld + gk, gk, kend, v[i]);
        else span(base + row * ld + gr, gr, rlim, v[i]);
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) v[i][j] = 0.f;
      }
    }
  }
  __device__ __forceinline__ void store(float *s, int stride, int tid) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int rr, kk;
      coords(tid + i * NT, rr, kk);
      if (KC) {
#pragma unroll
        for (int j = 0; j < V; ++j) s[(kk + j) * stride + rr] = v[i][j];
      } else if (V == 4) {
        *reinterpret_cast<float4 *>(&s[kk * stride + rr]) =
            make_float4(v[i][0], v[i][1 % V], v[i][2 % V], v[i][3 % V]);
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) s[kk * stride + rr + j] = v[i][j];
      }
    }
  }
};

// Epilogue on the 32x32 C map (row = (r&3) + 8*(r>>2) + 4*(lane>>5), col = lane&31), the same
// for the f32 (32x32x2) and bf16 (32x32x16) MFMAs: FWD bias + activation, DX activation
// backward against the layer input (in place), PARTIAL the split's slab.
template <int TM, int TN, int WM, int WN, int EPI>
__device__ __forceinline__ void gemm_epilogue(const f32x16 (&acc)[TM][TN], const GemmProblem &P,
                                              const GemmBatch &gb, int split, int m0, int n0,
                                              int M, int N, int wm, int wn, int lane) {
  constexpr int BM = 32 * TM * WM, BN = 32 * TN * WN;
  float *cbase = P.c + (EPI == EPI_PARTIAL ? static_cast<int64_t>(split) * gb.slab_stride : 0);
  auto emit = [&](auto checked) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + (wn * TN + j) * 32 + (lane & 31);
        float bias = 0.f;
        if (EPI == EPI_FWD && P.bias && (!checked || col < N)) bias = P.bias[col];
        // DX: the block's 16 aux loads first, then the stores -- c may alias aux, so a load after
        // a store waited for it (one memory round trip per element); each lane reads exactly
        // the elements it writes, so the order change is safe under aliasing
        float ax[16];
        if (EPI == EPI_DX) {
          // one branch per block on the operand's width (a per-element select serialised the
          // 16 loads behind it)
          if (P.aux16) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
              ax[r] = (!checked || (row < M && col < N))
                          ? static_cast<float>(P.aux16[static_cast<int64_t>(row) * P.ldc + col])
                          : 0.f;
            }
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
              ax[r] = (!checked || (row < M && col < N)) ? P.aux[static_cast<int64_t>(row) * P.ldc + col]
                                                         : 0.f;
            }
          }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (!checked || (row < M && col < N)) {
            const int64_t off = static_cast<int64_t>(row) * P.ldc + col;
            const float v = acc[i][j][r];
            if (EPI == EPI_FWD) cbase[off] = act_forward(P.bias ? v + bias : v, gb.act);
            else if (EPI == EPI_DX) cbase[off] = act_backward(v, ax[r], gb.act);
            else cbase[off] = v;
          }
        }
      }
    }
  };
  if (m0 + BM <= M && n0 + BN <= N) emit(std::false_type{});
  else emit(std::true_type{});
}

// VA / VB = vector width (1 or 4 floats) of the A / B operand's global loads.
// NBUF = 2: double-buffered LDS, one barrier per k-tile; NBUF = 1: one buffer (half the LDS, more
// blocks per CU), two barriers per k-tile.
template <int TM, int TN, int WM, int WN, int BK, int AMODE, int BMODE, int EPI, int VA, int VB,
          int NBUF>
__global__ __launch_bounds__(64 * WM * WN) void gemm_f32_kernel(GemmBatch gb) {
  constexpr int NT = 64 * WM * WN;
  constexpr int BM = 32 * TM * WM;
  constexpr int BN = 32 * TN * WN;
  // LDS images are [k][m] / [k][n].  A k-contiguous operand is transposed on its store: a row
  // stride == 1 (mod 32) puts the 32 lanes of a store group on 32 distinct banks.  An m/n-
  // contiguous operand is stored as it arrives, 16-B aligned rows for ds_write_b128.
  constexpr int SA = (AMODE == A_MK) ? BM + 1 : BM + 4;
  constexpr int SB = (BMODE == B_NK) ? BN + 1 : BN + 4;
  static_assert(BK % 2 == 0, "BK must be even for 32x32x2");
  __shared__ __attribute__((aligned(16))) float lds[NBUF * BK * (SA + SB)];

  const GemmProblem P = (blockIdx.z == 0) ? gb.p[0] : gb.p[1];
  int M = P.m, N = P.n, K = gb.k;
  if (gb.rows_n) {
    if (EPI == EPI_PARTIAL) K = *gb.rows_n;
    else M = *gb.rows_n;
  }
  int tile_m, tile_n;
  if (!xcd_tile(static_cast<int>(blockIdx.x), (M + BM - 1) / BM, (N + BN - 1) / BN, tile_m, tile_n))
    return;  // uniform per block
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  if (m0 >= M || n0 >= N) return;  // uniform per block
  int kbeg = 0, kend = K;
  const int split = (EPI == EPI_PARTIAL) ? static_cast<int>(blockIdx.y) : 0;
  if (EPI == EPI_PARTIAL) {
    kbeg = static_cast<int>((static_cast<int64_t>(split) * K) / gb.splits);
    kend = static_cast<int>((static_cast<int64_t>(split + 1) * K) / gb.splits);
  }
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;

  OperandTile<BM, BK, NT, VA, AMODE == A_MK> ta;
  OperandTile<BN, BK, NT, VB, BMODE == B_NK> tb;
  auto gload = [&](int k0) {
    // interior tiles (all of these shapes but edge tiles) take the branch-free path
    const bool kfull = k0 + BK <= kend;
    if (kfull && m0 + BM <= M) ta.load_full(P.a, P.lda, m0, k0, tid);
    else ta.load(P.a, P.lda, m0, M, k0, kend, tid);
    if (kfull && n0 + BN <= N) tb.load_full(P.b, P.ldb, n0, k0, tid);
    else tb.load(P.b, P.ldb, n0, N, k0, kend, tid);
  };
  auto lstore = [&](int buf) {
    float *As = lds + buf * BK * (SA + SB);
    ta.store(As, SA, tid);
    tb.store(As + BK * SA, SB, tid);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const bool do_colsum = (EPI == EPI_PARTIAL) && P.colsum && tile_n == 0 && tid < BM;
  float colacc = 0.f;

  const int ntiles = (kend - kbeg + BK - 1) / BK;
  if (ntiles > 0) {
    gload(kbeg);
    lstore(0);
  }
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < ntiles; ++kt) {
    if (kt + 1 < ntiles) gload(kbeg + (kt + 1) * BK);
    const float *As = lds + (NBUF == 2 ? cur : 0) * BK * (SA + SB);
    const float *Bs = As + BK * SA;
    // fragments for k-pair kp+1 are read from LDS while the MFMAs of kp run
    float av[TM], bv[TN];
    auto frag = [&](int kp, float(&a)[TM], float(&b)[TN]) {
      const int kk = 2 * kp + (lane >> 5);
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = As[kk * SA + (wm * TM + i) * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = Bs[kk * SB + (wn * TN + j) * 32 + (lane & 31)];
    };
    frag(0, av, bv);
#pragma unroll
    for (int kp = 0; kp < BK / 2; ++kp) {
      float an[TM], bn[TN];
      if (kp + 1 < BK / 2) frag(kp + 1, an, bn);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      if (kp + 1 < BK / 2) {
#pragma unroll
        for (int i = 0; i < TM; ++i) av[i] = an[i];
#pragma unroll
        for (int j = 0; j < TN; ++j) bv[j] = bn[j];
      }
    }
    if (do_colsum) {
      float s = 0.f;
#pragma unroll
      for (int kk = 0; kk < BK; ++kk) s += As[kk * SA + tid];
      colacc += s;
    }
    if (NBUF == 2) {
      if (kt + 1 < ntiles) lstore(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    } else if (kt + 1 < ntiles) {
      __syncthreads();  // every wave is done reading the single buffer
      lstore(0);
      __syncthreads();
    }
  }

  gemm_epilogue<TM, TN, WM, WN, EPI>(acc, P, gb, split, m0, n0, M, N, wm, wn, lane);
  if (do_colsum && m0 + tid < M)
    P.colsum[static_cast<int64_t>(split) * gb.slab_stride + m0 + tid] = colacc;
}

// ============================================================================================
// bf16 GEMM (precision mode PPO_PREC_BF16: bf16 operands, f32 accumulate, f32 in/out in HBM).
// Operands are rounded to bf16 (RNE, v_cvt_pk_bf16_f32) as they are staged into LDS images
// [row][k] with k contiguous and a row stride of BK + 8 bf16 (16 B of padding): the 16-B
// fragment read of mfma_f32_32x32x16_bf16 (lane (r, h) takes k = 8h..8h+7 of row r) from 8
// consecutive rows then lands on 8 distinct 4-bank groups.  The C map and epilogues are the
// f32 kernel's.
// ============================================================================================
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const f32x2 f = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2));
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// One operand's share of a k-tile, staged through registers into a bf16 LDS image.
// KC (global [r][k], k contiguous): image [R][BK + 8] (k contiguous; 16 B of row padding), a
//   unit is 4 consecutive k of one row -> one 8-B store; fragments are 16-B row reads.
// !KC (global [k][r], r contiguous -- activations with k = row, weights [out][in] in dgrad):
//   image [BK][R + 32] stored as it arrives (4 consecutive r of one k -> one 8-B store), and
//   fragments come from ds_read_b64_tr_b16, the gfx950 transposing read (two per fragment).
//   The 32-bf16 row padding makes a 32-lane half's 4 rows x 2 column groups cover all 64 banks.
// V = 4: 16-B global loads (8-B for a bf16 source).  sum4 (optional): f32 per-thread sums of the
// r-group's 4 values over every k this thread staged (bias gradient of the wgrad A operand, before
// bf16 rounding).  SRC16: the operand is already bf16 in global memory (a producer wrote the
// RNE-rounded copy the f32 path would stage): its bits go to the image as loaded.
template <int R, int BK, int NT, int V, bool KC, bool SRC16 = false>
struct StageBF16 {
  static constexpr int NU = R * BK / (4 * NT);
  static_assert((R * BK) % (4 * NT) == 0, "tile/thread mismatch");
  static constexpr int ROW = KC ? BK + 8 : R + 32;  // image row stride (bf16)
  static constexpr int IMAGE = KC ? R * ROW : BK * ROW;
  using Src = typename std::conditional<SRC16, __bf16, float>::type;
  float v[SRC16 ? 1 : NU][4];
  uint2 raw[SRC16 ? NU : 1];  // SRC16: 4 bf16 per unit

  __device__ __forceinline__ static void coords(int e, int &rr, int &kk) {
    if (KC) {
      kk = (e % (BK / 4)) * 4;
      rr = e / (BK / 4);
    } else {
      rr = (e % (R / 4)) * 4;
      kk = e / (R / 4);
    }
  }
  // 4 consecutive floats of one global row starting at column `first` (limit `lim`)
  __device__ __forceinline__ static void quad(const float *src, int first, int lim, bool full,
                                              float *out) {
    if (V == 4 && (full || first + 3 < lim)) {
      const float4 x = *reinterpret_cast<const float4 *>(src);
      out[0] = x.x, out[1] = x.y, out[2] = x.z, out[3] = x.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) out[j] = (full || first + j < lim) ? src[j] : 0.f;
    }
  }
  // 4 consecutive bf16 of one global row starting at column `first` (limit `lim`), zero past it
  __device__ __forceinline__ static uint2 quad16(const __bf16 *src, int first, int lim, bool full) {
    if (V == 4 && (full || first + 3 < lim)) return *reinterpret_cast<const uint2 *>(src);
    const uint16_t *s16 = reinterpret_cast<const uint16_t *>(src);
    uint32_t h[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) h[j] = (full || first + j < lim) ? s16[j] : 0u;
    return make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
  }
  template <bool FULL>
  __device__ __forceinline__ void load(const Src *base, int64_t ld, int r0, int rlim, int k0,
                                       int kend, int tid) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      int rr, kk;
      coords(tid + u * NT, rr, kk);
      const int gr = r0 + rr, gk = k0 + kk;
      if constexpr (SRC16) {
        const bool in = KC ? (FULL || gr < rlim) : (FULL || gk < kend);
        raw[u] = !in ? make_uint2(0u, 0u)
                     : KC ? quad16(base + static_cast<int64_t>(gr) * ld + gk, gk, kend, FULL)
                          : quad16(base + static_cast<int64_t>(gk) * ld + gr, gr, rlim, FULL);
        continue;
      } else if (KC) {
        if (FULL || gr < rlim) quad(base + static_cast<int64_t>(gr) * ld + gk, gk, kend, FULL, v[u]);
        else
#pragma unroll
          for (int j = 0; j < 4; ++j) v[u][j] = 0.f;
      } else {
        if (FULL || gk < kend) quad(base + static_cast<int64_t>(gk) * ld + gr, gr, rlim, FULL, v[u]);
        else
#pragma unroll
          for (int j = 0; j < 4; ++j) v[u][j] = 0.f;
      }
    }
  }
  __device__ __forceinline__ void sum4(float (&acc)[4]) const {  // !KC: rr is fixed per thread
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      if constexpr (SRC16) {  // bf16 -> f32 is exact: the sums of the values the MFMAs consume
        acc[0] += __uint_as_float(raw[u].x << 16);
        acc[1] += __uint_as_float(raw[u].x & 0xffff0000u);
        acc[2] += __uint_as_float(raw[u].y << 16);
        acc[3] += __uint_as_float(raw[u].y & 0xffff0000u);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += v[u][j];
      }
    }
  }
  __device__ __forceinline__ void store(__bf16 *s, int tid) const {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      int rr, kk;
      coords(tid + u * NT, rr, kk);
      __bf16 *dst = KC ? s + rr * ROW + kk : s + kk * ROW + rr;
      if constexpr (SRC16)
        *reinterpret_cast<uint2 *>(dst) = raw[u];
      else
        *reinterpret_cast<uint2 *>(dst) =
            make_uint2(pack_bf16x2(v[u][0], v[u][1]), pack_bf16x2(v[u][2], v[u][3]));
    }
  }
  // MFMA 32x32x16 operand fragment of the 32-row block at tile-local row r0, k-step ks:
  // lane (r = lane&31, h = lane>>5) gets rows r0 + r, k = 16ks + 8h .. +7.
  __device__ __forceinline__ static bf16x8 frag(const __bf16 *img, int r0, int ks, int lane) {
    if (KC)
      return *reinterpret_cast<const bf16x8 *>(img + (r0 + (lane & 31)) * ROW + 16 * ks +
                                               8 * (lane >> 5));
    // ds_read_b64_tr_b16: in each 16-lane group g, lane 4q+p addresses row q of a 4 x 16 block
    // (columns 4p..4p+3) and lane i receives column i of the 4 rows.  Group g covers
    // r = 16(g&1) + i and k = 8(g>>1) + {0..3 | 4..7}.
    const int i = lane & 15, g = lane >> 4;
    const __bf16 *a = img + (16 * ks + 8 * (g >> 1) + (i >> 2)) * ROW + r0 + 16 * (g & 1) +
                      4 * (i & 3);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(a));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(a + 4 * ROW));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 w = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, w);
  }
};

template <int TM, int TN, int WM, int WN, int BK, int AMODE, int BMODE, int EPI, int VA, int VB,
          bool A16 = false, bool B16 = false>
__global__ __launch_bounds__(64 * WM * WN) void gemm_bf16_kernel(GemmBatch gb) {
  constexpr int NT = 64 * WM * WN;
  constexpr int BM = 32 * TM * WM;
  constexpr int BN = 32 * TN * WN;
  static_assert(BK % 16 == 0, "BK must be a multiple of 16 for 32x32x16");
  using StA = StageBF16<BM, BK, NT, VA, AMODE == A_MK, A16>;
  using StB = StageBF16<BN, BK, NT, VB, BMODE == B_NK, B16>;
  constexpr int IMG = StA::IMAGE + StB::IMAGE;
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * IMG];

  const GemmProblem P = (blockIdx.z == 0) ? gb.p[0] : gb.p[1];
  int M = P.m, N = P.n, K = gb.k;
  if (gb.rows_n) {
    if (EPI == EPI_PARTIAL) K = *gb.rows_n;
    else M = *gb.rows_n;
  }
  int tile_m, tile_n, split = 0;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  if (EPI == EPI_PARTIAL && gb.splits % kXcds == 0) {
    // split-K weight gradients: every tile of a split on one XCD (workgroups are dealt to the
    // XCDs by linear id mod 8), so the split's k-rows of both operands are fetched into one L2
    // and reused by all its tiles instead of once per XCD holding one of them
    const int X = static_cast<int>(gridDim.x);
    const int lin = static_cast<int>(blockIdx.x) + X * static_cast<int>(blockIdx.y);
    const int j = lin / kXcds;
    split = lin % kXcds + kXcds * (j / X);
    const int id = j % X;
    if (id >= tiles_m * tiles_n) return;  // uniform per block
    tile_m = id / tiles_n;
    tile_n = id - tile_m * tiles_n;
  } else {
    if (!xcd_tile(static_cast<int>(blockIdx.x), tiles_m, tiles_n, tile_m, tile_n))
      return;  // uniform per block
    if (EPI == EPI_PARTIAL) split = static_cast<int>(blockIdx.y);
  }
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  if (m0 >= M || n0 >= N) return;  // uniform per block
  int kbeg = 0, kend = K;
  if (EPI == EPI_PARTIAL) {
    kbeg = static_cast<int>((static_cast<int64_t>(split) * K) / gb.splits);
    kend = static_cast<int>((static_cast<int64_t>(split + 1) * K) / gb.splits);
  }
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;

  StA ta;
  StB tb;
  const typename StA::Src *pa;
  const typename StB::Src *pb;
  if constexpr (A16) pa = P.a16; else pa = P.a;
  if constexpr (B16) pb = P.b16; else pb = P.b;
  auto gload = [&](int k0) {
    const bool kfull = k0 + BK <= kend;
    if (kfull && m0 + BM <= M) ta.template load<true>(pa, P.lda, m0, M, k0, kend, tid);
    else ta.template load<false>(pa, P.lda, m0, M, k0, kend, tid);
    if (kfull && n0 + BN <= N) tb.template load<true>(pb, P.ldb, n0, N, k0, kend, tid);
    else tb.template load<false>(pb, P.ldb, n0, N, k0, kend, tid);
  };
  auto lstore = [&](int buf) {
    __bf16 *As = lds + buf * IMG;
    ta.store(As, tid);
    tb.store(As + StA::IMAGE, tid);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // bias gradient of the wgrad A operand (A_KM: dY, k = rows): every thread keeps f32 sums of
  // its fixed 4-column group over the k it stages (before bf16 rounding), combined in a fixed
  // order through LDS after the k loop
  constexpr bool COLSUM = (EPI == EPI_PARTIAL) && AMODE == A_KM;
  const bool do_colsum = COLSUM && P.colsum && tile_n == 0;
  float csum[4] = {0.f, 0.f, 0.f, 0.f};

  const int ntiles = (kend - kbeg + BK - 1) / BK;
  if (ntiles > 0) {
    gload(kbeg);
    if (COLSUM) ta.sum4(csum);
    lstore(0);
  }
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < ntiles; ++kt) {
    if (kt + 1 < ntiles) gload(kbeg + (kt + 1) * BK);
    const __bf16 *As = lds + cur * IMG;
    const __bf16 *Bs = As + StA::IMAGE;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = StA::frag(As, (wm * TM + i) * 32, ks, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bv[j] = StB::frag(Bs, (wn * TN + j) * 32, ks, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < ntiles) {
      if (COLSUM) ta.sum4(csum);
      lstore(cur ^ 1);
    }
    __syncthreads();
    cur ^= 1;
  }
  gemm_epilogue<TM, TN, WM, WN, EPI>(acc, P, gb, split, m0, n0, M, N, wm, wn, lane);
  if constexpr (COLSUM) {
    // thread t holds columns 4*(t % (BM/4)) .. +3 for k-offsets t / (BM/4) (+ NT/(BM/4) * u):
    // fold the NT/(BM/4) partials per column group in index order
    constexpr int G = BM / 4, PARTS = NT / G;
    static_assert(NT % G == 0, "colsum layout");
    float *red = reinterpret_cast<float *>(lds);  // the k loop is over (trailing barrier)
    if (do_colsum) {
      const int grp = tid % G, part = tid / G;
#pragma unroll
      for (int j = 0; j < 4; ++j) red[part * BM + 4 * grp + j] = csum[j];
    }
    __syncthreads();
    if (do_colsum && tid < BM && m0 + tid < M) {
      float s = 0.f;
      for (int q = 0; q < PARTS; ++q) s += red[q * BM + tid];
      P.colsum[static_cast<int64_t>(split) * gb.slab_stride + m0 + tid] = s;
      if (P.colsum2) P.colsum2[static_cast<int64_t>(split) * gb.slab_stride + m0 + tid] = s;
    }
  }
}

// ============================================================================================
// Host-side launch helpers
// ============================================================================================
static double gemm_flops(const GemmBatch &gb, int nprob, int epi) {
  double f = 0;
  for (int i = 0; i < nprob; ++i) {
    const GemmProblem &p = gb.p[i];
    const double k = (epi == EPI_PARTIAL) ? gb.k : gb.k;
    f += 2.0 * p.m * p.n * k;
  }
  return f;
}

constexpr int kGemmBK = 32;

// float4 loads need every row of the operand 16-B aligned: ld % 4 == 0 and a 16-B aligned base.
static bool vec4_ok(const GemmBatch &gb, int nprob, bool operand_a) {
  for (int i = 0; i < nprob; ++i) {
    const GemmProblem &p = gb.p[i];
    const int64_t ld = operand_a ? p.lda : p.ldb;
    const void *base = operand_a ? static_cast<const void *>(p.a) : static_cast<const void *>(p.b);
    if (ld % 4 || reinterpret_cast<uintptr_t>(base) % 16) return false;
  }
  return true;
}

template <int TM, int TN, int WM, int WN, int AMODE, int BMODE, int EPI, int NBUF, int VA, int VB>
static void launch_gemm_v(const GemmBatch &gb, int nprob, dim3 grid, hipStream_t st) {
  TimRec rec{EPI == EPI_FWD ? KC_GEMM_FWD : (EPI == EPI_DX ? KC_GEMM_DGRAD : KC_GEMM_WGRAD),
             nullptr, 0.0, 0.0};
  if (tim_active()) {
    rec.name = intern_name("gemm_f32_kernel<%d, %d, %d, %d, %d, %d, %d, %d, %d, %d, %d>", TM, TN,
                           WM, WN, kGemmBK, AMODE, BMODE, EPI, VA, VB, NBUF);
    rec.flops = gemm_flops(gb, nprob, EPI);
    for (int i = 0; i < nprob; ++i) {  // algorithmic: A + B read once, C written once (f32)
      const GemmProblem &p = gb.p[i];
      rec.bytes += 4.0 * (static_cast<double>(p.m) * gb.k + static_cast<double>(gb.k) * p.n +
                          static_cast<double>(p.m) * p.n * (EPI == EPI_DX ? 2 : 1));
    }
  }
  launch_k(rec, gemm_f32_kernel<TM, TN, WM, WN, kGemmBK, AMODE, BMODE, EPI, VA, VB, NBUF>, grid,
           dim3(64 * WM * WN), 0, st, gb);
}

constexpr int kGemmBKBf16 = 64;

template <int TM, int TN, int WM, int WN, int AMODE, int BMODE, int EPI, int VA, int VB,
          bool A16 = false, bool B16 = false>
static void launch_gemm_bf16_v(const GemmBatch &gb, int nprob, dim3 grid, hipStream_t st) {
  TimRec rec{EPI == EPI_FWD ? KC_GEMM_FWD : (EPI == EPI_DX ? KC_GEMM_DGRAD : KC_GEMM_WGRAD),
             nullptr, 0.0, 0.0};
  if (tim_active()) {
    rec.name = (A16 || B16)
                   ? intern_name("gemm_bf16_kernel<%d, %d, %d, %d, %d, %d, %d, %d, %d, %d, %s, %s>",
                                 TM, TN, WM, WN, kGemmBKBf16, AMODE, BMODE, EPI, VA, VB,
                                 A16 ? "true" : "false", B16 ? "true" : "false")
                   : intern_name("gemm_bf16_kernel<%d, %d, %d, %d, %d, %d, %d, %d, %d, %d>", TM, TN,
                                 WM, WN, kGemmBKBf16, AMODE, BMODE, EPI, VA, VB);
    rec.flops = gemm_flops(gb, nprob, EPI);
    // algorithmic: A + B read once (4 B, or 2 B for a bf16 operand), C written once (f32)
    const double ea = A16 ? 2.0 : 4.0, eb = B16 ? 2.0 : 4.0;
    for (int i = 0; i < nprob; ++i) {
      const GemmProblem &p = gb.p[i];
      rec.bytes += ea * static_cast<double>(p.m) * gb.k + eb * static_cast<double>(gb.k) * p.n +
                   4.0 * static_cast<double>(p.m) * p.n * (EPI == EPI_DX ? 2 : 1);
    }
  }
  launch_k(rec, gemm_bf16_kernel<TM, TN, WM, WN, kGemmBKBf16, AMODE, BMODE, EPI, VA, VB, A16, B16>,
           grid, dim3(64 * WM * WN), 0, st, gb);
}

// 8-B vector loads of a bf16 operand: ld % 4 == 0 and an 8-B aligned base, every problem
static bool vec4_ok16(const GemmBatch &gb, int nprob, bool operand_a) {
  for (int i = 0; i < nprob; ++i) {
    const GemmProblem &p = gb.p[i];
    const int64_t ld = operand_a ? p.lda : p.ldb;
    const void *base = operand_a ? static_cast<const void *>(p.a16) : static_cast<const void *>(p.b16);
    if (ld % 4 || reinterpret_cast<uintptr_t>(base) % 8) return false;
  }
  return true;
}

// bf16 operands from global memory (the BiLSTM's dG, h_prev, gathered rows and features, and its
// bf16 weight copy): A alone, A and B, or B alone with an f32 A (FWD, PARTIAL), vector loads for
// the bf16 operands -- the producers keep those buffers 8-B aligned with ld % 4 == 0, which the
// host checks
template <int TM, int TN, int WM, int WN, int AMODE, int BMODE, int EPI>
static int launch_gemm_bf16_src(const GemmBatch &gb, int nprob, dim3 grid, hipStream_t st) {
  const bool a16 = gb.p[0].a16 != nullptr, b16 = gb.p[0].b16 != nullptr;
  for (int i = 1; i < nprob; ++i)
    PPO_REQUIRE((gb.p[i].a16 != nullptr) == a16 && (gb.p[i].b16 != nullptr) == b16,
                "gemm: mixed bf16 / f32 operands in one batch");
  PPO_REQUIRE((!a16 || vec4_ok16(gb, nprob, true)) && (!b16 || vec4_ok16(gb, nprob, false)),
              "gemm: bf16-source operands need 8-B aligned rows (ld %% 4 == 0)");
  // an f32 B operand (weights, or rows of an odd width) may need scalar loads
  const bool vb = b16 || vec4_ok(gb, nprob, false);
  if constexpr (EPI == EPI_DX) {
    PPO_REQUIRE(false, "gemm: no bf16-source DX variant");
  } else {
    if (!a16) {  // f32 A (the wgrad's dY, its column sums taken before rounding), bf16 B
      if (vec4_ok(gb, nprob, true))
        launch_gemm_bf16_v<TM, TN, WM, WN, AMODE, BMODE, EPI, 4, 4, false, true>(gb, nprob, grid, st);
      else
        launch_gemm_bf16_v<TM, TN, WM, WN, AMODE, BMODE, EPI, 1, 4, false, true>(gb, nprob, grid, st);
    } else if (b16)
      launch_gemm_bf16_v<TM, TN, WM, WN, AMODE, BMODE, EPI, 4, 4, true, true>(gb, nprob, grid, st);
    else if (vb)
      launch_gemm_bf16_v<TM, TN, WM, WN, AMODE, BMODE, EPI, 4, 4, true, false>(gb, nprob, grid, st);
    else
      launch_gemm_bf16_v<TM, TN, WM, WN, AMODE, BMODE, EPI, 4, 1, true, false>(gb, nprob, grid, st);
  }
  PPO_LAUNCHED();
  return 0;
}

template <int TM, int TN, int WM, int WN, int AMODE, int BMODE, int EPI, int NBUF = 2>
static int launch_gemm(const GemmBatch &gb, int nprob, int max_m, int max_n, hipStream_t st) {
  constexpr int BM = 32 * TM * WM, BN = 32 * TN * WN;
  const int tiles = ceil_div(max_m, BM) * ceil_div(max_n, BN);
  dim3 grid(tiles, EPI == EPI_PARTIAL ? gb.splits : 1, nprob);
  const bool va = vec4_ok(gb, nprob, true), vb = vec4_ok(gb, nprob, false);
  if (gb.prec == PPO_PREC_BF16) {
    // bf16 operands already in global memory (every problem of the batch alike); compiled for
    // the tiles launch_big / run_rowwise / run_partial pick for them only
    if (gb.p[0].a16 || gb.p[0].b16) {
      constexpr bool tile_ok = (TM == 2 && TN == 1 && WM == 2 && WN == 4) ||
                               (TM == 1 && TN == 1 && WM == 1 && WN == 4) ||
                               (TM == 1 && TN == 1 && WM == 4 && WN == 1);
      if constexpr (tile_ok) {
        return launch_gemm_bf16_src<TM, TN, WM, WN, AMODE, BMODE, EPI>(gb, nprob, grid, st);
      } else {
        PPO_REQUIRE(false, "gemm: no bf16-source variant of the %dx%d tile", BM, BN);
      }
    }
    // the bf16 kernel is always double-buffered; NBUF only selects among the f32 variants
    if (va && vb)
      launch_gemm_bf16_v<TM, TN, WM, WN, AMODE, BMODE, EPI, 4, 4>(gb, nprob, grid, st);
    else if (va)
      launch_gemm_bf16_v<TM, TN, WM, WN, AMODE, BMODE, EPI, 4, 1>(gb, nprob, grid, st);
    else if (vb)
      launch_gemm_bf16_v<TM, TN, WM, WN, AMODE, BMODE, EPI, 1, 4>(gb, nprob, grid, st);
    else
      launch_gemm_bf16_v<TM, TN, WM, WN, AMODE, BMODE, EPI, 1, 1>(gb, nprob, grid, st);
    PPO_LAUNCHED();
    return 0;
  }
  for (int i = 0; i < nprob; ++i)
    PPO_REQUIRE(!gb.p[i].a16 && !gb.p[i].b16, "gemm: bf16 operands need precision bf16");
  if (va && vb)
    launch_gemm_v<TM, TN, WM, WN, AMODE, BMODE, EPI, NBUF, 4, 4>(gb, nprob, grid, st);
  else if (va)
    launch_gemm_v<TM, TN, WM, WN, AMODE, BMODE, EPI, NBUF, 4, 1>(gb, nprob, grid, st);
  else if (vb)
    launch_gemm_v<TM, TN, WM, WN, AMODE, BMODE, EPI, NBUF, 1, 4>(gb, nprob, grid, st);
  else
    launch_gemm_v<TM, TN, WM, WN, AMODE, BMODE, EPI, NBUF, 1, 1>(gb, nprob, grid, st);
  PPO_LAUNCHED();
  return 0;
}

// Experiment knobs for the large-M tiles (read once): PPO_GEMM_NBUF=1|2 LDS buffers,
// PPO_GEMM_WIDE=1 for 128x256 tiles (4 waves, 64x128 per wave).
static int env_knob(const char *name, int dflt) {
  const char *v = getenv(name);
  return v ? atoi(v) : dflt;
}
static const int g_nbuf = env_knob("PPO_GEMM_NBUF", 2);
static const int g_wide = env_knob("PPO_GEMM_WIDE", 0);
// The 128x128 tiles as 8 waves of 64x32 (two waves per SIMD; PPO_GEMM_W8=0: 4 waves of 64x64) --
// the occupancy that paid on the wide path's LDS-DMA GEMMs; measured
// (tools/ab_w8.sh): BiLSTM line +6 %, f32 leg +11 %, pixel CNN +2 %; the GPU parity suite passes
// with either (gpurun r03z / r03z2).
static const int g_w8 = env_knob("PPO_GEMM_W8", 1);

template <int TM, int TN, int WM, int WN, int AMODE, int BMODE, int EPI>
static int launch_big(const GemmBatch &gb, int nprob, int max_m, int max_n, hipStream_t st) {
  if constexpr ((TM == 2 && TN == 2 && WM == 2 && WN == 2) || (TM == 2 && TN == 4 && WM == 2 && WN == 2)) {
    // bf16-source batches take the 8-wave 128x128 tile whatever the experiment knobs say
    if (gb.p[0].a16 || gb.p[0].b16)
      return launch_gemm<2, 1, 2, 4, AMODE, BMODE, EPI, 2>(gb, nprob, max_m, max_n, st);
  }
  if constexpr (TM == 2 && TN == 2 && WM == 2 && WN == 2) {
    if (g_w8) {
      if (g_nbuf == 1)
        return launch_gemm<2, 1, 2, 4, AMODE, BMODE, EPI, 1>(gb, nprob, max_m, max_n, st);
      return launch_gemm<2, 1, 2, 4, AMODE, BMODE, EPI, 2>(gb, nprob, max_m, max_n, st);
    }
  }
  if (g_nbuf == 1)
    return launch_gemm<TM, TN, WM, WN, AMODE, BMODE, EPI, 1>(gb, nprob, max_m, max_n, st);
  return launch_gemm<TM, TN, WM, WN, AMODE, BMODE, EPI, 2>(gb, nprob, max_m, max_n, st);
}

// FWD (A_MK, B_NK) and DX (A_MK, B_KN): rows-major M; big tiles when the row count is large.
template <int BMODE, int EPI>
static int run_rowwise(const GemmBatch &gb, int nprob, int rows, int max_n, hipStream_t st) {
  if (rows >= 8192) {
    if (g_wide && max_n > 128)
      return launch_big<2, 4, 2, 2, A_MK, BMODE, EPI>(gb, nprob, rows, max_n, st);
    return launch_big<2, 2, 2, 2, A_MK, BMODE, EPI>(gb, nprob, rows, max_n, st);
  }
  return launch_gemm<1, 1, 1, 4, A_MK, BMODE, EPI>(gb, nprob, rows, max_n, st);
}

[[maybe_unused]] static int run_partial(const GemmBatch &gb, int nprob, int max_m, int max_n, hipStream_t st) {
  if (max_m <= 32) return launch_gemm<1, 1, 1, 4, A_KM, B_KN, EPI_PARTIAL>(gb, nprob, max_m, max_n, st);
  if (max_n <= 32) return launch_gemm<1, 1, 4, 1, A_KM, B_KN, EPI_PARTIAL>(gb, nprob, max_m, max_n, st);
  return launch_big<2, 2, 2, 2, A_KM, B_KN, EPI_PARTIAL>(gb, nprob, max_m, max_n, st);
}


}  // namespace ppo
