// bf16-resident GEMMs of the wide layered path (nets whose layers the fused kernels do not cover:
// Humanoid 3x512 with O=376, A=17; network_block_creator.py:74-86, ppo.py:109-135).
//
// Activations, pre-activation gradients and weight images live in HBM as bf16, so both operands
// of every product stream straight from HBM/L2 into LDS by LDS-DMA (global_load_lds_dwordx4,
// 16 B per lane) -- no register staging, no f32 -> bf16 conversion in the k-loop, half the bytes
// of the f32 layered path.  v_mfma_f32_32x32x16_bf16, f32 accumulate.
//
//   NT   C[m][n] = sum_k A[m][k] B[n][k]          A [m][k] (activations / gradients, k contiguous),
//                                                 B [n][k] (weight image W, or its transpose W^T)
//        epilogues: FWD   bf16 act(C + bias)          (layer forward)
//                   DGRAD bf16 act'(aux) * C          (input gradient, written over aux) and the
//                                                     f32 column sums of the result per row tile
//                                                     (bias gradient partials)
//                   F32   f32 C (+ bias)              (head pre-activations; the BiLSTM's
//                                                     input projection)
//   TT   slab[split][m][n] = sum_{k in split} A[k][m] B[k][n]   (weight gradient dY^T X, split-K
//                                                 over minibatch rows; both operands k-outer)
//
// LDS images.  NT operands: [R][64] bf16 (128-B rows), 16-B chunk c of row r stored at chunk
// c ^ ((r >> 1) & 7): the A/B fragment read (ds_read_b128, lane -> row r0 + (lane & 31), chunk
// 2ks + (lane >> 5)) hits 16 distinct 16-B bank slots in every 16-lane group.  TT operands:
// [64][R] bf16 read with ds_read_b64_tr_b16 (the gfx950 transposing read); chunk c of k-row kr
// stored at c ^ swz(kr) so that the 4 k-rows x 64 B of a 32-lane read cover all 64 banks.  LDS-DMA
// writes a wave-instruction's 1 KB linearly, so the swizzle is applied to the per-lane GLOBAL
// source address (the source and read permutations are the same involution).
//
// Epilogue: the accumulator tile goes to LDS as f32 (the staging buffers are dead by then) and
// every thread then owns 8 consecutive columns of a set of rows: 16-B bf16 stores / 32-B f32
// stores, coalesced per row, the bias / aux vectors loaded once per thread.  Column sums run over
// the LDS tile in row order (bitwise reproducible).
//
// Row padding contract (host side, wide path allocator): every row buffer has at least
// round_up(rows, 128) rows and its k extent rounded up to 64 (zero filled); rows at or past the
// device row count are WRITTEN AS ZERO by FWD / DGRAD / the gather, so a TT k-loop may run over
// round_up(count, 64) rows.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"
#include "timing.h"

namespace ppo {
namespace wide {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int kBK = 64;
constexpr int kRowPad = 128;  // row buffers are padded to a multiple of this many rows

enum { WK_FWD = 0, WK_DGRAD = 1, WK_F32 = 2, WK_WGRAD = 3 };

struct WideProblem {
  const __bf16 *a;
  int64_t lda;
  const __bf16 *b;
  int64_t ldb;
  void *c;              // bf16 (FWD, DGRAD) or f32 (F32; WGRAD: slab of split 0)
  int64_t ldc;
  const float *bias;    // FWD, nullable
  const __bf16 *aux;    // DGRAD: the layer's output activations (same layout as c; c may alias)
  float *colsum;        // DGRAD: column sums per row tile, [tile_m][n] with row stride n_colsum
  int64_t n_colsum;
  int m, n, k;          // m, n: extents (m: row upper bound); k: NT reduction (multiple of 64)
  int64_t slab_stride;  // WGRAD: floats between split slabs
  // WGRAD, nullable: per split, the column sums of A over the split's k rows (the bias gradient
  // of a dY^T X product), at acol[split * slab_stride + m]; acol2 receives the same values
  float *acol, *acol2;
};

struct WideBatch {
  WideProblem p[2];
  const int32_t *rows_n;  // device row count (NT: m; WGRAD: the k extent), nullable
  int act;
  int splits;             // WGRAD
};

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  const f2 f = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, b2));
}

__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// ---- NT operand: [R][64] image, R/8 LDS-DMA wave-instructions per k-tile ---------------------
template <int R, int NW>
struct RowImage {
  static constexpr int BYTES = R * kBK * 2;
  static constexpr int NINST = R / 8;  // 1 KB each: 8 rows of 128 B
  static_assert(R % 32 == 0, "row tile");
  // issue this wave's share of the fill of k-tile k0 (global rows r0.., src row stride ld)
  __device__ __forceinline__ static void fill(__bf16 *img, const __bf16 *src, int64_t ld, int k0,
                                              int wid, int lane) {
#pragma unroll
    for (int j = 0; j < (NINST + NW - 1) / NW; ++j) {
      const int i = wid + NW * j;
      if (NINST % NW == 0 || i < NINST) {
        const int row = 8 * i + (lane >> 3);
        const int lc = (lane & 7) ^ ((row >> 1) & 7);
        const __bf16 *g = src + static_cast<int64_t>(row) * ld + k0 + 8 * lc;
        __builtin_amdgcn_global_load_lds(g, (lds_void *)(img + 512 * i), 16, 0, 0);
      }
    }
  }
  // MFMA 32x32x16 fragment: lane -> row r0 + (lane & 31), k = 16 ks + 8 (lane >> 5) .. +7
  __device__ __forceinline__ static bf16x8 frag(const __bf16 *img, int r0, int ks, int lane) {
    const int row = r0 + (lane & 31);
    const int pc = (2 * ks + (lane >> 5)) ^ ((row >> 1) & 7);
    return *reinterpret_cast<const bf16x8 *>(img + row * kBK + 8 * pc);
  }
};

// ---- TT operand: [64][R] image (k-rows of R bf16), read transposed --------------------------
template <int R>
__device__ __forceinline__ int tt_swz(int kr) {
  return R >= 128 ? 4 * (kr & 3) : (R == 64 ? 4 * ((kr >> 1) & 1) : 0);
}

template <int R, int NW>
struct ColImage {
  static constexpr int BYTES = R * kBK * 2;
  static constexpr int NINST = BYTES / 1024;
  static constexpr int CHUNKS = R / 8;          // 16-B chunks per k-row
  static constexpr int ROWS_PER_INST = 1024 / (2 * R);
  // R = 256 rows are 512 B: the same bank pattern mod 256 B as R = 128, so the same swizzle
  static_assert(R == 32 || R == 64 || R == 128 || R == 256, "TT tile width");
  __device__ __forceinline__ static void fill(__bf16 *img, const __bf16 *src, int64_t ld, int k0,
                                              int wid, int lane) {
#pragma unroll
    for (int j = 0; j < (NINST + NW - 1) / NW; ++j) {
      const int i = wid + NW * j;
      if (NINST % NW == 0 || i < NINST) {
        const int kr = ROWS_PER_INST * i + lane / CHUNKS;
        const int lc = (lane % CHUNKS) ^ tt_swz<R>(kr);
        const __bf16 *g = src + static_cast<int64_t>(k0 + kr) * ld + 8 * lc;
        __builtin_amdgcn_global_load_lds(g, (lds_void *)(img + 512 * i), 16, 0, 0);
      }
    }
  }
  // MFMA fragment of the 32 columns at c0: lane (i = lane & 15, g = lane >> 4) reads k-rows
  // 16 ks + 8 (g >> 1) + (i >> 2) (+4), columns c0 + 16 (g & 1) + 4 (i & 3) .. +3
  __device__ __forceinline__ static bf16x8 frag(const __bf16 *img, int c0, int ks, int lane) {
    const int i = lane & 15, g = lane >> 4;
    const int kr = 16 * ks + 8 * (g >> 1) + (i >> 2);
    const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
    const int sw = tt_swz<R>(kr);  // equal for kr and kr + 4
    const __bf16 *a = img + kr * R + 8 * ((col >> 3) ^ sw) + (col & 7);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(a));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(a + 4 * R));
    const s16x8 w = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, w);
  }
};

// XCD-aware tile order: blocks b, b + 8, ... share an XCD (and its L2); give each XCD group one
// contiguous run of row-major (tile_m, tile_n) ids, bijective for any tile count.
__device__ __forceinline__ void xcd_map(int b, int tiles, int &id) {
  const int q = tiles / 8, r = tiles % 8, x = b % 8;
  id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// LDS-DMA wave-instructions of one operand image (instantiates only the image kind in use)
template <bool TT, int R, int NW>
struct ImageInst { static constexpr int v = RowImage<R, NW>::NINST; };
template <int R, int NW>
struct ImageInst<true, R, NW> { static constexpr int v = ColImage<R, NW>::NINST; };

template <int TM, int TN, int WM, int WN, int KIND, int NS>
struct WideCfg {
  static constexpr int NW = WM * WN;
  static constexpr int NT = 64 * NW;
  static constexpr int BM = 32 * TM * WM;
  static constexpr int BN = 32 * TN * WN;
  static constexpr bool TT = KIND == WK_WGRAD;
  static constexpr int IMG_A = BM * kBK * 2, IMG_B = BN * kBK * 2;
  static constexpr int STAGE = IMG_A + IMG_B;
  static constexpr int SC = BN + 4;  // f32 epilogue tile row stride (floats)
  // the f32 epilogue tile is staged one wave-row band at a time when the whole tile would not fit
  // in LDS (256 x 256 tiles: two 128-row halves of 133 KB)
  static constexpr int EH = BM * SC * 4 > 160 * 1024 ? WM : 1;
  static constexpr int ER = BM / EH;  // rows per epilogue band
  static constexpr int EPI = ER * SC * 4;
  static constexpr int LDS = (NS * STAGE > EPI ? NS * STAGE : EPI);
  // LDS-DMA wave-instructions per wave per k-tile (equal for every wave: counted vmcnt waits)
  static constexpr int NI_A = ImageInst<TT, BM, NW>::v;
  static constexpr int NI_B = ImageInst<TT, BN, NW>::v;
  static_assert(NI_A % NW == 0 && NI_B % NW == 0, "uneven LDS-DMA split over the waves");
  static constexpr int PER = (NI_A + NI_B) / NW;
  static_assert(PER * (NS - 2) < 64, "vmcnt range");
  static_assert(EH == 1 || !TT, "banded epilogue only for the NT kinds");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// s_waitcnt vmcnt(PER * n) for a runtime n in [0, NMAX]: the immediate is an instruction field
template <int PER, int N>
__device__ __forceinline__ void vm_wait_le(int n) {
  if constexpr (N == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (n >= N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER * N) : "memory");
    else vm_wait_le<PER, N - 1>(n);
  }
}

// One workgroup's tile: bx / bz stand for blockIdx.x / .z of a launch of this kind alone, lds
// is the block's C::LDS bytes.
template <int TM, int TN, int WM, int WN, int KIND, int NS>
__device__ __forceinline__ void wide_gemm_body(const WideBatch &wb, int bx, int bz, char *lds) {
  using C = WideCfg<TM, TN, WM, WN, KIND, NS>;
  constexpr int NW = C::NW, NT = C::NT, BM = C::BM, BN = C::BN;

  const WideProblem P = (bz == 0) ? wb.p[0] : wb.p[1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_m = (P.m + BM - 1) / BM, tiles_n = (P.n + BN - 1) / BN;
  const int tiles = tiles_m * tiles_n;
  int id, split = 0;
  if constexpr (C::TT) {
    // WGRAD: blockIdx.x enumerates (split, tile).  Every tile of a split reads the same k-rows of
    // both operands, so all of them go to one XCD (blocks b, b + 8, ... share an XCD and its L2):
    // split s on XCD s % 8, its rows fetched from HBM once instead of once per XCD holding one of
    // its tiles.  Bijective when the split count is a multiple of 8; otherwise split-major.
    const int b = bx;
    if (b >= tiles * wb.splits) return;
    if (wb.splits % 8 == 0) {
      const int x = b % 8, j = b / 8;
      split = x + 8 * (j / tiles);
      id = j % tiles;
    } else {
      split = b / tiles;
      id = b % tiles;
    }
  } else {
    if (bx >= tiles) return;
    xcd_map(bx, tiles, id);
  }
  const int tile_m = id / tiles_n, tile_n = id % tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int count = wb.rows_n ? *wb.rows_n : (C::TT ? P.k : P.m);

  // k-tile range
  int kt0 = 0, kt1;
  if constexpr (C::TT) {
    const int nk = (count + kBK - 1) / kBK;
    kt0 = static_cast<int>((static_cast<int64_t>(split) * nk) / wb.splits);
    kt1 = static_cast<int>((static_cast<int64_t>(split + 1) * nk) / wb.splits);
  } else {
    kt1 = P.k / kBK;
    if (m0 >= count) {  // tile wholly past the row count: zero output rows and colsum row
      if (KIND == WK_DGRAD && P.colsum)
        for (int c = tid; c < BN; c += NT)
          if (n0 + c < P.n) P.colsum[static_cast<int64_t>(tile_m) * P.n_colsum + n0 + c] = 0.f;
      constexpr int CG = BN / 8;
      const int rows = min(BM, P.m - m0);
      for (int i = tid; i < rows * CG; i += NT) {
        const int r = i / CG, n = n0 + 8 * (i % CG);
        if (n >= P.n) continue;
        const int64_t o = static_cast<int64_t>(m0 + r) * P.ldc + n;
        if (KIND == WK_F32) {
          float *dst = static_cast<float *>(P.c) + o;
          *reinterpret_cast<float4 *>(dst) = make_float4(0.f, 0.f, 0.f, 0.f);
          *reinterpret_cast<float4 *>(dst + 4) = make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
          *reinterpret_cast<uint4 *>(static_cast<__bf16 *>(P.c) + o) = make_uint4(0u, 0u, 0u, 0u);
        }
      }
      return;
    }
  }

  __bf16 *stage0 = reinterpret_cast<__bf16 *>(lds);
  auto img_a = [&](int buf) { return stage0 + buf * (C::STAGE / 2); };
  auto img_b = [&](int buf) { return stage0 + buf * (C::STAGE / 2) + C::IMG_A / 2; };
  auto fill = [&](int buf, int kt) {
    const int k0 = kt * kBK;
    if constexpr (C::TT) {
      ColImage<BM, NW>::fill(img_a(buf), P.a + m0, P.lda, k0, wid, lane);
      ColImage<BN, NW>::fill(img_b(buf), P.b + n0, P.ldb, k0, wid, lane);
    } else {
      RowImage<BM, NW>::fill(img_a(buf), P.a + static_cast<int64_t>(m0) * P.lda, P.lda, k0, wid, lane);
      RowImage<BN, NW>::fill(img_b(buf), P.b + static_cast<int64_t>(n0) * P.ldb, P.ldb, k0, wid, lane);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // WGRAD column sums of A (acol): the wn == 0 waves of the tile_n == 0 blocks add the 8 bf16
  // k-values of each A fragment they feed the MFMA (lane l: column l & 31 of its 32-column tile,
  // k-rows 8 (l >> 5) .. +7 of each 16-deep k-step) in a fixed order
  const bool do_acol = C::TT && P.acol && tile_n == 0 && wn == 0;
  float csum[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) csum[i] = 0.f;

  // NS-stage LDS ring: tiles kt+1 .. kt+NS-1 in flight while tile kt is computed
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (kt0 + s < kt1) fill(s, kt0 + s);
  int buf = 0;
  for (int kt = kt0; kt < kt1; ++kt) {
    // this wave's DMA of tile kt has landed (the younger tiles may stay in flight), then every
    // wave's by the barrier; every wave is done reading buffer (kt - 1) % NS, refilled below
    vm_wait_le<C::PER, NS - 2>(min(NS - 2, kt1 - 1 - kt));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + NS - 1 < kt1) fill(buf == 0 ? NS - 1 : buf - 1, kt + NS - 1);
    const __bf16 *ia = img_a(buf), *ib = img_b(buf);
#pragma unroll
    for (int ks = 0; ks < kBK / 16; ++ks) {
      bf16x8 av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if constexpr (C::TT) av[i] = ColImage<BM, NW>::frag(ia, (wm * TM + i) * 32, ks, lane);
        else av[i] = RowImage<BM, NW>::frag(ia, (wm * TM + i) * 32, ks, lane);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (C::TT) bv[j] = ColImage<BN, NW>::frag(ib, (wn * TN + j) * 32, ks, lane);
        else bv[j] = RowImage<BN, NW>::frag(ib, (wn * TN + j) * 32, ks, lane);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
      if constexpr (C::TT) {
        if (do_acol) {
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const uint4 u = __builtin_bit_cast(uint4, av[i]);
            csum[i] += ((bf_lo(u.x) + bf_hi(u.x)) + (bf_lo(u.y) + bf_hi(u.y))) +
                       ((bf_lo(u.z) + bf_hi(u.z)) + (bf_lo(u.w) + bf_hi(u.w)));
          }
        }
      }
    }
    buf = buf + 1 == NS ? 0 : buf + 1;
  }
  if constexpr (C::TT) {
    if (do_acol) {  // the two lane halves hold the same columns' other k-rows
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float s = csum[i] + __shfl_xor(csum[i], 32, 64);
        const int mcol = m0 + (wm * TM + i) * 32 + lane;
        if (lane < 32 && mcol < P.m) {
          const int64_t o = static_cast<int64_t>(split) * P.slab_stride + mcol;
          P.acol[o] = s;
          if (P.acol2) P.acol2[o] = s;
        }
      }
    }
  }
  __syncthreads();  // the staging buffers become the epilogue tile

  float *tile = reinterpret_cast<float *>(lds);
  // accumulators of wave-row band eh -> f32 LDS tile [ER][SC]
  auto stage_band = [&](int eh) {
    if (C::EH > 1 && wm != eh) return;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5) - eh * C::ER;
          const int col = (wn * TN + j) * 32 + (lane & 31);
          tile[row * C::SC + col] = acc[i][j][r];
        }
  };

  if constexpr (KIND == WK_WGRAD) {
    stage_band(0);
    __syncthreads();
    // f32 slab store, 4 columns per item
    constexpr int CG = BN / 4, RSTEP = NT / CG;
    static_assert(NT % CG == 0, "epilogue layout");
    const int cg = tid % CG, r0 = tid / CG;
    const int n = n0 + 4 * cg;
    float *slab = static_cast<float *>(P.c) + static_cast<int64_t>(split) * P.slab_stride;
    for (int r = r0; r < BM; r += RSTEP) {
      const int m = m0 + r;
      if (m >= P.m) break;
      const float4 v = *reinterpret_cast<const float4 *>(tile + r * C::SC + 4 * cg);
      float *dst = slab + static_cast<int64_t>(m) * P.ldc + n;
      if (n + 3 < P.n && (P.ldc & 3) == 0) {
        *reinterpret_cast<float4 *>(dst) = v;
      } else {
        if (n < P.n) dst[0] = v.x;
        if (n + 1 < P.n) dst[1] = v.y;
        if (n + 2 < P.n) dst[2] = v.z;
        if (n + 3 < P.n) dst[3] = v.w;
      }
    }
    return;
  } else {
    // 8 columns per item: bf16 16-B stores (FWD / DGRAD) or f32 2 x 16-B stores (F32)
    constexpr int CG = BN / 8, RSTEP = NT / CG;
    static_assert(NT % CG == 0, "epilogue layout");
    static_assert(KIND != WK_DGRAD || BN <= NT, "one column-sum thread per column");
    const int cg = tid % CG, r0 = tid / CG;
    const int n = n0 + 8 * cg;
    const bool ncol = n < P.n;  // P.n is a multiple of 8 on this path (host-checked)
    float bias[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bias[e] = 0.f;
    if ((KIND == WK_FWD || KIND == WK_F32) && P.bias && ncol) {
      const float4 b0 = *reinterpret_cast<const float4 *>(P.bias + n);
      const float4 b1 = *reinterpret_cast<const float4 *>(P.bias + n + 4);
      bias[0] = b0.x, bias[1] = b0.y, bias[2] = b0.z, bias[3] = b0.w;
      bias[4] = b1.x, bias[5] = b1.y, bias[6] = b1.z, bias[7] = b1.w;
    }
    float csum = 0.f;  // DGRAD: column n0 + tid, summed over the tile's rows in row order
#pragma unroll 1
    for (int eh = 0; eh < C::EH; ++eh) {
      if (eh > 0) __syncthreads();  // the previous band's tile reads are done
      stage_band(eh);
      __syncthreads();
      const int mb = m0 + eh * C::ER;  // first row of the band
      for (int r = r0; r < C::ER; r += RSTEP) {
        const int m = mb + r;
        if (m >= P.m) break;  // never past the allocation's row bound
        float *t = tile + r * C::SC + 8 * cg;
        const float4 x0 = *reinterpret_cast<const float4 *>(t);
        const float4 x1 = *reinterpret_cast<const float4 *>(t + 4);
        float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        const bool live = m < count;
        if (!ncol) continue;
        if constexpr (KIND == WK_F32) {
          if (P.bias)  // f32 C + bias (the BiLSTM's input projection); the heads pass none
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = v[e] + bias[e];
          float *dst = static_cast<float *>(P.c) + static_cast<int64_t>(m) * P.ldc + n;
          *reinterpret_cast<float4 *>(dst) =
              live ? make_float4(v[0], v[1], v[2], v[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
          *reinterpret_cast<float4 *>(dst + 4) =
              live ? make_float4(v[4], v[5], v[6], v[7]) : make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
          if constexpr (KIND == WK_FWD) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = live ? act_forward(v[e] + bias[e], wb.act) : 0.f;
          } else {  // DGRAD: act'(y) with y the bf16 layer output, in place
            const uint4 y = *reinterpret_cast<const uint4 *>(P.aux + static_cast<int64_t>(m) * P.ldc + n);
            const float yf[8] = {bf_lo(y.x), bf_hi(y.x), bf_lo(y.y), bf_hi(y.y),
                                 bf_lo(y.z), bf_hi(y.z), bf_lo(y.w), bf_hi(y.w)};
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = live ? act_backward(v[e], yf[e], wb.act) : 0.f;
            if (P.colsum) {  // the bias gradient sums the f32 values (before bf16 rounding)
              *reinterpret_cast<float4 *>(t) = make_float4(v[0], v[1], v[2], v[3]);
              *reinterpret_cast<float4 *>(t + 4) = make_float4(v[4], v[5], v[6], v[7]);
            }
          }
          const uint4 o = make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]),
                                     pack2(v[6], v[7]));
          *reinterpret_cast<uint4 *>(static_cast<__bf16 *>(P.c) + static_cast<int64_t>(m) * P.ldc + n) = o;
        }
      }
      if (KIND == WK_DGRAD && P.colsum) {
        // column sums over the band's rows: NT / BN row groups of consecutive rows per column,
        // then the groups combined in group order (fixed: bitwise reproducible)
        constexpr int RG = NT / BN, RPG = (C::ER + RG - 1) / RG;
        __syncthreads();
        const int rows = min(C::ER, P.m - mb);
        const int c = tid % BN, g = tid / BN;
        float s = 0.f;
        for (int r = g * RPG; r < min(rows, (g + 1) * RPG); ++r) s += tile[r * C::SC + c];
        __syncthreads();  // every group's reads of the band are done: reuse its first row
        tile[g * C::SC + c] = s;
        __syncthreads();
        if (tid < BN) {
          float t = tile[tid];
#pragma unroll
          for (int q = 1; q < RG; ++q) t += tile[q * C::SC + tid];
          csum += t;
        }
      }
    }
    if (KIND == WK_DGRAD && P.colsum && tid < BN && n0 + tid < P.n)
      P.colsum[static_cast<int64_t>(tile_m) * P.n_colsum + n0 + tid] = csum;
  }
}

template <int TM, int TN, int WM, int WN, int KIND, int NS>
__global__ __launch_bounds__(64 * WM * WN) void wide_gemm_kernel(WideBatch wb) {
  __shared__ __attribute__((aligned(16))) char lds[WideCfg<TM, TN, WM, WN, KIND, NS>::LDS];
  wide_gemm_body<TM, TN, WM, WN, KIND, NS>(wb, blockIdx.x, blockIdx.z, lds);
}

// A layer's WGRAD and DGRAD in one launch (the backward's per-layer pair: both read the layer's dZ,
// neither writes what the other reads -- DGRAD writes the next layer's dZ to its own buffer):
// blocks [0, wg_blocks) run the WGRAD grid, the rest the DGRAD grid, each with the block index it
// has in a launch of its own (wg_blocks a multiple of 8 keeps both XCD maps).
template <int TM, int TN, int WM, int WN, int NS>
__global__ __launch_bounds__(64 * WM * WN) void wide_pair_kernel(WideBatch wg, WideBatch dg,
                                                                 int wg_blocks) {
  constexpr int LW = WideCfg<TM, TN, WM, WN, WK_WGRAD, NS>::LDS;
  constexpr int LD = WideCfg<TM, TN, WM, WN, WK_DGRAD, NS>::LDS;
  __shared__ __attribute__((aligned(16))) char lds[LW > LD ? LW : LD];
  const int b = static_cast<int>(blockIdx.x);
  if (b < wg_blocks) wide_gemm_body<TM, TN, WM, WN, WK_WGRAD, NS>(wg, b, blockIdx.z, lds);
  else wide_gemm_body<TM, TN, WM, WN, WK_DGRAD, NS>(dg, b - wg_blocks, blockIdx.z, lds);
}

}  // namespace wide
}  // namespace ppo
