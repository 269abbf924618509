// Device helpers shared by the fused bf16 kernels (fused_update.hip, fused_policy.hip):
// bf16 packing, the XOR-swizzled LDS activation images with their row / transposed fragment
// reads, the 32x32x16 bf16 MFMA, the wave-half reduce-scatter, and the weight-ring k-pass.
#pragma once

#include "common.h"
#include "fused_update.h"

namespace ppo {
namespace fu {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int R = kFusedRows;
constexpr int NW = 8;           // waves per workgroup (two per SIMD, 256 registers each)
constexpr int NT = 64 * NW;
constexpr int DZP = 12;         // dz row pitch (floats): 48-B rows, conflict-free row reads

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  const f32x2 f = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2));
}
__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// ---- LDS images ----------------------------------------------------------------------------
// H-wide bf16 image, pitch a multiple of 256 B: 16-B chunk c of row r lives at
// r*pitch + 16*(c ^ swz(r)), swz(r) = ((r&3)<<2) | ((r>>2)&3) (XOR touches the low 4 chunk bits).
__device__ __forceinline__ int img_off(int r, int c, int pitch) {
  return r * pitch + 16 * (c ^ (((r & 3) << 2) | ((r >> 2) & 3)));
}
// X image: 64-B rows (4 chunks), chunk c of row r at r*64 + 16*(c ^ ((r>>2)&3)).
__device__ __forceinline__ int x_off(int r, int c) { return r * 64 + 16 * (c ^ ((r >> 2) & 3)); }

// a pointer as address space 1 (global): loads through it are global_load, not flat_load
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T *gptr(const T *p) {
  return (const __attribute__((address_space(1))) T *)(p);
}

__device__ __forceinline__ bf16x8 lds_b128(const char *p) { return *reinterpret_cast<const bf16x8 *>(p); }

__device__ __forceinline__ bf16x8 tr_pair(const char *a, const char *b) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(a));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(b));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// 32x32x16 operand whose k runs over image ROWS k0..k0+15 and whose m/n runs over image
// COLUMNS col0..col0+31: lane (c = lane&31, h = lane>>5) gets rows k0+8h..+7 of column col0+c.
// ds_read_b64_tr_b16: in 16-lane group g, lane 4q+p addresses block row q, columns 4p..4p+3.
__device__ __forceinline__ bf16x8 tr_frag(const char *img, int pitch, int k0, int col0, int lane) {
  const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
  const int row = k0 + 8 * (g >> 1) + q;
  const int c = (col0 >> 3) + 2 * (g & 1) + (p >> 1);
  return tr_pair(img + img_off(row, c, pitch) + 8 * (p & 1),
                 img + img_off(row + 4, c, pitch) + 8 * (p & 1));
}
__device__ __forceinline__ bf16x8 tr_frag_x(const char *img, int k0, int lane) {
  const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
  const int row = k0 + 8 * (g >> 1) + q;
  const int c = 2 * (g & 1) + (p >> 1);
  return tr_pair(img + x_off(row, c) + 8 * (p & 1), img + x_off(row + 4, c) + 8 * (p & 1));
}

// Explicit wait states before VALU reads of accumulators produced by the last MFMAs of a rolled
// loop: a 16-pass v_mfma_f32_32x32x16_bf16 result needs 18 wait states before a VALU read, and
// hipcc's hazard recognizer undercounts across the loop-exit edge (observed: a v_mov of the last
// accumulator ~12 instructions after the MFMA with only s_nop 0 -> partially written lanes,
// timing-dependent results).  The asm takes the accumulators as operands so nothing that reads
// them can be scheduled above it.
template <int NACC>
__device__ __forceinline__ void mfma_drain(f32x16 (&acc)[NACC]) {
  if constexpr (NACC == 1) {
    asm volatile("s_nop 15\n\ts_nop 7" : "+v"(acc[0]));
  } else {
    asm volatile("s_nop 15\n\ts_nop 7" : "+v"(acc[0]), "+v"(acc[1]));
  }
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// ---- 16x16x32 bf16 MFMA (the head products) ------------------------------------------------
// A[16 x 32]: lane l holds A[l & 15][8 (l >> 4) + j]; B[32 x 16]: B[8 (l >> 4) + j][l & 15];
// D[16 x 16]: lane l holds D[4 (l >> 4) + i][l & 15], i = 0..3 (cdna_hip_programming.md s3).
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 16x16x32 operand whose k runs over image ROWS k0..k0+31 and whose m/n runs over image COLUMNS
// col0..col0+15: lane (c = lane & 15, g = lane >> 4) gets rows k0 + 8g .. +7 of column col0 + c.
// Same ds_read_b64_tr_b16 block pattern as tr_frag: a 32-lane half's two blocks sit 8 rows apart
// in the same 16 columns (conflict-free on the XOR-swizzled image).
__device__ __forceinline__ bf16x8 tr_frag16(const char *img, int pitch, int k0, int col0, int lane) {
  const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
  const int row = k0 + 8 * g + q;
  const int c = (col0 >> 3) + (p >> 1);
  return tr_pair(img + img_off(row, c, pitch) + 8 * (p & 1),
                 img + img_off(row + 4, c, pitch) + 8 * (p & 1));
}

// bf16 head-weight image: 16 rows (heads; rows >= the net's head width are zero) of H bf16 plus
// 8 bf16 of padding, so the 16 lanes of a 16x16x32 B-operand read hit 16 distinct bank groups.
template <int H>
struct HeadImg {
  static constexpr int PITCH = 2 * H + 16;  // bytes
  static constexpr int BYTES = 16 * PITCH;
};

// dz images of one 64-row chunk (bf16, the head-backward MFMA operands): row-major [64][16]
// (d2 = dz . Wh, B operand: 8 heads of one row) and head-major [16][64 + 8] (head dW, A operand:
// 8 rows of one head).
constexpr int kDzRowBytes = 32;
constexpr int kDzTPitch = 2 * (kFusedRows + 8);

// Stage the net's head weights as the bf16 image (one pass over the block) and return this lane's
// d2-MFMA A fragment W_h^T: lane (c = lane & 31, h = lane >> 5) of wave w holds
// W_h[8h + j][32w + c], j = 0..7 (call after a barrier that follows the staging).
template <int H>
__device__ __forceinline__ void stage_head_image(char *img, const float *wh, int nh_real, int tid,
                                                 int nt) {
  for (int i = tid; i < 16 * (H / 2); i += nt) {
    const int a = i / (H / 2), f = 2 * (i % (H / 2));
    const float x0 = a < nh_real ? wh[a * H + f] : 0.f;
    const float x1 = a < nh_real ? wh[a * H + f + 1] : 0.f;
    *reinterpret_cast<uint32_t *>(img + a * HeadImg<H>::PITCH + 2 * f) = pack2(x0, x1);
  }
}
template <int H>
__device__ __forceinline__ bf16x8 head_t_frag(const char *img, int w, int lane) {
  const int c = lane & 31, h = lane >> 5;
  typedef short s16x8_t __attribute__((ext_vector_type(8)));
  s16x8_t v;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    v[j] = *reinterpret_cast<const short *>(img + (8 * h + j) * HeadImg<H>::PITCH + 2 * (32 * w + c));
  return __builtin_bit_cast(bf16x8, v);
}

// ---- cross-lane exchange on the VALU (DPP / v_permlane16_swap) instead of ds_bpermute ----------
// Only lane patterns that are their own inverse are used (quad_perm xor, row_half_mirror,
// row_mirror, row_ror:8), so a partner pair always exchanges with each other.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141; // lane i <-> 7 - i within each 8 lanes
constexpr int kDppRor8 = 0x128;       // lane i <-> i ^ 8 within each 16-lane row
// Sum over each 16-lane row, every lane ending with the same value: the adds are exactly those of
// the xor-1/2/4/8 butterfly (the half-mirror partner of a lane holds the other quad's sum).
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<kDppXor1>(v);
  v += dpp_f<kDppXor2>(v);
  v += dpp_f<kDppHalfMirror>(v);
  v += dpp_f<kDppRor8>(v);
  return v;
}

// Fixed-order reduce-scatter of 16 per-lane values over the 32 lanes of a wave half.  Level 1
// pairs lanes m, m^16 (v_permlane16_swap: X'+Y' = keep + received on every lane), level 2 m, m^8,
// level 3 m, m^7 (half mirror: same b4/b3, opposite b2), level 4 m, m^2, then a final m, m^1 add:
// lane m holds the full sum of value q(m) = 8*b4(m) + 4*b3(m) + 2*b2(m) + b1(m) (bit k of m: bk),
// duplicated on lanes m, m^1.  All exchanges are VALU ops (no LDS round trips).
__device__ __forceinline__ float rs16(float (&v)[16], int lane) {
  const int m = lane & 31;
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // rows 0/2 keep v[i] (+ partner's v[i]), rows 1/3 v[i + 8]
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 8]), false, false);
    v[i] = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  }
  {
    const bool up = m & 8;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float send = up ? v[i] : v[i + 4];
      const float keep = up ? v[i + 4] : v[i];
      v[i] = keep + dpp_f<kDppRor8>(send);
    }
  }
  {
    const bool up = m & 4;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float send = up ? v[i] : v[i + 2];
      const float keep = up ? v[i + 2] : v[i];
      v[i] = keep + dpp_f<kDppHalfMirror>(send);
    }
  }
  {
    const bool up = m & 2;
    const float send = up ? v[0] : v[1];
    const float keep = up ? v[1] : v[0];
    v[0] = keep + dpp_f<kDppXor2>(send);
  }
  return v[0] + dpp_f<kDppXor1>(v[0]);
}
// feature (within a 32-wide tile, lane half h) whose sum rs16 leaves on lane m
__device__ __forceinline__ int rs16_feature(int lane) {
  const int m = lane & 31, h = lane >> 5;
  const int q = 8 * ((m >> 4) & 1) + 4 * ((m >> 3) & 1) + 2 * ((m >> 2) & 1) + ((m >> 1) & 1);
  return (q & 3) + 8 * (q >> 2) + 4 * h;
}

__device__ __forceinline__ int reg_feature(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// acc[t] += W[32w + r][:] . img[32t + r][:] over k = 0..H-1 for row tiles t < NTILE (2: the
// update kernel's 64-row chunks; 1: the rollout step's 32-row workgroups).  A operand
// = the L2-resident bf16 weight image in FRAGMENT-MAJOR order (w_frag below: the 64 lanes' 16-B
// fragments of one (k-step, wave) are one contiguous 1 KB block, so a ring load is 8 full cache
// lines instead of 32 partial row pieces), B operand = 16-B row reads of the LDS activation image.
// Weight fragments run through a ring of PD + 1 registers: the load for k-step s + PD is issued
// before the MFMAs of step s (the first PD by wring_prime, a phase earlier), so L2 latency hides
// behind 2*PD MFMAs per wave; the B reads of step s + 1 overlap step s; sched_barrier pins one
// k-step per scheduling region so the compiler cannot hoist the whole pass's loads (register
// blow-up).
constexpr int PD = 3;  // prefetch distance (k-steps); ring period PD + 1 = 4

// Fragment-major H x H image: element (o, i) -- output feature o, input column i -- of the
// 32x32x16 A operand for (k-step s = i / 16, wave w = o / 32, lane h*32 + r) lives at
// ((s * (H/32) + w) * 64 + h * 32 + r) * 8 + (i & 7), h = (i / 8) & 1, r = o & 31.
__device__ __forceinline__ int64_t w_frag(int o, int i, int H) {
  return (static_cast<int64_t>((i >> 4) * (H >> 5) + (o >> 5)) * 64 + ((i >> 3) & 1) * 32 + (o & 31)) * 8 +
         (i & 7);
}
// The wave's fragment of k-step 0 (lane = h * 32 + r); k-step s is s * 16 * H elements further.
template <int H>
__device__ __forceinline__ const __bf16 *w_frag_base(const __bf16 *img, int w, int lane) {
  return img + (static_cast<int64_t>(w) * 64 + lane) * 8;
}

template <int H>
__device__ __forceinline__ void wring_prime(const __bf16 *wfrag, bf16x8 (&ring)[PD + 1]) {
#pragma unroll
  for (int s = 0; s < PD; ++s) ring[s] = *reinterpret_cast<const bf16x8 *>(wfrag + static_cast<int64_t>(16 * H) * s);
}
template <int H, int NTILE>
__device__ __forceinline__ void mlp_pass(const __bf16 *wfrag, const char *img, int r, int h,
                                         bf16x8 (&ring)[PD + 1], f32x16 (&acc)[NTILE]) {
  constexpr int KS = H / 16;
  static_assert(KS % (PD + 1) == 0, "ring period must divide the k-steps");
  const int swz = ((r & 3) << 2) | ((r >> 2) & 3);
  const char *rowp = img + r * (2 * H);
  // rolled over all ring periods but the last (one load per k-step: the vmcnt waits of the rolled
  // loop assume a uniform count) ...
#pragma unroll 1
  for (int s0 = 0; s0 < KS - (PD + 1); s0 += PD + 1) {
#pragma unroll
    for (int u = 0; u <= PD; ++u) {
      const int s = s0 + u;
      const bf16x8 af = ring[u];
      ring[(u + PD) % (PD + 1)] = *reinterpret_cast<const bf16x8 *>(wfrag + static_cast<int64_t>(16 * H) * (s + PD));
      const char *p = rowp + 16 * ((2 * s + h) ^ swz);
#pragma unroll
      for (int t = 0; t < NTILE; ++t) acc[t] = mfma(af, lds_b128(p + t * 32 * (2 * H)), acc[t]);
    }
  }
  // ... and the last period peeled: only its first k-step still prefetches (step KS-1), so no
  // redundant weight loads are in flight when the pass ends (a wait on them, forced by a
  // register reuse after the pass, cost a full L2 round trip per pass)
#pragma unroll
  for (int u = 0; u <= PD; ++u) {
    const int s = KS - (PD + 1) + u;
    const bf16x8 af = ring[u];
    if (s + PD < KS)
      ring[(u + PD) % (PD + 1)] = *reinterpret_cast<const bf16x8 *>(wfrag + static_cast<int64_t>(16 * H) * (s + PD));
    const char *p = rowp + 16 * ((2 * s + h) ^ swz);
#pragma unroll
    for (int t = 0; t < NTILE; ++t) acc[t] = mfma(af, lds_b128(p + t * 32 * (2 * H)), acc[t]);
  }
  mfma_drain(acc);
}

}  // namespace fu

}  // namespace ppo
