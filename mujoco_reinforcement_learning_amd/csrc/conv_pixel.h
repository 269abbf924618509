// The pixel layer of the encoder (conv.h L1: 84x84x3 u8 -> 20x20x32, k8 s4) in bf16 mode, as a
// stride-1 2x2 convolution over the space-to-depth image of the frame.
//
// Space-to-depth.  The frame [84][84][3] is cut into 21x21 blocks of 4x4 pixels; block (by, bx)
// holds the 48 values (dy, dx, ci) = frame[4by + dy][4bx + dx][ci].  Kernel tap (ky, kx) =
// (4ty + dy, 4tx + dx) with ty, tx in {0, 1}, so
//   y[oy, ox, co] = b[co] + sum_{ty, tx} sum_{(dy, dx, ci)} S[oy + ty, ox + tx][(dy, dx, ci)] W[co, ci, ky, kx]
// -- a product with K = 4 taps x 48 channels whose operand rows are whole 48-value blocks: one
// 16-B LDS read gives 8 consecutive k of a position, where the implicit GEMM of conv.h gathers
// 4-byte pieces of 8-pixel window rows from global memory.  A frame row y, block bx is 12
// contiguous bytes of the frame (byte 12 * (21y + bx)) and 12 contiguous values of block
// (y / 4, bx) at (y % 4) * 12: staging is 1764 12-byte units per frame.
//
// S lives in LDS as bf16 (RNE of u8 / 255, the value conv.h's staging rounds to), 56 values per
// block (48 + 8 pad: the 112-B stride puts 16 consecutive blocks' 16-B rows on distinct banks).
//
//   pixel_fwd_kernel    y = relu(conv + b), both nets per frame (the frame is staged once):
//                       persistent workgroups of 10 waves, one frame at a time, wave (z, w) net
//                       z's output rows 4w .. 4w+3 (5 tiles of 16 positions); the transposed
//                       product y^T[co][p] = W'[co][k] S^T[k][p] on v_mfma_f32_16x16x32_bf16 with
//                       the net's W' (12 fragments) in registers and one S fragment per 2 MFMAs
//                       (both nets' W' in one wave's registers spills); each lane stores 4
//                       consecutive channels of one position (8 B).
//   pixel_wgrad_kernel  dW[co][(tap, ch)] = sum_p dz[p][co] S[p + tap][ch] (+ db = sum_p dz), one
//                       split of the minibatch's frames per workgroup (the split's f32 slab in
//                       torch order, reduced in a fixed order by the engine's slab pass): 8 waves,
//                       wave (nh, kp) the N tiles 3nh .. 3nh+2 (of 6 x 32 columns) of both nets
//                       over the k-steps kp, kp + 4, ... (positions 16 ks .. +15); dz staged as
//                       bf16 [p][co] (f32 column sums first), both operands read with
//                       ds_read_b64_tr_b16 on v_mfma_f32_32x32x16_bf16; the four k-parts fold in
//                       LDS in a fixed order at the end.
// Reference: none (the reference has no pixel path).
#pragma once

#include "conv.h"

namespace ppo {
namespace conv {

constexpr int kS2dSide = 21;                      // blocks per dimension
constexpr int kS2dBlocks = kS2dSide * kS2dSide;   // 441
constexpr int kS2dCh = 48;                        // (dy, dx, ci)
constexpr int kS2dPitch = 56;                     // bf16 per block in LDS
constexpr int kS2dBytes = kS2dBlocks * kS2dPitch * 2;
constexpr int kPixUnits = 84 * kS2dSide;          // 12-byte frame units (y, bx)
constexpr int kPixFrameBytes = L1::PIN * L1::cin; // 21168
static_assert(kPixFrameBytes == 12 * kPixUnits, "frame units");
static_assert(L1::k == 8 && L1::s == 4 && L1::cin == 3 && L1::cout == 32 && L1::hout == 20,
              "pixel layer geometry");

struct PixArgs {
  const uint8_t *frames;   // [frames][84][84][3]
  const int32_t *rows;     // image j is frame rows[j] (null: frame j)
  int nimg;
  const float *w[2];       // torch-order weights [32][3][8][8] (f32 parameters)
  const float *bias[2];    // FWD
  __bf16 *out[2];          // FWD: HWC activations [img][400][32]
  const float *dz[2];      // WGRAD: f32 gradient at the pre-activation [img][400][32]
  float *slab[2];          // WGRAD: split 0 of the layer's slabs (dW torch order, then db)
  int64_t slab_stride;
  int splits;
};

__device__ __forceinline__ const uint8_t *pix_frame(const PixArgs &q, int img) {
  const int64_t f = q.rows ? static_cast<int64_t>(q.rows[img]) : img;
  return q.frames + f * kPixFrameBytes;
}

__device__ __forceinline__ void pix_unit_load(const uint8_t *frame, int u, uint32_t (&w)[3]) {
  const uint32_t *p = reinterpret_cast<const uint32_t *>(frame) + 3 * u;
  w[0] = p[0];
  w[1] = p[1];
  w[2] = p[2];
}

// bf16(x * fl(1/255)) == bf16(x / 255) for every u8 x (tests/test_pixel_scale.py checks all 256;
// the f32 products differ from the quotients in 126 of them, never after the bf16 rounding), so
// the bf16 staging multiplies instead of running the IEEE divide sequence per byte.
constexpr float kInv255 = 1.f / 255.f;

// the same units held in a clang vector (components x, y, z): arrays of these stay in registers
// where arrays of uint32_t[3] were kept in scratch memory in pixel_wgrad_kernel
typedef uint32_t pix_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void pix_unit_load(const uint8_t *frame, int u, pix_u32x4 &w) {
  const uint32_t *p = reinterpret_cast<const uint32_t *>(frame) + 3 * u;
  w.x = p[0];
  w.y = p[1];
  w.z = p[2];
}

// unit u = (y, bx) -> 12 bf16 at block (y / 4, bx), offset (y % 4) * 12
__device__ __forceinline__ void pix_unit_store(__bf16 *s, int u, const uint32_t (&w)[3]);
__device__ __forceinline__ void pix_unit_store(__bf16 *s, int u, const pix_u32x4 &v) {
  const uint32_t w[3] = {v.x, v.y, v.z};
  pix_unit_store(s, u, w);
}
__device__ __forceinline__ void pix_unit_store(__bf16 *s, int u, const uint32_t (&w)[3]) {
  const int y = u / kS2dSide, bx = u - y * kS2dSide;
  __bf16 *dst = s + ((y >> 2) * kS2dSide + bx) * kS2dPitch + (y & 3) * 12;
  uint32_t o[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const uint32_t word = w[j >> 1];
    const int sh = 16 * (j & 1);
    const float lo = static_cast<float>((word >> sh) & 255u) * kInv255;
    const float hi = static_cast<float>((word >> (sh + 8)) & 255u) * kInv255;
    o[j] = pack_bf16x2(lo, hi);
  }
#pragma unroll
  for (int j = 0; j < 3; ++j)
    *reinterpret_cast<uint2 *>(dst + 4 * j) = make_uint2(o[2 * j], o[2 * j + 1]);
}

// torch offset of W'[co][k], k = tap * 48 + (dy * 12 + dx * 3 + ci)
__device__ __forceinline__ int pix_w_offset(int co, int k) {
  const int tap = k / kS2dCh, n = k - tap * kS2dCh;
  const int dy = n / 12, r = n - dy * 12, dx = r / 3, ci = r - dx * 3;
  const int ky = 4 * (tap >> 1) + dy, kx = 4 * (tap & 1) + dx;
  return co * L1::kdim + ci * (L1::k * L1::k) + ky * L1::k + kx;
}

// S block of output position p (0 .. 399) at tap offset 0
__device__ __forceinline__ int pix_block(int p) {
  const int oy = p / L1::wout;
  return oy * kS2dSide + (p - oy * L1::wout);
}

// Workgroup barrier for the per-image LDS hand-offs: waits for this wave's LDS operations only.
// __syncthreads() is a workgroup-scope release / acquire, which also waits for every global load
// and store the wave has in flight -- the next image's prefetch and this image's output stores --
// and serialised one memory round trip per image.  The same barrier as common.h's lds_sync.
__device__ __forceinline__ void lds_barrier() { lds_sync(); }

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---- forward ----------------------------------------------------------------------------------
constexpr int kPixFwdWaves = 10;
constexpr int kPixFwdThreads = 64 * kPixFwdWaves;
constexpr int kPixFwdUnits = (kPixUnits + kPixFwdThreads - 1) / kPixFwdThreads;  // 6

__global__ __launch_bounds__(kPixFwdThreads) void pixel_fwd_kernel(PixArgs q) {
  __shared__ __attribute__((aligned(16))) __bf16 fs[kS2dBlocks * kS2dPitch];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int z = wv / 5, wr = wv - 5 * z;  // net, output rows 4 wr .. 4 wr + 3

  // W' of both nets staged once through LDS as bf16 [z][co][k] (the frame image's space, before
  // the first frame), then the net's fragments: lane holds W'[16 mt + r][32 ks + 8 g .. +7]
  for (int e = tid; e < 2 * L1::cout * L1::kdim; e += kPixFwdThreads) {
    const int zz = e / (L1::cout * L1::kdim), rem = e - zz * (L1::cout * L1::kdim);
    const int co = rem / L1::kdim, k = rem - co * L1::kdim;
    const float v = q.w[zz][pix_w_offset(co, k)];
    fs[e] = __builtin_bit_cast(__bf16, static_cast<uint16_t>(pack_bf16x2(v, 0.f) & 0xffffu));
  }
  __syncthreads();
  bf16x8_t wf[2][6];
  float bias[2][4];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
    for (int ks = 0; ks < 6; ++ks)
      wf[mt][ks] = *reinterpret_cast<const bf16x8_t *>(
          fs + (z * L1::cout + 16 * mt + r) * L1::kdim + 32 * ks + 8 * g);
#pragma unroll
    for (int i = 0; i < 4; ++i) bias[mt][i] = q.bias[z][16 * mt + 4 * g + i];
  }

  // per-lane S offsets (bf16) of the k-steps: tap offset + channel
  int koff[6];
#pragma unroll
  for (int ks = 0; ks < 6; ++ks) {
    const int k0 = 32 * ks + 8 * g, tap = k0 / kS2dCh;
    koff[ks] = ((tap >> 1) * kS2dSide + (tap & 1)) * kS2dPitch + (k0 - tap * kS2dCh);
  }

  uint32_t pre[kPixFwdUnits][3];
  auto prefetch = [&](int img) __attribute__((always_inline)) {
    const uint8_t *f = pix_frame(q, img);
#pragma unroll
    for (int i = 0; i < kPixFwdUnits; ++i) {
      const int u = tid + i * kPixFwdThreads;
      pix_unit_load(f, u < kPixUnits ? u : kPixUnits - 1, pre[i]);
    }
  };
  int img = blockIdx.x;
  if (img < q.nimg) prefetch(img);
  for (; img < q.nimg; img += gridDim.x) {
    lds_barrier();  // every wave is done reading the previous frame
#pragma unroll
    for (int i = 0; i < kPixFwdUnits; ++i) {
      const int u = tid + i * kPixFwdThreads;
      if (u < kPixUnits) pix_unit_store(fs, u, pre[i]);
    }
    lds_barrier();
    if (img + static_cast<int>(gridDim.x) < q.nimg) prefetch(img + gridDim.x);

#pragma unroll 1
    for (int t = 0; t < 5; ++t) {
      const int p = 80 * wr + 16 * t + r;  // this lane's B column / C column
      const __bf16 *sb = fs + pix_block(p) * kS2dPitch;
      f32x4 acc[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) {
        const bf16x8_t b = *reinterpret_cast<const bf16x8_t *>(sb + koff[ks]);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[mt][ks], b, acc[mt], 0, 0, 0);
      }
      // C: lane holds rows (co) 4g .. 4g+3 of column (position) r
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        float y[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) y[i] = act_forward(acc[mt][i] + bias[mt][i], PPO_ACT_RELU);
        __bf16 *dst = q.out[z] + (static_cast<int64_t>(img) * L1::P + p) * L1::cout + 16 * mt + 4 * g;
        *reinterpret_cast<uint2 *>(dst) = make_uint2(pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3]));
      }
    }
  }
}

// ---- weight gradient --------------------------------------------------------------------------
constexpr int kPixWgWaves = 8;
constexpr int kPixWgThreads = 64 * kPixWgWaves;
constexpr int kPixPosPad = 416;                   // 26 k-steps of 16 positions (400 .. 415 zero)
constexpr int kPixDzPitch = 64;                   // bf16 per dz row: 32 channels + 32 pad
constexpr int kPixDzUnits = 2 * L1::P * L1::cout / 4;   // float4 units of both nets' dz: 6400
constexpr int kPixWgDzIters = (kPixDzUnits + kPixWgThreads - 1) / kPixWgThreads;  // 13
constexpr int kPixWgFrIters = (kPixUnits + kPixWgThreads - 1) / kPixWgThreads;    // 4
constexpr int kPixWgDzOff = kS2dBytes;            // bytes
constexpr int kPixWgLds = kPixWgDzOff + 2 * kPixPosPad * kPixDzPitch * 2;
static_assert(kPixWgLds <= 160 * 1024, "pixel wgrad LDS");
static_assert(3 * 32 * 32 * 3 * 2 * 4 <= kPixWgLds, "k-part fold scratch");

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

__device__ __forceinline__ bf16x8_t pix_tr_pair(const __bf16 *lo, const __bf16 *hi) {
  const s16x4_t a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)(lo));
  const s16x4_t b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t *)(hi));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 w = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8_t, w);
}

__global__ __launch_bounds__(kPixWgThreads) void pixel_wgrad_kernel(PixArgs q) {
  __shared__ __attribute__((aligned(16))) char pix_lds[kPixWgLds];
  __bf16 *fs = reinterpret_cast<__bf16 *>(pix_lds);
  __bf16 *dzs = reinterpret_cast<__bf16 *>(pix_lds + kPixWgDzOff);  // [2][416][64]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nh = wv & 1, kp = wv >> 1;
  const int split = blockIdx.x;
  const int i0 = static_cast<int>((static_cast<int64_t>(split) * q.nimg) / q.splits);
  const int i1 = static_cast<int>((static_cast<int64_t>(split + 1) * q.nimg) / q.splits);

  // zero rows 400 .. 415 of both dz images (never staged)
  for (int e = tid; e < 2 * (kPixPosPad - L1::P) * kPixDzPitch / 4; e += kPixWgThreads) {
    const int z = e / ((kPixPosPad - L1::P) * kPixDzPitch / 4);
    const int rem = e - z * ((kPixPosPad - L1::P) * kPixDzPitch / 4);
    *reinterpret_cast<uint2 *>(dzs + (z * kPixPosPad + L1::P) * kPixDzPitch + 4 * rem) = make_uint2(0u, 0u);
  }

  // transposed-read geometry (gemm.h StageBF16::frag): 16-lane group gq, lane i: rows (positions)
  // 16 ks + 8 (gq >> 1) + (i >> 2) (+4 for the high half), columns 16 (gq & 1) + 4 (i & 3)
  const int ti = lane & 15, gq = lane >> 4;
  const int prow = 8 * (gq >> 1) + (ti >> 2);
  const int pcol = 16 * (gq & 1) + 4 * (ti & 3);
  int scol[3];  // S offset (bf16) of this lane's 4 columns of N tile 3 nh + j: tap block + channel
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int n = 32 * (3 * nh + j) + pcol, tap = n / kS2dCh;
    scol[j] = ((tap >> 1) * kS2dSide + (tap & 1)) * kS2dPitch + (n - tap * kS2dCh);
  }

  f32x16 acc[2][3];
#pragma unroll
  for (int z = 0; z < 2; ++z)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[z][j][e] = 0.f;
  float csum[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};

  float4 pd[kPixWgDzIters];
  pix_u32x4 pf[kPixWgFrIters];
  auto prefetch = [&](int img) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < kPixWgDzIters; ++i) {
      const int e = tid + i * kPixWgThreads;
      const int ec = e < kPixDzUnits ? e : kPixDzUnits - 1;
      const int z = ec / (kPixDzUnits / 2), w = ec - z * (kPixDzUnits / 2);
      pd[i] = *reinterpret_cast<const float4 *>(q.dz[z] + static_cast<int64_t>(img) * (L1::P * L1::cout) + 4 * w);
    }
    const uint8_t *f = pix_frame(q, img);
#pragma unroll
    for (int i = 0; i < kPixWgFrIters; ++i) {
      const int u = tid + i * kPixWgThreads;
      pix_unit_load(f, u < kPixUnits ? u : kPixUnits - 1, pf[i]);
    }
  };

  if (i0 < i1) prefetch(i0);
  for (int img = i0; img < i1; ++img) {
    lds_barrier();  // every wave is done reading the previous frame's images
#pragma unroll
    for (int i = 0; i < kPixWgDzIters; ++i) {
      const int e = tid + i * kPixWgThreads;
      if (e < kPixDzUnits) {
        const int z = e / (kPixDzUnits / 2), w = e - z * (kPixDzUnits / 2);
        const int p = w >> 3, c4 = (w & 7) * 4;
        const float4 v = pd[i];
        // z is a run-time value: select instead of indexing (an indexed csum lived in scratch);
        // adding +0 to the other net's sums leaves them bitwise unchanged
        const bool z0 = z == 0;
        csum[0][0] += z0 ? v.x : 0.f;
        csum[0][1] += z0 ? v.y : 0.f;
        csum[0][2] += z0 ? v.z : 0.f;
        csum[0][3] += z0 ? v.w : 0.f;
        csum[1][0] += z0 ? 0.f : v.x;
        csum[1][1] += z0 ? 0.f : v.y;
        csum[1][2] += z0 ? 0.f : v.z;
        csum[1][3] += z0 ? 0.f : v.w;
        *reinterpret_cast<uint2 *>(dzs + (z * kPixPosPad + p) * kPixDzPitch + c4) =
            make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
      }
    }
#pragma unroll
    for (int i = 0; i < kPixWgFrIters; ++i) {
      const int u = tid + i * kPixWgThreads;
      if (u < kPixUnits) pix_unit_store(fs, u, pf[i]);
    }
    lds_barrier();
    if (img + 1 < i1) prefetch(img + 1);

#pragma unroll 1
    for (int ks = kp; ks < kPixPosPad / 16; ks += 4) {
      const int plo = 16 * ks + prow, phi = plo + 4;
      bf16x8_t a[2];
#pragma unroll
      for (int z = 0; z < 2; ++z) {
        const __bf16 *d = dzs + z * kPixPosPad * kPixDzPitch + pcol;
        a[z] = pix_tr_pair(d + plo * kPixDzPitch, d + phi * kPixDzPitch);
      }
      // S rows of positions >= 400 (zero dz) read a valid block
      const int blo = pix_block(plo < L1::P ? plo : L1::P - 1) * kS2dPitch;
      const int bhi = pix_block(phi < L1::P ? phi : L1::P - 1) * kS2dPitch;
#pragma unroll
      for (int j = 0; j < 3; ++j) {  // one B fragment at a time (an array of them sat in scratch)
        const bf16x8_t b = pix_tr_pair(fs + blo + scol[j], fs + bhi + scol[j]);
#pragma unroll
        for (int z = 0; z < 2; ++z)
          acc[z][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[z], b, acc[z][j], 0, 0, 0);
      }
    }
  }
  __syncthreads();  // LDS free for the folds

  // fold the four k-parts in order (kp 0 + 1 + 2 + 3), one net at a time, and write the slab:
  // C map row (co) = (e & 3) + 8 (e >> 2) + 4 (lane >> 5), column n = 32 (3 nh + j) + (lane & 31)
  float *scratch = reinterpret_cast<float *>(pix_lds);  // [kp - 1][nh][j][e][lane]
#pragma unroll
  for (int z = 0; z < 2; ++z) {
    if (kp > 0) {
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          scratch[((((kp - 1) * 2 + nh) * 3 + j) * 16 + e) * 64 + lane] = acc[z][j][e];
    }
    __syncthreads();
    if (kp == 0) {
      float *slab = q.slab[z] + static_cast<int64_t>(split) * q.slab_stride;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int n = 32 * (3 * nh + j) + (lane & 31);
        const int tap = n / kS2dCh, ch = n - tap * kS2dCh;
        const int dy = ch / 12, rr = ch - dy * 12, dx = rr / 3, ci = rr - dx * 3;
        const int ky = 4 * (tap >> 1) + dy, kx = 4 * (tap & 1) + dx;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          float v = acc[z][j][e];
#pragma unroll
          for (int pp = 0; pp < 3; ++pp) v += scratch[(((pp * 2 + nh) * 3 + j) * 16 + e) * 64 + lane];
          const int co = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
          slab[co * L1::kdim + ci * (L1::k * L1::k) + ky * L1::k + kx] = v;
        }
      }
    }
    __syncthreads();
  }

  // bias gradient: thread t staged channels 4 (t % 8) .. +3 of every net; fold the 64 threads of
  // a channel group in index order
  float *red = reinterpret_cast<float *>(pix_lds);  // [z][tid][4]
#pragma unroll
  for (int z = 0; z < 2; ++z)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[(z * kPixWgThreads + tid) * 4 + i] = csum[z][i];
  __syncthreads();
  if (tid < 2 * L1::cout) {
    const int z = tid / L1::cout, co = tid - z * L1::cout, grp = co >> 2, i = co & 3;
    float s = 0.f;
    for (int t = grp; t < kPixWgThreads; t += 8) s += red[(z * kPixWgThreads + t) * 4 + i];
    q.slab[z][static_cast<int64_t>(split) * q.slab_stride + L1::cout * L1::kdim + co] = s;
  }
}

}  // namespace conv
}  // namespace ppo
