// Input gradients of the encoder's inner layers (conv.h L2: 20x20x32 -> 9x9x64 k4 s2, L3:
// 9x9x64 -> 7x7x64 k3 s1) in bf16 mode, one image at a time with the gradient image in LDS.
//
// Product.  A stride-S layer with a KS = S*T kernel is, on the space-to-depth image of its input
// (S x S blocks, N = S*S*CIN values per block), a stride-1 T x T convolution, so its transpose is
//   dX[b = (by, bx)][n = (dy, dx, ci)] = sum_{ty, tx} sum_co dz[by - ty, bx - tx][co] W[co, ci, S ty + dy, S tx + dx]
// with dz = 0 outside the ZD x ZD output grid: per image a GEMM of M = OB^2 blocks (OB = WIN / S),
// N, K = T^2 * 64 whose dz operand rows are 8 consecutive channels of one padded grid cell.  L2:
// S 2, T 2, N 128, K 256, 100 blocks; L3: S 1, T 3, N 64, K 576, 81 positions.  The conv.h DGRAD
// gathers its operands from global memory 4 channels at a time and splits by stride phase; here
// the image's dz is staged once (bf16, RNE -- the value conv.h stages) into a zero-bordered
// ZP x ZP grid (ZP = OB + T - 1) and every fragment is one 16-B LDS read.
//
// dgrad_lds_kernel: persistent workgroups of 8 waves, one image per iteration (the next image's
// dz prefetched into registers during the products); wave (z, group, part) = net z, N tiles
// NTW*group .. +NTW-1 (W'^T fragments in registers, from the bf16 pack of dg_pack_kernel), block
// tiles part, part + PSPLIT, ...; the transposed product dX^T[n][b] = W'^T[n][k] dz^T[k][b] on
// v_mfma_f32_16x16x32_bf16, so a lane's 4 accumulators are 4 consecutive input channels of one
// input pixel: relu' from the layer input (8-B bf16 load), one 16-B f32 store.
// Reference: none (the reference has no pixel path).
#pragma once

#include "conv.h"
#include "conv_pixel.h"

namespace ppo {
namespace conv {

template <int CIN_, int WIN_, int S_, int T_, int ZD_, bool DZCHW_, int NTW_, int PSPLIT_>
struct DgGeo {
  static constexpr int CIN = CIN_, WIN = WIN_, S = S_, T = T_, ZD = ZD_, NTW = NTW_, PSPLIT = PSPLIT_;
  static constexpr bool DZCHW = DZCHW_;
  static constexpr int CO = 64;
  static constexpr int KS = S * T;                  // kernel size
  static constexpr int OB = WIN / S;                // blocks per dimension
  static constexpr int M = OB * OB;                 // blocks
  static constexpr int PT = (M + 15) / 16;          // block tiles
  static constexpr int N = S * S * CIN;             // values per block
  static constexpr int NT = N / 16;                 // N tiles
  static constexpr int KD = T * T * CO;             // reduction length
  static constexpr int KSTEPS = KD / 32;
  static constexpr int PAD = T - 1;
  static constexpr int ZP = OB + T - 1;             // padded grid
  static constexpr int PITCH = CO + 8;              // bf16 per grid cell (144 B)
  static constexpr int ZDZ = ZD * ZD * CO;          // dz floats per image
  static_assert(WIN % S == 0 && (WIN - KS) / S + 1 == ZD, "geometry");
  static_assert((NT / NTW) * PSPLIT == 4, "four waves per net");
};
using L2D = DgGeo<32, 20, 2, 2, 9, false, 2, 1>;
using L3D = DgGeo<64, 9, 1, 3, 7, true, 2, 2>;
static_assert(L2D::KS == L2::k && L2D::CIN == L2::cin && L2D::ZD == L2::hout, "L2");
static_assert(L3D::KS == L3::k && L3D::CIN == L3::cin && L3D::ZD == L3::hout, "L3");

struct DgArgs {
  const __bf16 *wt[2];   // W'^T [N][KD] bf16 (dg_pack_kernel)
  const float *dz[2];    // gradient at the layer's pre-activation: HWC [img][ZD^2][64] or CHW
  const __bf16 *xin[2];  // layer input activations, HWC bf16 [img][WIN^2][CIN] (relu')
  float *dout[2];        // gradient at the previous layer's pre-activation, HWC f32
  int nimg;
};

// W'^T[z][n][k] = bf16(W[co][ci][S ty + dy][S tx + dx]), n = (dy S + dx) CIN + ci, k = (ty T + tx) 64 + co
template <class D>
__global__ __launch_bounds__(256) void dg_pack_kernel(const float *w0, const float *w1, __bf16 *o0,
                                                      __bf16 *o1) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (e >= 2LL * D::N * D::KD) return;
  const int z = static_cast<int>(e / (D::N * D::KD));
  const int rem = static_cast<int>(e - static_cast<int64_t>(z) * D::N * D::KD);
  const int n = rem / D::KD, k = rem - n * D::KD;
  const int blk = n / D::CIN, ci = n - blk * D::CIN, dy = blk / D::S, dx = blk - dy * D::S;
  const int tap = k / D::CO, co = k - tap * D::CO, ty = tap / D::T, tx = tap - ty * D::T;
  const int ky = D::S * ty + dy, kx = D::S * tx + dx;
  const float v = (z ? w1 : w0)[((co * D::CIN + ci) * D::KS + ky) * D::KS + kx];
  (z ? o1 : o0)[rem] = __builtin_bit_cast(__bf16, static_cast<uint16_t>(pack_bf16x2(v, 0.f) & 0xffffu));
}

template <class D>
struct DgStage {
  static constexpr int NTH = 512;
  static constexpr int UNITS = D::DZCHW ? 2 * D::ZDZ : 2 * D::ZDZ / 4;  // floats / float4s
  static constexpr int ITERS = (UNITS + NTH - 1) / NTH;
  static constexpr int LDS = 2 * D::ZP * D::ZP * D::PITCH * 2;
  // relu' of the layer input: one bit per element (bit set where !(x <= 0), act_backward's
  // pass condition), built from the prefetched bf16 input, 8 elements per 16-B unit and byte
  static constexpr int XUNITS = 2 * D::WIN * D::WIN * D::CIN / 8;
  static constexpr int XITERS = (XUNITS + NTH - 1) / NTH;
  static constexpr int MASK = XUNITS;                // bytes, both nets
};

typedef __bf16 dg_bf16x8 __attribute__((ext_vector_type(8)));
// 16-B staging registers: a clang vector, not HIP's uint4 struct -- arrays of the struct were kept
// in scratch memory (ScratchSize 48-128 B per lane) instead of registers
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef float dg_f32x4 __attribute__((ext_vector_type(4)));

template <class D>
__global__ __launch_bounds__(512) void dgrad_lds_kernel(DgArgs q) {
  using St = DgStage<D>;
  __shared__ __attribute__((aligned(16))) __bf16 dzs[St::LDS / 2];  // [z][ZP*ZP][PITCH]
  __shared__ uint8_t xmask[St::MASK];                                 // [z][element / 8]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int z = wv >> 2, wz = wv & 3;
  const int grp = wz / D::PSPLIT, part = wz - grp * D::PSPLIT;

  for (int e = tid; e < St::LDS / 16; e += 512) reinterpret_cast<uint4 *>(dzs)[e] = make_uint4(0u, 0u, 0u, 0u);

  // W'^T fragments of this wave's N tiles: lane holds W'^T[16 nt + c][32 ks + 8 g .. +7]
  dg_bf16x8 wf[D::NTW][D::KSTEPS];
#pragma unroll
  for (int j = 0; j < D::NTW; ++j)
#pragma unroll
    for (int ks = 0; ks < D::KSTEPS; ++ks)
      wf[j][ks] = *reinterpret_cast<const dg_bf16x8 *>(
          q.wt[z] + static_cast<int64_t>(16 * (D::NTW * grp + j) + c) * D::KD + 32 * ks + 8 * g);

  float pre[St::ITERS][D::DZCHW ? 1 : 4];
  uint4 prex[St::XITERS];
  auto prefetch = [&](int img) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < St::XITERS; ++i) {
      const int u = tid + i * 512;
      const int uc = u < St::XUNITS ? u : St::XUNITS - 1;
      const int zz = uc / (St::XUNITS / 2), w = uc - zz * (St::XUNITS / 2);
      prex[i] = *reinterpret_cast<const uint4 *>(q.xin[zz] + static_cast<int64_t>(img) * (D::WIN * D::WIN * D::CIN) + 8 * w);
    }
#pragma unroll
    for (int i = 0; i < St::ITERS; ++i) {
      const int e = tid + i * 512;
      const int ec = e < St::UNITS ? e : St::UNITS - 1;
      const int zz = ec / (St::UNITS / 2), w = ec - zz * (St::UNITS / 2);
      const float *src = q.dz[zz] + static_cast<int64_t>(img) * D::ZDZ;
      if constexpr (D::DZCHW) {
        pre[i][0] = src[w];
      } else {
        const float4 v = *reinterpret_cast<const float4 *>(src + 4 * w);
        pre[i][0] = v.x, pre[i][1] = v.y, pre[i][2] = v.z, pre[i][3] = v.w;
      }
    }
  };
  auto stage = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < St::XITERS; ++i) {
      const int u = tid + i * 512;
      if (u < St::XUNITS) {
        const uint32_t w4[4] = {prex[i].x, prex[i].y, prex[i].z, prex[i].w};
        uint32_t bits = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t h = (w4[j >> 1] >> (16 * (j & 1))) & 0xffffu;
          bits |= (__uint_as_float(h << 16) <= 0.f ? 0u : 1u) << j;
        }
        xmask[u] = static_cast<uint8_t>(bits);
      }
    }
#pragma unroll
    for (int i = 0; i < St::ITERS; ++i) {
      const int e = tid + i * 512;
      if (e < St::UNITS) {
        const int zz = e / (St::UNITS / 2), w = e - zz * (St::UNITS / 2);
        if constexpr (D::DZCHW) {  // w = co * ZD^2 + p
          const int co = w / (D::ZD * D::ZD), p = w - co * (D::ZD * D::ZD);
          const int py = p / D::ZD, px = p - py * D::ZD;
          dzs[(zz * D::ZP * D::ZP + (py + D::PAD) * D::ZP + px + D::PAD) * D::PITCH + co] =
              __builtin_bit_cast(__bf16, static_cast<uint16_t>(pack_bf16x2(pre[i][0], 0.f) & 0xffffu));
        } else {  // w = p * 16 + channel quad
          const int p = w >> 4, c4 = (w & 15) * 4;
          const int py = p / D::ZD, px = p - py * D::ZD;
          *reinterpret_cast<uint2 *>(dzs + (zz * D::ZP * D::ZP + (py + D::PAD) * D::ZP + px + D::PAD) * D::PITCH + c4) =
              make_uint2(pack_bf16x2(pre[i][0], pre[i][1]), pack_bf16x2(pre[i][2], pre[i][3]));
        }
      }
    }
  };

  int img = blockIdx.x;
  if (img < q.nimg) prefetch(img);
  __syncthreads();  // the zeroed borders before any interior store
  for (; img < q.nimg; img += gridDim.x) {
    lds_barrier();  // every wave is done reading the previous image's grid and mask
    stage();
    lds_barrier();
    if (img + static_cast<int>(gridDim.x) < q.nimg) prefetch(img + gridDim.x);
    const __bf16 *grid = dzs + z * D::ZP * D::ZP * D::PITCH;
    const uint8_t *mk = xmask + z * (St::XUNITS / 2);
#pragma unroll 1
    for (int pt = part; pt < D::PT; pt += D::PSPLIT) {
      const int m = 16 * pt + c;
      const int mc = m < D::M ? m : D::M - 1;
      const int by = mc / D::OB, bx = mc - by * D::OB;
      const __bf16 *cell = grid + ((by + D::PAD) * D::ZP + bx + D::PAD) * D::PITCH;
      dg_f32x4 acc[D::NTW];
#pragma unroll
      for (int j = 0; j < D::NTW; ++j) acc[j] = dg_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < D::KSTEPS; ++ks) {
        const int k0 = 32 * ks + 8 * g, tap = k0 / D::CO, co0 = k0 - tap * D::CO;
        const int ty = tap / D::T, tx = tap - ty * D::T;
        const dg_bf16x8 b = *reinterpret_cast<const dg_bf16x8 *>(cell - (ty * D::ZP + tx) * D::PITCH + co0);
#pragma unroll
        for (int j = 0; j < D::NTW; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][ks], b, acc[j], 0, 0, 0);
      }
      if (m < D::M) {
#pragma unroll
        for (int j = 0; j < D::NTW; ++j) {
          const int n = 16 * (D::NTW * grp + j) + 4 * g;  // rows n .. n+3: 4 channels of one pixel
          const int blk = n / D::CIN, ci = n - blk * D::CIN, dy = blk / D::S, dx = blk - dy * D::S;
          const int el = ((D::S * by + dy) * D::WIN + D::S * bx + dx) * D::CIN + ci;  // ci % 4 == 0
          const uint32_t bits = static_cast<uint32_t>(mk[el >> 3]) >> (el & 7);
          *reinterpret_cast<float4 *>(q.dout[z] + static_cast<int64_t>(img) * (D::WIN * D::WIN * D::CIN) + el) =
              make_float4((bits & 1u) ? acc[j][0] : 0.f, (bits & 2u) ? acc[j][1] : 0.f,
                          (bits & 4u) ? acc[j][2] : 0.f, (bits & 8u) ? acc[j][3] : 0.f);
        }
      }
    }
  }
}


// ==============================================================================================
// Forward and weight gradient of L2 / L3 on the space-to-depth image of the layer input.
//
// The input image (bf16 HWC, both nets) is staged into LDS as S x S blocks of NIN = S*S*CIN values
// (PITCH = NIN + 8 bf16 per block).  With k = tap * NIN + n over the T x T taps of the
// stride-1 form, the forward is y[p][co] = sum_k W'[co][k] S[p + tap][n] (M = HO^2 output
// positions, K = T^2 NIN) and the weight gradient dW'[co][k] = sum_p dz[p][co] S[p + tap][n].
//   fwd_lds_kernel    persistent, one image per iteration; wave (z, group, part) = net z, output
//                     channel tiles NTW*group .. (W' fragments in registers), position tiles part,
//                     part + PSPLIT, ...; transposed product on v_mfma_f32_16x16x32_bf16: a lane
//                     holds 4 consecutive channels of one position (L2: one 8-B bf16 HWC store;
//                     L3: the f32 features in torch's CHW flatten order).
//   wgrad_lds_kernel  one split of the minibatch per workgroup, the split's dW of both nets in
//                     registers (wave (z, group): N tiles group, group + 4, ... of 32 columns, both
//                     64-channel halves); dz staged bf16 [p][co] after its f32 column sums (the
//                     bias gradient); both operands by ds_read_b64_tr_b16 on
//                     v_mfma_f32_32x32x16_bf16 over 16-position k-steps; the slab in torch order.
// ==============================================================================================
template <int CIN_, int WIN_, int S_, int T_, bool OUTCHW_, int NTW_, int PSPLIT_>
struct FwGeo {
  static constexpr int CIN = CIN_, WIN = WIN_, S = S_, T = T_, NTW = NTW_, PSPLIT = PSPLIT_;
  static constexpr bool OUTCHW = OUTCHW_;
  static constexpr int CO = 64;
  static constexpr int KS = S * T;
  static constexpr int OBI = WIN / S;               // input blocks per dimension
  static constexpr int NIN = S * S * CIN;           // values per block
  static constexpr int PITCH = NIN + 8;
  static constexpr int HO = OBI - T + 1;            // output positions per dimension
  static constexpr int M = HO * HO;
  static constexpr int PT = (M + 15) / 16;
  static constexpr int KD = T * T * NIN;
  static constexpr int KSTEPS = KD / 32;
  static constexpr int IMG = WIN * WIN * CIN;       // input bf16 per image
  static constexpr int UNITS = 2 * IMG / 8;         // 16-B units of both nets' inputs
  static constexpr int SIMG = OBI * OBI * PITCH;    // staged bf16 per net
  // wgrad: 32-column N tiles over K, 16-position k-steps
  static constexpr int NT32 = KD / 32;
  static constexpr int NPW = (NT32 + 3) / 4;        // N tiles per wave (interleaved)
  static constexpr int MP = (M + 15) / 16 * 16;     // padded positions
  static constexpr int DZPITCH = CO + 32;           // bf16 per dz row (tr-read banks)
  static constexpr int DZIMG = MP * DZPITCH;
  static_assert(WIN % S == 0 && (WIN - KS) / S + 1 == HO, "geometry");
  static_assert((CO / 16 / NTW) * PSPLIT == 4, "four waves per net");
  static_assert(NIN % 32 == 0, "a 32-column tile stays inside one tap");
};
using L2F = FwGeo<32, 20, 2, 2, false, 2, 2>;
using L3F = FwGeo<64, 9, 1, 3, true, 2, 2>;
static_assert(L2F::HO == L2::hout && L2F::KS == L2::k && L2F::KD == L2::kdim, "L2");
static_assert(L3F::HO == L3::hout && L3F::KS == L3::k && L3F::KD == L3::kdim, "L3");

struct FwArgs {
  const __bf16 *wp[2];   // FWD: W' [64][KD] bf16 (fw_pack_kernel)
  const float *bias[2];
  const __bf16 *xin[2];  // layer input activations, HWC bf16 [img][WIN^2][CIN]
  void *out[2];          // FWD: L2 bf16 HWC [img][HO^2][64]; L3 f32 CHW [img][64 * HO^2]
  const float *dz[2];    // WGRAD: gradient at the pre-activation (L2 HWC, L3 CHW), f32
  float *slab[2];        // WGRAD: split 0 of the layer's slabs (dW torch order, then db)
  int64_t slab_stride;
  int splits;
  int nimg;
};

// W'[z][co][k] = bf16(W[co][ci][S ty + dy][S tx + dx]), k = (ty T + tx) NIN + (dy S + dx) CIN + ci
template <class D>
__device__ __forceinline__ int fw_w_offset(int co, int k) {
  const int tap = k / D::NIN, n = k - tap * D::NIN, ty = tap / D::T, tx = tap - ty * D::T;
  const int blk = n / D::CIN, ci = n - blk * D::CIN, dy = blk / D::S, dx = blk - dy * D::S;
  return ((co * D::CIN + ci) * D::KS + D::S * ty + dy) * D::KS + D::S * tx + dx;
}

template <class D>
__global__ __launch_bounds__(256) void fw_pack_kernel(const float *w0, const float *w1, __bf16 *o0,
                                                      __bf16 *o1) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= 2 * D::CO * D::KD) return;
  const int z = e / (D::CO * D::KD), rem = e - z * (D::CO * D::KD);
  const int co = rem / D::KD, k = rem - co * D::KD;
  const float v = (z ? w1 : w0)[fw_w_offset<D>(co, k)];
  (z ? o1 : o0)[rem] = __builtin_bit_cast(__bf16, static_cast<uint16_t>(pack_bf16x2(v, 0.f) & 0xffffu));
}

// 16-B unit u of both nets' input images -> its block slot in the staged image
template <class D>
__device__ __forceinline__ int fw_unit_slot(int u, int &z) {
  z = u / (D::UNITS / 2);
  const int w = u - z * (D::UNITS / 2);
  const int pix = w / (D::CIN / 8), c8 = (w - pix * (D::CIN / 8)) * 8;
  const int y = pix / D::WIN, x = pix - y * D::WIN;
  const int blk = (y / D::S) * D::OBI + x / D::S, seg = (y % D::S) * D::S + x % D::S;
  return z * D::SIMG + blk * D::PITCH + seg * D::CIN + c8;
}

template <class D>
__global__ __launch_bounds__(512) void fwd_lds_kernel(FwArgs q) {
  constexpr int ITERS = (D::UNITS + 511) / 512;
  __shared__ __attribute__((aligned(16))) __bf16 sx[2 * D::SIMG];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int z = wv >> 2, wz = wv & 3;
  const int grp = wz / D::PSPLIT, part = wz - grp * D::PSPLIT;

  dg_bf16x8 wf[D::NTW][D::KSTEPS];
  float bias[D::NTW][4];
#pragma unroll
  for (int j = 0; j < D::NTW; ++j) {
    const int co = 16 * (D::NTW * grp + j);
#pragma unroll
    for (int ks = 0; ks < D::KSTEPS; ++ks)
      wf[j][ks] = *reinterpret_cast<const dg_bf16x8 *>(q.wp[z] + (co + c) * D::KD + 32 * ks + 8 * g);
#pragma unroll
    for (int i = 0; i < 4; ++i) bias[j][i] = q.bias[z][co + 4 * g + i];
  }

  u32x4_t pre[ITERS];
  auto prefetch = [&](int img) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < ITERS; ++i) {
      const int u = tid + i * 512;
      const int uc = u < D::UNITS ? u : D::UNITS - 1;
      const int zz = uc / (D::UNITS / 2), w = uc - zz * (D::UNITS / 2);
      pre[i] = *reinterpret_cast<const u32x4_t *>(q.xin[zz] + static_cast<int64_t>(img) * D::IMG + 8 * w);
    }
  };
  int img = blockIdx.x;
  if (img < q.nimg) prefetch(img);
  for (; img < q.nimg; img += gridDim.x) {
    lds_barrier();
#pragma unroll
    for (int i = 0; i < ITERS; ++i) {
      const int u = tid + i * 512;
      if (u < D::UNITS) {
        int zz;
        *reinterpret_cast<u32x4_t *>(sx + fw_unit_slot<D>(u, zz)) = pre[i];
      }
    }
    lds_barrier();
    if (img + static_cast<int>(gridDim.x) < q.nimg) prefetch(img + gridDim.x);
    const __bf16 *im = sx + z * D::SIMG;
#pragma unroll 1
    for (int pt = part; pt < D::PT; pt += D::PSPLIT) {
      const int p = 16 * pt + c;
      const int pc = p < D::M ? p : D::M - 1;
      const int oy = pc / D::HO, ox = pc - oy * D::HO;
      const __bf16 *cell = im + (oy * D::OBI + ox) * D::PITCH;
      dg_f32x4 acc[D::NTW];
#pragma unroll
      for (int j = 0; j < D::NTW; ++j) acc[j] = dg_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < D::KSTEPS; ++ks) {
        const int k0 = 32 * ks + 8 * g, tap = k0 / D::NIN, n0 = k0 - tap * D::NIN;
        const int ty = tap / D::T, tx = tap - ty * D::T;
        const dg_bf16x8 b = *reinterpret_cast<const dg_bf16x8 *>(cell + (ty * D::OBI + tx) * D::PITCH + n0);
#pragma unroll
        for (int j = 0; j < D::NTW; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][ks], b, acc[j], 0, 0, 0);
      }
      if (p < D::M) {
#pragma unroll
        for (int j = 0; j < D::NTW; ++j) {
          const int co = 16 * (D::NTW * grp + j) + 4 * g;
          float y[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) y[i] = act_forward(acc[j][i] + bias[j][i], PPO_ACT_RELU);
          if constexpr (D::OUTCHW) {
            float *o = static_cast<float *>(q.out[z]) + static_cast<int64_t>(img) * (D::CO * D::M) + co * D::M + p;
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i * D::M] = y[i];
          } else {
            __bf16 *o = static_cast<__bf16 *>(q.out[z]) + (static_cast<int64_t>(img) * D::M + p) * D::CO + co;
            *reinterpret_cast<uint2 *>(o) = make_uint2(pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3]));
          }
        }
      }
    }
  }
}

template <class D>
__global__ __launch_bounds__(512) void wgrad_lds_kernel(FwArgs q) {
  constexpr int XITERS = (D::UNITS + 511) / 512;
  // dz units: HWC float4s (thread's channel quad fixed: tid % 16); CHW: thread (z, co, sub) reads
  // positions sub, sub + 4, ... of one channel row (its bias sum stays in one register)
  constexpr int DZU = 2 * D::M * D::CO / 4;
  constexpr int DITERS = D::OUTCHW ? (D::M + 3) / 4 : (DZU + 511) / 512;
  static_assert(!D::OUTCHW || 2 * D::CO * 4 == 512, "CHW staging: 4 threads per channel row");
  constexpr int SX_BYTES = 2 * D::SIMG * 2;
  __shared__ __attribute__((aligned(16))) char lds[SX_BYTES + 2 * D::DZIMG * 2];
  __bf16 *sx = reinterpret_cast<__bf16 *>(lds);
  __bf16 *sd = reinterpret_cast<__bf16 *>(lds + SX_BYTES);  // [z][MP][DZPITCH]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int z = wv >> 2, grp = wv & 3;
  const int split = blockIdx.x;
  const int i0 = static_cast<int>((static_cast<int64_t>(split) * q.nimg) / q.splits);
  const int i1 = static_cast<int>((static_cast<int64_t>(split + 1) * q.nimg) / q.splits);

  // zero the padded positions M .. MP-1 of both dz images (never staged)
  for (int e = tid; e < 2 * (D::MP - D::M) * D::DZPITCH / 8; e += 512) {
    const int per = (D::MP - D::M) * D::DZPITCH / 8, zz = e / per, w = e - zz * per;
    *reinterpret_cast<uint4 *>(sd + zz * D::DZIMG + D::M * D::DZPITCH + 8 * w) = make_uint4(0u, 0u, 0u, 0u);
  }

  // tr-read geometry (gemm.h StageBF16::frag): 16-lane group gq, lane i
  const int ti = lane & 15, gq = lane >> 4;
  const int prow = 8 * (gq >> 1) + (ti >> 2);
  const int pcol = 16 * (gq & 1) + 4 * (ti & 3);
  // this lane's column offset (bf16) in the staged image for each of the wave's N tiles
  int ncol[D::NPW];
#pragma unroll
  for (int j = 0; j < D::NPW; ++j) {
    const int t = grp + 4 * j, tt = t < D::NT32 ? t : 0;
    const int k = 32 * tt + pcol, tap = k / D::NIN, ty = tap / D::T, tx = tap - ty * D::T;
    ncol[j] = (ty * D::OBI + tx) * D::PITCH + (k - tap * D::NIN);
  }

  f32x16 acc[2][D::NPW];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < D::NPW; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[h][j][e] = 0.f;
  float csum[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};  // HWC: channel quad tid % 16
  float crow = 0.f;                                                  // CHW: this thread's row
  const int cz = tid >> 8, cco = (tid >> 2) & 63, csub = tid & 3;

  u32x4_t px[XITERS];
  float pd[DITERS][D::OUTCHW ? 1 : 4];
  auto prefetch = [&](int img) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < XITERS; ++i) {
      const int u = tid + i * 512;
      const int uc = u < D::UNITS ? u : D::UNITS - 1;
      const int zz = uc / (D::UNITS / 2), w = uc - zz * (D::UNITS / 2);
      px[i] = *reinterpret_cast<const u32x4_t *>(q.xin[zz] + static_cast<int64_t>(img) * D::IMG + 8 * w);
    }
#pragma unroll
    for (int i = 0; i < DITERS; ++i) {
      if constexpr (D::OUTCHW) {
        const int pp = csub + 4 * i;
        pd[i][0] = q.dz[cz][static_cast<int64_t>(img) * (D::M * D::CO) + cco * D::M + (pp < D::M ? pp : D::M - 1)];
      } else {
        const int e = tid + i * 512;
        const int ec = e < DZU ? e : DZU - 1;
        const int zz = ec / (DZU / 2), w = ec - zz * (DZU / 2);
        const float4 v = *reinterpret_cast<const float4 *>(q.dz[zz] + static_cast<int64_t>(img) * (D::M * D::CO) + 4 * w);
        pd[i][0] = v.x, pd[i][1] = v.y, pd[i][2] = v.z, pd[i][3] = v.w;
      }
    }
  };

  if (i0 < i1) prefetch(i0);
  for (int img = i0; img < i1; ++img) {
    lds_barrier();
#pragma unroll
    for (int i = 0; i < XITERS; ++i) {
      const int u = tid + i * 512;
      if (u < D::UNITS) {
        int zz;
        *reinterpret_cast<u32x4_t *>(sx + fw_unit_slot<D>(u, zz)) = px[i];
      }
    }
#pragma unroll
    for (int i = 0; i < DITERS; ++i) {
      if constexpr (D::OUTCHW) {
        const int pp = csub + 4 * i;
        if (pp < D::M) {
          crow += pd[i][0];
          sd[cz * D::DZIMG + pp * D::DZPITCH + cco] =
              __builtin_bit_cast(__bf16, static_cast<uint16_t>(pack_bf16x2(pd[i][0], 0.f) & 0xffffu));
        }
        continue;
      }
      const int e = tid + i * 512;
      if (e < DZU) {
        const int zz = e / (DZU / 2), w = e - zz * (DZU / 2);
        if constexpr (!D::OUTCHW) {  // w = p * 16 + channel quad (= tid % 16)
          const int p = w >> 4, c4 = (w & 15) * 4;
#pragma unroll
          for (int j = 0; j < 4; ++j) {  // zz is a run-time value: select, not index
            csum[0][j] += zz == 0 ? pd[i][j] : 0.f;
            csum[1][j] += zz == 0 ? 0.f : pd[i][j];
          }
          *reinterpret_cast<uint2 *>(sd + zz * D::DZIMG + p * D::DZPITCH + c4) =
              make_uint2(pack_bf16x2(pd[i][0], pd[i][1]), pack_bf16x2(pd[i][2], pd[i][3]));
        }
      }
    }
    lds_barrier();
    if (img + 1 < i1) prefetch(img + 1);

    const __bf16 *im = sx + z * D::SIMG;
    const __bf16 *dzi = sd + z * D::DZIMG;
#pragma unroll 1
    for (int ks = 0; ks < D::MP / 16; ++ks) {
      const int plo = 16 * ks + prow, phi = plo + 4;
      bf16x8_t a[2];
#pragma unroll
      for (int h = 0; h < 2; ++h)
        a[h] = pix_tr_pair(dzi + plo * D::DZPITCH + 32 * h + pcol, dzi + phi * D::DZPITCH + 32 * h + pcol);
      const int qlo = plo < D::M ? plo : D::M - 1, qhi = phi < D::M ? phi : D::M - 1;
      const int ylo = qlo / D::HO, yhi = qhi / D::HO;
      const int clo = (ylo * D::OBI + qlo - ylo * D::HO) * D::PITCH;
      const int chi = (yhi * D::OBI + qhi - yhi * D::HO) * D::PITCH;
#pragma unroll
      for (int j = 0; j < D::NPW; ++j) {
        if (grp + 4 * j < D::NT32) {
          const bf16x8_t b = pix_tr_pair(im + clo + ncol[j], im + chi + ncol[j]);
#pragma unroll
          for (int h = 0; h < 2; ++h)
            acc[h][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[h], b, acc[h][j], 0, 0, 0);
        }
      }
    }
  }

  // the slab: C map row (co within half h) = (e & 3) + 8 (e >> 2) + 4 (lane >> 5), column lane & 31
  float *slab = q.slab[z] + static_cast<int64_t>(split) * q.slab_stride;
#pragma unroll
  for (int j = 0; j < D::NPW; ++j) {
    const int t = grp + 4 * j;
    if (t < D::NT32) {
      const int k = 32 * t + (lane & 31);
      const int off = fw_w_offset<D>(0, k);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int co = 32 * h + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
          slab[co * D::KD + off] = acc[h][j][e];
        }
    }
  }

  // bias gradient (f32, before rounding), folded in a fixed order
  __syncthreads();
  float *red = reinterpret_cast<float *>(lds);
  if constexpr (D::OUTCHW) {
    (void)csum;
    red[tid] = crow;
    __syncthreads();
    if (tid < 2 * D::CO) {  // (z, co) row: its 4 sub-sums in order
      const float s = ((red[4 * tid] + red[4 * tid + 1]) + red[4 * tid + 2]) + red[4 * tid + 3];
      const int zz = tid / D::CO, co = tid - zz * D::CO;
      q.slab[zz][static_cast<int64_t>(split) * q.slab_stride + D::CO * D::KD + co] = s;
    }
  } else {
#pragma unroll
    for (int zz = 0; zz < 2; ++zz)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(zz * 512 + tid) * 4 + i] = csum[zz][i];
    __syncthreads();
    if (tid < 2 * D::CO) {
      const int zz = tid / D::CO, co = tid - zz * D::CO, quad = co >> 2, i = co & 3;
      float s = 0.f;
      for (int t = quad; t < 512; t += 16) s += red[(zz * 512 + t) * 4 + i];
      q.slab[zz][static_cast<int64_t>(split) * q.slab_stride + D::CO * D::KD + co] = s;
    }
  }
}

}  // namespace conv
}  // namespace ppo
