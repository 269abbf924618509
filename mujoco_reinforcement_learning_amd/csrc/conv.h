// Implicit-GEMM convolutions of the pixel encoder (BASELINE.json configs[4]: dm_control
// cheetah-run, 84x84x3 pixel observations) on gfx950 MFMA.  No im2col buffer exists: the GEMM
// operands are gathered from the activation tensors as they are staged into LDS.
//
// Layouts.  Activations are HWC per image ([img][y][x][c], c contiguous); pixels are the rollout
// buffer's u8 frames, read through the minibatch row index.  The reduction index of the forward
// product is k = (ky, kx, ci) with ci innermost, so 4 consecutive k are 4 contiguous input
// elements (for the 3-channel pixel layer: a row of the 8-wide window is 24 contiguous bytes).
// Weights are kept in torch order [co][ci][ky][kx] in the flat parameter vector and repacked to
// [co][(ky kx) ci] (conv_pack_kernel) before every use.
//
// Three products per layer (G = geometry, P = output positions, PIN = input positions):
//   FWD    y[img, p, co]  = relu(sum_k im2col(x)[img, p, k] W[co, k] + b[co])
//            M = img*P, N = COUT, K = KS*KS*CIN;  A gathered from x, B = W
//   DGRAD  dx[img, q, ci] = relu'(x[img, q, ci]) * sum_{taps, co} dz[img, (q - tap)/ST, co] W[co, tap, ci]
//            split by stride phase (blockIdx.z = (py, px)): input positions q = ST*j + (py, px)
//            see exactly the taps (py + ST*ty, px + ST*tx), ty, tx < KS/ST, so
//            M = img*(HIN/ST)*(WIN/ST), N = CIN, K = (KS/ST)^2 * COUT -- no zero taps except at
//            the borders; A gathered from dz, B gathered from W
//   WGRAD  dW[co, k] = sum_{img, p} dz[img, p, co] im2col(x)[img, p, k]   (+ db = sum dz)
//            M = COUT, N = KS*KS*CIN, K = img*P split over workgroups; one f32 slab per split in
//            torch order, reduced in a fixed order afterwards (deterministic)
// The last layer's output (the flattened features) is written f32 in torch's CHW flatten order
// [img][co*P + p], which is what the first Linear layer expects, and its gradient arrives in the
// same order (DZCHW).
//
// Precision: BF = bf16 operands (RNE at staging) on v_mfma_f32_32x32x16_bf16, f32 accumulate,
// bf16 activations in HBM (exactly the values the next product rounds to); !BF = exact f32 on
// v_mfma_f32_32x32x2_f32 with f32 activations (the parity mode).  Gradients at pre-activations
// and all bias sums are f32.  Reference: none -- the reference has no pixel / CNN path
// (running_dm_control.py:56-91 is state-observation), see DESIGN.md.
#pragma once

#include "gemm.h"

namespace ppo {
namespace conv {

template <int HIN, int WIN, int CIN, int COUT, int KS, int ST>
struct Geo {
  static constexpr int hin = HIN, win = WIN, cin = CIN, cout = COUT, k = KS, s = ST;
  static constexpr int hout = (HIN - KS) / ST + 1, wout = (WIN - KS) / ST + 1;
  static constexpr int P = hout * wout, PIN = HIN * WIN;
  static constexpr int kdim = KS * KS * CIN;
  static constexpr int tk = KS / ST;                  // DGRAD taps per dimension and phase
  static constexpr int hq = HIN / ST, wq = WIN / ST;  // DGRAD positions per dimension and phase
  static_assert(KS % ST == 0 && HIN % ST == 0 && WIN % ST == 0, "phase decomposition");
  static_assert(COUT % 32 == 0, "output channels: multiple of 32");
  static_assert((KS * CIN) % 4 == 0, "a window row must be whole 4-element units");
};

// The Nature-DQN encoder on 84x84x3 pixels (the encoder this engine declares).
using L1 = Geo<84, 84, 3, 32, 8, 4>;   // -> 20x20x32
using L2 = Geo<20, 20, 32, 64, 4, 2>;  // -> 9x9x64
using L3 = Geo<9, 9, 64, 64, 3, 1>;    // -> 7x7x64 = 3136 features
constexpr int kFeatures = L3::P * L3::cout;

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };
constexpr int kWgradMaxFrames = 1024;  // frames one WGRAD split may span (host-checked)

struct ConvNet {
  const void *in;       // layer input: u8 pixel frames (through rows) / bf16 / f32 HWC
  const float *w;       // packed weights [COUT][(ky kx) ci]
  const float *bias;    // FWD (nullable)
  void *out;            // FWD: HWC activation (bf16 / f32) or, for the last layer, CHW f32 features
  const float *dz;      // DGRAD / WGRAD: f32 gradient at this layer's pre-activation
  float *dout;          // DGRAD: f32 gradient at the previous layer's pre-activation (HWC)
  float *slab;          // WGRAD: split 0 of this layer's slabs: dW [COUT][CIN][KS][KS], then db
  int has_bias;
};

struct ConvArgs {
  ConvNet net[2];
  int nimg;
  const int32_t *rows;   // pixel input: image j is frame rows[j] of `in` (null: frame j)
  int splits;            // WGRAD
  int64_t slab_stride;   // WGRAD: floats between splits
};

// ---- element access ----------------------------------------------------------------------------
__device__ __forceinline__ void load4(const uint8_t *p, float (&o)[4]) {
  const uint32_t u = *reinterpret_cast<const uint32_t *>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = static_cast<float>((u >> (8 * j)) & 255u) / 255.f;  // x / 255
}
__device__ __forceinline__ void load4(const __bf16 *p, float (&o)[4]) {
  const uint2 u = *reinterpret_cast<const uint2 *>(p);
  o[0] = __uint_as_float(u.x << 16);
  o[1] = __uint_as_float(u.x & 0xffff0000u);
  o[2] = __uint_as_float(u.y << 16);
  o[3] = __uint_as_float(u.y & 0xffff0000u);
}
__device__ __forceinline__ void load4(const float *p, float (&o)[4]) {
  const float4 v = *reinterpret_cast<const float4 *>(p);
  o[0] = v.x, o[1] = v.y, o[2] = v.z, o[3] = v.w;
}
__device__ __forceinline__ float load1(const uint8_t *p) { return static_cast<float>(*p) / 255.f; }
__device__ __forceinline__ float load1(const __bf16 *p) {
  return __uint_as_float(static_cast<uint32_t>(*reinterpret_cast<const uint16_t *>(p)) << 16);
}
__device__ __forceinline__ float load1(const float *p) { return *p; }
__device__ __forceinline__ void store1(__bf16 *p, float v) {
  *reinterpret_cast<uint16_t *>(p) = static_cast<uint16_t>(pack_bf16x2(v, 0.f) & 0xffffu);
}
__device__ __forceinline__ void store1(float *p, float v) { *p = v; }
__device__ __forceinline__ void zero4(float (&o)[4]) { o[0] = o[1] = o[2] = o[3] = 0.f; }

// ---- one operand's LDS image -----------------------------------------------------------------
// KC: [R][k] (k contiguous; a unit = 4 consecutive k of one row); !KC: [k][R] (a unit = 4
// consecutive rows of one k).  BF: the bf16 images / fragment reads of gemm.h's StageBF16;
// !BF: f32 images padded so the 32x32x2 fragment reads are conflict-free.
template <int R, int BK, int NT, bool KC, bool BF>
struct Img {
  using SB = StageBF16<R, BK, NT, 4, KC>;
  static constexpr int NU = R * BK / (4 * NT);
  static_assert((R * BK) % (4 * NT) == 0, "tile / thread mismatch");
  static constexpr int FROW = KC ? BK + 1 : R + 4;     // f32 image row stride (floats)
  static constexpr int BYTES = BF ? SB::IMAGE * 2 : (KC ? R : BK) * FROW * 4;
  __device__ __forceinline__ static void coords(int e, int &rr, int &kk) {
    if (KC) {
      kk = (e % (BK / 4)) * 4;
      rr = e / (BK / 4);
    } else {
      rr = (e % (R / 4)) * 4;
      kk = e / (R / 4);
    }
  }
  __device__ __forceinline__ static void store(char *img, int rr, int kk, const float (&v)[4]) {
    if constexpr (BF) {
      __bf16 *s = reinterpret_cast<__bf16 *>(img);
      __bf16 *dst = KC ? s + rr * SB::ROW + kk : s + kk * SB::ROW + rr;
      *reinterpret_cast<uint2 *>(dst) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    } else {
      float *s = reinterpret_cast<float *>(img);
      if (KC) {
#pragma unroll
        for (int j = 0; j < 4; ++j) s[rr * FROW + kk + j] = v[j];
      } else {
        *reinterpret_cast<float4 *>(s + kk * FROW + rr) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
  // bf16: the 32x32x16 fragment of rows r0.., k-step ks; f32: the 32x32x2 operand of k-pair kp
  __device__ __forceinline__ static bf16x8 frag16(const char *img, int r0, int ks, int lane) {
    return SB::frag(reinterpret_cast<const __bf16 *>(img), r0, ks, lane);
  }
  __device__ __forceinline__ static float frag2(const char *img, int r0, int kp, int lane) {
    const float *s = reinterpret_cast<const float *>(img);
    const int r = r0 + (lane & 31), k = 2 * kp + (lane >> 5);
    return KC ? s[r * FROW + k] : s[k * FROW + r];
  }
};

// ---- the kernel ---------------------------------------------------------------------------------
// TIN: storage of the layer input (uint8_t pixels, __bf16 / float activations); TOUT: FWD output
// storage (ignored by OUTCHW, which writes f32 features).  DZCHW: dz is in the CHW flatten order
// (the last layer, whose gradient comes from the first Linear layer).
template <class G, int MODE, typename TIN, typename TOUT, bool BF, bool DZCHW, bool OUTCHW, int WM,
          int WN, int TM, int TN, int BK>
__global__ __launch_bounds__(64 * WM * WN) void conv_kernel(ConvArgs q) {
  constexpr int NT = 64 * WM * WN;
  constexpr int BM = 32 * TM * WM;
  constexpr int BN = 32 * TN * WN;
  constexpr bool AKC = MODE != MODE_WGRAD;  // A [m][k]: im2col rows (FWD), dz gather (DGRAD)
  constexpr bool BKC = MODE == MODE_FWD;    // B [n][k]: weights (FWD); [k][n] otherwise
  using IA = Img<BM, BK, NT, AKC, BF>;
  using IB = Img<BN, BK, NT, BKC, BF>;
  constexpr int NCLS = MODE == MODE_DGRAD ? G::s * G::s : 1;
  static_assert(BK % 16 == 0, "BK");
  __shared__ __attribute__((aligned(16))) char lds[2 * (IA::BYTES + IB::BYTES)];
  __shared__ int sframe[MODE == MODE_WGRAD ? kWgradMaxFrames : 1];  // WGRAD: the split's rows[]

  // DGRAD: blockIdx.x enumerates (tile, stride-phase class).  The s^2 classes of one row tile read
  // the same images' dz, so they run on one XCD at the same time (blocks b, b + 8, ... share an
  // XCD and its L2): dz streams from HBM once per launch instead of once per class.
  const int z = static_cast<int>(blockIdx.z);
  int cls = 0, bx = static_cast<int>(blockIdx.x);
  if constexpr (NCLS > 1) {
    const int tiles_all = ((q.nimg * G::hq * G::wq + BM - 1) / BM) * ((G::cin + BN - 1) / BN);
    const int b = bx;
    if (tiles_all % 8 == 0) {
      cls = (b / 8) % NCLS;
      bx = (b % 8) + 8 * (b / (8 * NCLS));
    } else {
      cls = b % NCLS;
      bx = b / NCLS;
    }
  }
  const int py = cls / G::s, px = cls % G::s;
  const ConvNet &Nt = q.net[z];
  const TIN *const xin = static_cast<const TIN *>(Nt.in);
  const int M = MODE == MODE_FWD ? q.nimg * G::P
              : MODE == MODE_DGRAD ? q.nimg * G::hq * G::wq : G::cout;
  constexpr int N = MODE == MODE_FWD ? G::cout : MODE == MODE_DGRAD ? G::cin : G::kdim;
  const int K = MODE == MODE_FWD ? G::kdim
              : MODE == MODE_DGRAD ? G::tk * G::tk * G::cout : q.nimg * G::P;
  int tile_m, tile_n, wsplit = 0;
  if constexpr (NCLS > 1) {  // the class map above already groups a tile's work on one XCD
    const int tn = (N + BN - 1) / BN;
    if (bx >= ((M + BM - 1) / BM) * tn) return;
    tile_m = bx / tn;
    tile_n = bx - tile_m * tn;
  } else if constexpr (MODE == MODE_WGRAD) {
    // blockIdx.x enumerates (split, tile): every tile of a split reads the same positions' dz and
    // frames, so they go to one XCD (split s on XCD s % 8) -- the layer's dz and inputs stream from
    // HBM once per launch instead of once per tile
    const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN, tiles = tm * tn;
    if (bx >= tiles * q.splits) return;
    int id;
    if (q.splits % 8 == 0) {
      const int x = bx % 8, j = bx / 8;
      wsplit = x + 8 * (j / tiles);
      id = j % tiles;
    } else {
      wsplit = bx / tiles;
      id = bx % tiles;
    }
    tile_m = id / tn;
    tile_n = id - tile_m * tn;
  } else {
    if (!xcd_tile(bx, (M + BM - 1) / BM, (N + BN - 1) / BN, tile_m, tile_n)) return;
  }
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  int kbeg = 0, kend = K;
  const int split = MODE == MODE_WGRAD ? wsplit : 0;
  if (MODE == MODE_WGRAD) {
    kbeg = static_cast<int>((static_cast<int64_t>(split) * K) / q.splits);
    kend = static_cast<int>((static_cast<int64_t>(split + 1) * K) / q.splits);
  }
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;

  // first element of image img's receptive field for output position p (row-invariant part of
  // the im2col gather)
  auto field = [&](int img, int p) -> const TIN * {
    const int oy = p / G::wout, ox = p - oy * G::wout;
    const int64_t frame = q.rows ? static_cast<int64_t>(q.rows[img]) : img;
    return xin + frame * (G::PIN * G::cin) + (G::s * oy * G::win + G::s * ox) * G::cin;
  };
  // WGRAD over minibatch frames (the pixel layer): the split's frame indices rows[img] staged in
  // LDS once, so a k-tile's im2col gathers are one global round trip, not a dependent index load
  // followed by the pixel load
  int img0 = 0;
  if constexpr (MODE == MODE_WGRAD) {
    if (q.rows) {
      img0 = kbeg / G::P;
      const int nimg_split = (kend > kbeg ? (kend - 1) / G::P : img0) - img0 + 1;
      for (int i = tid; i < nimg_split; i += NT) sframe[i] = q.rows[img0 + i];
      __syncthreads();  // uniform (q.rows is a kernel argument)
    }
  }
  auto field_w = [&](int img, int p) -> const TIN * {
    const int oy = p / G::wout, ox = p - oy * G::wout;
    const int64_t frame = q.rows ? static_cast<int64_t>(sframe[img - img0]) : img;
    return xin + frame * (G::PIN * G::cin) + (G::s * oy * G::win + G::s * ox) * G::cin;
  };
  // 4 consecutive reduction columns c..c+3 of an im2col row (one window row: contiguous)
  auto im2col4 = [&](const TIN *f, int c, float (&o)[4]) {
    const int ky = c / (G::k * G::cin);
    load4(f + ky * G::win * G::cin + (c - ky * G::k * G::cin), o);
  };
  // dz at (img, output position p), channels co..co+3
  auto dz4 = [&](int img, int p, int co, float (&o)[4]) {
    if (DZCHW) {
      const float *d = Nt.dz + static_cast<int64_t>(img) * (G::cout * G::P) + co * G::P + p;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = d[j * G::P];
    } else {
      load4(Nt.dz + (static_cast<int64_t>(img) * G::P + p) * G::cout + co, o);
    }
  };

  // ---- per-unit row state, fixed across k-steps -------------------------------------------
  float va[IA::NU][4], vb[IB::NU][4];
  // Every gather below loads unconditionally from a clamped, in-bounds address and masks the value
  // (a load under a branch makes the compiler drain every earlier load at the merge, so a k-tile's
  // NU gathers would run one memory round trip after another; DESIGN.md s4 "loads behind branches")
  const TIN *arow[IA::NU];  // FWD: receptive field of the unit's row
  bool arow_ok[IA::NU];
  int aimg[IA::NU], ajy[IA::NU], ajx[IA::NU];  // DGRAD: the unit row's image / phase position
  if constexpr (MODE == MODE_FWD) {
#pragma unroll
    for (int u = 0; u < IA::NU; ++u) {
      int rr, kk;
      IA::coords(tid + u * NT, rr, kk);
      const int m = m0 + rr;
      const int mc = m < M ? m : M - 1;  // clamped: every gather loads, masked at use
      arow[u] = field(mc / G::P, mc % G::P);
      arow_ok[u] = m < M;
    }
  }
  if constexpr (MODE == MODE_DGRAD) {
#pragma unroll
    for (int u = 0; u < IA::NU; ++u) {
      int rr, kk;
      IA::coords(tid + u * NT, rr, kk);
      const int m = m0 + rr;
      const int img = m / (G::hq * G::wq), j = m - img * (G::hq * G::wq);
      aimg[u] = m < M ? img : -1;
      ajy[u] = j / G::wq;
      ajx[u] = j - (j / G::wq) * G::wq;
    }
  }

  auto mask4 = [](bool ok, float (&o)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = ok ? o[j] : 0.f;
  };
  auto gload = [&](int k0) {
#pragma unroll
    for (int u = 0; u < IA::NU; ++u) {
      int rr, kk;
      IA::coords(tid + u * NT, rr, kk);
      if constexpr (MODE == MODE_FWD) {
        im2col4(arow[u], k0 + kk, va[u]);
        mask4(arow_ok[u], va[u]);
      } else if constexpr (MODE == MODE_DGRAD) {
        const int c = k0 + kk, t = c / G::cout, co = c - t * G::cout;
        const int oy = ajy[u] - t / G::tk, ox = ajx[u] - t % G::tk;
        const bool ok = aimg[u] >= 0 && oy >= 0 && oy < G::hout && ox >= 0 && ox < G::wout;
        dz4(ok ? aimg[u] : 0, ok ? oy * G::wout + ox : 0, co, va[u]);
        mask4(ok, va[u]);
      } else {  // WGRAD: A[k = position][m = co]
        const int kr = k0 + kk;
        const bool ok = kr < kend;
        const int kc = ok ? kr : kbeg;
        dz4(kc / G::P, kc % G::P, m0 + rr, va[u]);
        mask4(ok, va[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < IB::NU; ++u) {
      int rr, kk;
      IB::coords(tid + u * NT, rr, kk);
      if constexpr (MODE == MODE_FWD) {  // B[n = co][k]
        load4(Nt.w + static_cast<int64_t>(n0 + rr) * G::kdim + k0 + kk, vb[u]);
      } else if constexpr (MODE == MODE_DGRAD) {  // B[k = (t, co)][n = ci]
        const int c = k0 + kk, t = c / G::cout, co = c - t * G::cout;
        const int ky = py + G::s * (t / G::tk), kx = px + G::s * (t % G::tk);
        load4(Nt.w + static_cast<int64_t>(co) * G::kdim + (ky * G::k + kx) * G::cin + n0 + rr, vb[u]);
      } else {  // WGRAD: B[k = position][n = (tap, ci)]
        const int kr = k0 + kk, c = n0 + rr;
        const bool ok = kr < kend && c < N;
        const int kc = ok ? kr : kbeg;
        im2col4(field_w(kc / G::P, kc % G::P), ok ? c : 0, vb[u]);
        mask4(ok, vb[u]);
      }
    }
  };
  auto lstore = [&](int buf) {
    char *a = lds + buf * (IA::BYTES + IB::BYTES);
    char *b = a + IA::BYTES;
#pragma unroll
    for (int u = 0; u < IA::NU; ++u) {
      int rr, kk;
      IA::coords(tid + u * NT, rr, kk);
      IA::store(a, rr, kk, va[u]);
    }
#pragma unroll
    for (int u = 0; u < IB::NU; ++u) {
      int rr, kk;
      IB::coords(tid + u * NT, rr, kk);
      IB::store(b, rr, kk, vb[u]);
    }
  };

  // WGRAD bias gradient: column sums of dz (f32, before rounding); a thread's A units share one
  // 4-column group (NT % (BM/4) == 0), combined in a fixed order after the k loop
  constexpr bool COLSUM = MODE == MODE_WGRAD;
  float csum[4] = {0.f, 0.f, 0.f, 0.f};
  auto colsum = [&]() {
    if constexpr (COLSUM) {
#pragma unroll
      for (int u = 0; u < IA::NU; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) csum[j] += va[u][j];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int ntiles = (kend - kbeg + BK - 1) / BK;
  if (ntiles > 0) {
    gload(kbeg);
    colsum();
    lstore(0);
  }
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < ntiles; ++kt) {
    if (kt + 1 < ntiles) gload(kbeg + (kt + 1) * BK);
    const char *As = lds + cur * (IA::BYTES + IB::BYTES);
    const char *Bs = As + IA::BYTES;
    if constexpr (BF) {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 av[TM], bv[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) av[i] = IA::frag16(As, (wm * TM + i) * 32, ks, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bv[j] = IB::frag16(Bs, (wn * TN + j) * 32, ks, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kp = 0; kp < BK / 2; ++kp) {
        float av[TM], bv[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) av[i] = IA::frag2(As, (wm * TM + i) * 32, kp, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bv[j] = IB::frag2(Bs, (wn * TN + j) * 32, kp, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    }
    if (kt + 1 < ntiles) {
      colsum();
      lstore(cur ^ 1);
    }
    __syncthreads();
    cur ^= 1;
  }

  // ---- epilogue (32x32 C map: row (r&3) + 8(r>>2) + 4(lane>>5), column lane&31) ------------
  const int64_t sb = static_cast<int64_t>(split) * q.slab_stride;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + (wn * TN + j) * 32 + (lane & 31);
      float bias = 0.f;
      if (MODE == MODE_FWD && Nt.bias) {
        const float bv = Nt.bias[n < N ? n : N - 1];
        bias = n < N ? bv : 0.f;
      }
      // DGRAD: the 16 activation operands of act' first, from clamped addresses (no load behind
      // the bounds test), then the stores
      float yv[16];
      if constexpr (MODE == MODE_DGRAD) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const int mc = m < M ? m : M - 1, nc = n < N ? n : N - 1;
          const int img = mc / (G::hq * G::wq), jj = mc - img * (G::hq * G::wq);
          const int qy = py + G::s * (jj / G::wq), qx = px + G::s * (jj % G::wq);
          yv[r] = load1(xin + (static_cast<int64_t>(img) * G::PIN + qy * G::win + qx) * G::cin + nc);
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= M || n >= N) continue;
        const float v = acc[i][j][r];
        if constexpr (MODE == MODE_FWD) {
          const float y = act_forward(v + bias, PPO_ACT_RELU);
          if constexpr (OUTCHW) {
            const int img = m / G::P, p = m - img * G::P;
            static_cast<float *>(Nt.out)[static_cast<int64_t>(img) * (G::cout * G::P) + n * G::P + p] = y;
          } else {
            store1(static_cast<TOUT *>(Nt.out) + static_cast<int64_t>(m) * G::cout + n, y);
          }
        } else if constexpr (MODE == MODE_DGRAD) {
          const int img = m / (G::hq * G::wq), jj = m - img * (G::hq * G::wq);
          const int qy = py + G::s * (jj / G::wq), qx = px + G::s * (jj % G::wq);
          const int64_t e = (static_cast<int64_t>(img) * G::PIN + qy * G::win + qx) * G::cin + n;
          Nt.dout[e] = act_backward(v, yv[r], PPO_ACT_RELU);
        } else {
          const int tap = n / G::cin, ci = n - tap * G::cin;
          Nt.slab[sb + static_cast<int64_t>(m) * G::kdim + ci * (G::k * G::k) + tap] = v;
        }
      }
    }
  }
  if constexpr (COLSUM) {
    constexpr int GR = BM / 4, PARTS = NT / GR;
    static_assert(NT % GR == 0, "colsum layout");
    if (!Nt.has_bias || tile_n != 0) return;  // uniform per block
    float *red = reinterpret_cast<float *>(lds);  // the k loop is over (trailing barrier)
    const int grp = tid % GR, part = tid / GR;
#pragma unroll
    for (int j = 0; j < 4; ++j) red[part * BM + 4 * grp + j] = csum[j];
    __syncthreads();
    if (tid < BM && m0 + tid < M) {
      float s = 0.f;
      for (int p = 0; p < PARTS; ++p) s += red[p * BM + tid];
      Nt.slab[sb + static_cast<int64_t>(G::cout) * G::kdim + m0 + tid] = s;
    }
  }
}

// Torch-order weights [COUT][CIN][KS][KS] -> packed [COUT][(ky kx) ci] for every layer of both
// nets (one launch: blockIdx.y = layer * 2 + net).
struct PackArgs {
  const float *src[6];
  float *dst[6];
  int cout[6], cin[6], k[6];
};
__global__ __launch_bounds__(256) void conv_pack_kernel(PackArgs a) {
  const int l = blockIdx.y;
  const int co_n = a.cout[l], ci_n = a.cin[l], ks = a.k[l];
  const int per = ci_n * ks * ks;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= static_cast<int64_t>(co_n) * per) return;
  const int co = static_cast<int>(i / per), r = static_cast<int>(i % per);
  const int tap = r / ci_n, ci = r % ci_n;
  a.dst[l][i] = a.src[l][static_cast<int64_t>(co) * per + ci * ks * ks + tap];
}

}  // namespace conv
}  // namespace ppo
