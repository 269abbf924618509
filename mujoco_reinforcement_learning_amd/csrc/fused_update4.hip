// The fused minibatch update (ppo.py:109-135) re-decomposed for ReLU
// nets: ONE wave per SIMD (4 waves, up to 512 registers each) and 128-row chunks, so every weight
// fragment streamed from L2 and every activation fragment read from LDS feeds twice the MFMAs of
// the 8-wave / 64-row kernel in fused_update.hip.
//
// Per 64 rows the 8-wave kernel's L1 and dgrad passes sat at ~3.2 k cycles against a 2,048-cycle
// MFMA floor, co-limited by the W1 stream (128 KB per pass per CU at ~64 B/clk) and the LDS
// B-operand reads (8 waves x 64 rows x 512 B at 128 B/clk).  Here a wave owns 64 output features
// (two 32-feature MFMA tiles) for 128 rows (four row tiles): per 128 rows the W1 stream is 128 KB
// (2,048 cycles) and the B reads 4 x 128 x 512 B (2,048 cycles) against 4,096 MFMA cycles.
//
// Registers (per lane): dW1 16 tiles (256) + dW0 2 tiles (32) + head dW 4 16x16 tiles (16),
// persistent; the pass accumulators 8 tiles (128), the W1 fragment ring and the B operands.
//
// LDS (158.5 KB): the A1 / D1 image (D1 written in place over A1 once dW1 has read A1), the A2 /
// D2 image (D2 in place over A2), the head image, biases and head constants, one 8 KB region that
// holds the chunk's row scalars during the forward / loss phases and its X image for dW0, and the
// dz images, whose 8.4 KB also park the NEXT chunk's X image between its prefetch and its L0 pass.
//
// Numerics are those of fused_update_kernel (oracle.use_bf16_gemms): bf16 operands of every fc
// product with f32 accumulation; biases, ReLU', the loss heads and every bias gradient in f32.
// Summation orders differ from fused_update_kernel (the head z is one K=256 chain here), so the
// two kernels agree to f32 rounding, not bitwise; each is bitwise deterministic run to run.
#include <cstdlib>
#include <type_traits>

#include "fused_common.h"

namespace ppo {

using namespace fu;

namespace f4 {

constexpr int H = 256;
constexpr int RR = 128;            // rows per chunk
constexpr int NW4 = 4;             // waves per workgroup: one per SIMD
constexpr int NT4 = 64 * NW4;
constexpr int PITCH = 2 * H;       // A1 / A2 image row pitch (bytes)
constexpr int DZTP = 2 * (RR + 8); // head-major dz image pitch (bytes)
constexpr int KS = H / 16;         // k-steps of a 32x32x16 pass over H
// Latency hiding with one wave per SIMD: PD = weight-ring prefetch distance (k-steps), BD =
// B-operand lookahead (k-steps).  Compiled configurations (ppo_ctx_fused_variant / PPO_F4_CFG):
// 0 = (7, 1), 1 = (3, 4), 2 = (7, 2).
template <int PD_, int BD_>
struct Cfg4 {
  static constexpr int PD = PD_, P = PD_ + 1, BD = BD_;
  static_assert(KS % P == 0, "ring period must divide the k-steps");
  static_assert(P % BD == 0, "B slots must cycle within a ring period");
};

struct Lds4 {
  static constexpr int WHB = 0;                              // bf16 head image [16][H + 8]
  static constexpr int BIAS = WHB + HeadImg<H>::BYTES;       // f32 b0[H], b1[H]
  static constexpr int HS = BIAS + 2 * H * 4;                // f32 head bias, logstd, log std, 1/var, 1/(2 var)
  static constexpr int S = HS + 80 * 4;                      // SROW [128][16] f32 (phases 2-4) / X image (5-7)
  static constexpr int IMG1 = S + RR * 64;                   // A1, then D1 in place
  static constexpr int IMG2 = IMG1 + RR * PITCH;             // A2, then D2 in place
  static constexpr int DZ = IMG2 + RR * PITCH;               // dz [128][16] bf16 (phases 4-5)
  static constexpr int DZT = DZ + RR * kDzRowBytes;          // dz^T [16][128 + 8] bf16
  static constexpr int XN = DZ;                              // the next chunk's X image (phases 6a-1)
  static constexpr int TOTAL = DZT + 16 * DZTP;
  static constexpr int RED = IMG1;                           // epilogue: f32 [4 waves][16][4]
  static_assert(TOTAL <= 163840, "LDS budget");
  static_assert(TOTAL - XN >= RR * 64, "the X image fits the dz region");
  static_assert(S % 16 == 0 && IMG1 % 16 == 0 && IMG2 % 16 == 0 && DZ % 16 == 0 && DZT % 16 == 0,
                "16-B aligned regions");
};

__device__ __forceinline__ uint16_t bf16_bits4(float x) { return static_cast<uint16_t>(pack2(x, 0.f) & 0xffffu); }

// dW1 accumulation pinned to AGPRs: the 16 dW1 tiles (256 registers) fill the AGPR half of the
// unified file, everything else lives in VGPRs.  Through inline asm the compiler cannot move these
// accumulators (its allocator otherwise splits the MFMA accumulators of both kinds across the two
// halves and spills).  The leading s_nop 1 covers a VALU write of an operand right before the MFMA
// (the hazard recognizer does not see into the asm); srcC = dst chains need no wait states.
__device__ __forceinline__ void mfma_agpr(f32x16 &acc, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// every other accumulator (pass tiles, dW0, head dW, head z) pinned to VGPRs the same way
__device__ __forceinline__ f32x16 mfma_v(const bf16x8 &a, const bf16x8 &b, f32x16 acc) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  return acc;
}
__device__ __forceinline__ f32x4 mfma16_v(const bf16x8 &a, const bf16x8 &b, f32x4 acc) {
  asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  return acc;
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int e = 0; e < 16; ++e) z[e] = 0.f;
  return z;
}

// 18 wait states before VALU reads of the last 32x32x16 results (fused_common.h mfma_drain), as a
// scheduling fence: no register operands, so the accumulators may stay in AGPRs
__device__ __forceinline__ void drain_fence() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int NACC>
__device__ __forceinline__ void drain8(f32x16 (&)[2][NACC]) { drain_fence(); }

// acc[f][rt] += W[64w + 32(ft0 + f) + r][:] . img[32rt + r][:] over k = 0..H-1 for f < NF: A
// operands from the fragment-major bf16 weight image (wf = the first tile's base for this lane),
// B operands 16-B row reads of the LDS image (row tile t's next k-step read issued as soon as its
// MFMAs have issued); weights C::PD k-steps ahead through the ring.
template <int NF, class C>
__device__ __forceinline__ void pass4(const __bf16 *wf, const char *img, int r, int h,
                                      bf16x8 (&ring)[C::P][NF], f32x16 (&acc)[NF][4]) {
  const int swz = ((r & 3) << 2) | ((r >> 2) & 3);
  const char *rowp = img + r * PITCH;
  constexpr int64_t STEP = 16 * H;  // elements per k-step of the fragment-major image
  constexpr int64_t TILE = 64 * 8;  // elements per 32-feature tile of one k-step
  // B operands BD k-steps ahead: slot s % BD holds k-step s; row tile t's read of step s + BD is
  // issued right after its MFMAs of step s (one wave per SIMD: nothing else hides LDS latency)
  bf16x8 bq[C::BD][4];
#pragma unroll
  for (int j = 0; j < C::BD; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) bq[j][t] = lds_b128(rowp + t * 32 * PITCH + 16 * ((2 * j + h) ^ swz));
#pragma unroll 1
  for (int s0 = 0; s0 < KS - C::P; s0 += C::P) {
#pragma unroll
    for (int u = 0; u < C::P; ++u) {
      const int s = s0 + u;
      bf16x8 a[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        a[f] = ring[u][f];
        ring[(u + C::PD) % C::P][f] = *reinterpret_cast<const bf16x8 *>(wf + STEP * (s + C::PD) + TILE * f);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int f = 0; f < NF; ++f) acc[f][t] = mfma_v(a[f], bq[u % C::BD][t], acc[f][t]);
        bq[u % C::BD][t] = lds_b128(rowp + t * 32 * PITCH + 16 * ((2 * (s + C::BD) + h) ^ swz));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // last period peeled: no weight prefetch past the end, no B read past the last k-step
#pragma unroll
  for (int u = 0; u < C::P; ++u) {
    const int s = KS - C::P + u;
    bf16x8 a[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      a[f] = ring[u][f];
      if (s + C::PD < KS)
        ring[(u + C::PD) % C::P][f] = *reinterpret_cast<const bf16x8 *>(wf + STEP * (s + C::PD) + TILE * f);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int f = 0; f < NF; ++f) acc[f][t] = mfma_v(a[f], bq[u % C::BD][t], acc[f][t]);
      if (s + C::BD < KS) bq[u % C::BD][t] = lds_b128(rowp + t * 32 * PITCH + 16 * ((2 * (s + C::BD) + h) ^ swz));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  drain_fence();
}

template <int NF, class C>
__device__ __forceinline__ void ring_prime4(const __bf16 *wf, bf16x8 (&ring)[C::P][NF]) {
#pragma unroll
  for (int s = 0; s < C::PD; ++s)
#pragma unroll
    for (int f = 0; f < NF; ++f)
      ring[s][f] = *reinterpret_cast<const bf16x8 *>(wf + static_cast<int64_t>(16 * H) * s + 64 * 8 * f);
}

// bias + ReLU of the accumulators of feature tiles ft0..ft0+NF-1 -> bf16 image columns
template <int NF>
__device__ __forceinline__ void store_act(char *img, const float *bias, f32x16 (&acc)[NF][4],
                                          int w, int ft0, int r, int h) {
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ft = ft0 + f;
      const float4 bv = *reinterpret_cast<const float4 *>(bias + 64 * w + 32 * ft + 8 * g + 4 * h);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float y0 = act_forward(acc[f][t][4 * g] + bv.x, PPO_ACT_RELU);
        const float y1 = act_forward(acc[f][t][4 * g + 1] + bv.y, PPO_ACT_RELU);
        const float y2 = act_forward(acc[f][t][4 * g + 2] + bv.z, PPO_ACT_RELU);
        const float y3 = act_forward(acc[f][t][4 * g + 3] + bv.w, PPO_ACT_RELU);
        *reinterpret_cast<uint2 *>(img + img_off(32 * t + r, 8 * w + 4 * ft + g, PITCH) + 8 * h) =
            make_uint2(pack2(y0, y1), pack2(y2, y3));
      }
    }
}

// d = acc * ReLU'(y) with y the image's activation, written over it in place; the bias gradient
// (sum over the chunk's rows) accumulated per feature in gb[ft] (rs16 layout)
template <int NF>
__device__ __forceinline__ void backward_in_place(char *img, f32x16 (&acc)[NF][4], float (&gb)[2],
                                                  int w, int ft0, int lane) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int ft = ft0 + f;
    // every activation read issued before any write: the compiler cannot prove the swizzled
    // addresses distinct, so interleaved read / write pairs would each wait out an LDS round trip
    uint2 yv[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        yv[t][g] = *reinterpret_cast<const uint2 *>(img + img_off(32 * t + r, 8 * w + 4 * ft + g, PITCH) + 8 * h);
    float bsum[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) bsum[e] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float d0 = act_backward(acc[f][t][4 * g], bf_lo(yv[t][g].x), PPO_ACT_RELU);
        const float d1 = act_backward(acc[f][t][4 * g + 1], bf_hi(yv[t][g].x), PPO_ACT_RELU);
        const float d2 = act_backward(acc[f][t][4 * g + 2], bf_lo(yv[t][g].y), PPO_ACT_RELU);
        const float d3 = act_backward(acc[f][t][4 * g + 3], bf_hi(yv[t][g].y), PPO_ACT_RELU);
        bsum[4 * g] += d0;
        bsum[4 * g + 1] += d1;
        bsum[4 * g + 2] += d2;
        bsum[4 * g + 3] += d3;
        yv[t][g] = make_uint2(pack2(d0, d1), pack2(d2, d3));
      }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<uint2 *>(img + img_off(32 * t + r, 8 * w + 4 * ft + g, PITCH) + 8 * h) = yv[t][g];
    gb[ft] += rs16(bsum, lane);
  }
}

// One net's workgroup.  NH: head width (actor A padded, or 1), ACTOR selects the loss head.
template <int NH, bool ACTOR, int NF, class C, bool STAMP>
__device__ __forceinline__ void body4(const FusedArgs &q, const FusedNet &N, char *lds) {
  using L = Lds4;
  constexpr int z = ACTOR ? 0 : 1;
  char *const whb = lds + L::WHB;
  const float *const b0s = reinterpret_cast<const float *>(lds + L::BIAS);
  const float *const b1s = b0s + H;
  const float *const hbias = reinterpret_cast<const float *>(lds + L::HS);
  char *const simg = lds + L::S;
  char *const img1 = lds + L::IMG1;
  char *const img2 = lds + L::IMG2;
  char *const dzimg = lds + L::DZ;
  char *const dztimg = lds + L::DZT;
  char *const xnimg = lds + L::XN;

  const int tid0 = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  int tid = tid0, lane = tid & 63, r = lane & 31, h = lane >> 5;
  // Lane-derived LDS addresses are loop-invariant across chunks; re-deriving them from an opaque
  // copy of the thread id in every phase keeps the compiler from hoisting (and spilling) dozens of
  // them out of the chunk loop (as fused_update.hip does).
#define OPAQUE_LANE()           \
  tid = tid0;                   \
  asm volatile("" : "+v"(tid)); \
  lane = tid & 63;              \
  r = lane & 31;                \
  h = lane >> 5
  // STAMP (diagnostic build, ppo_ctx_phase_stamps): s_memtime deltas per phase segment summed over
  // the chunks (wave 0's view; a segment ending at a barrier includes the wait for the others)
  uint64_t t_prev = 0, t_real0 = 0, t_acc[kStampSlots];
  if constexpr (STAMP) {
#pragma unroll
    for (int k = 0; k < kStampSlots; ++k) t_acc[k] = 0;
    t_prev = __builtin_amdgcn_s_memtime();
    t_real0 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
#define STAMP4(k)                                         \
  if constexpr (STAMP) {                                  \
    const uint64_t t_now = __builtin_amdgcn_s_memtime();  \
    t_acc[k] += t_now - t_prev;                           \
    t_prev = t_now;                                       \
  }
  const int A = q.act_dim;
  const int G = q.G;
  const int nchunks = (q.b + RR - 1) / RR;
  const int count = q.rows_n ? *q.rows_n : q.b;

  stage_head_image<H>(whb, N.wh, ACTOR ? A : 1, tid, NT4);
  for (int i = tid; i < 2 * H; i += NT4) {
    const float *b = i < H ? N.b0 : N.b1;
    (reinterpret_cast<float *>(lds + L::BIAS))[i] = b ? b[i % H] : 0.f;
  }
  if (tid < 32) {
    const int a = tid & 15;
    const bool ok = a < (ACTOR ? A : 1);
    (reinterpret_cast<float *>(lds + L::HS))[tid] =
        tid < 16 ? ((ok && N.bh) ? N.bh[a] : 0.f) : ((ACTOR && ok) ? q.logstd[a] : 0.f);
  }
  if (tid < 16) {  // per-head Normal constants: log(std), 1/var, 1/(2 var); std = exp(logstd)
    const bool ok = ACTOR && tid < A;
    const float sd = ok ? expf(q.logstd[tid]) : 1.f;
    const float var = sd * sd;
    (reinterpret_cast<float *>(lds + L::HS))[32 + tid] = ok ? logf(sd) : 0.f;
    (reinterpret_cast<float *>(lds + L::HS))[48 + tid] = 1.f / var;
    (reinterpret_cast<float *>(lds + L::HS))[64 + tid] = 1.f / (2.f * var);
  }

  // 32 B of a chunk's staged states (bf16 [row][32]) / row scalars (f32 [row][16]) per thread:
  // row tid >> 1, half tid & 1; rows past the minibatch read row 0 and are zeroed
  auto load_x = [&](int c, uint4 (&v)[2]) {
    const int xrow = tid >> 1, xhalf = tid & 1;
    const int j = c * RR + xrow;
    const bool ok = c < nchunks && j < q.b;
    const uint4 *src = reinterpret_cast<const uint4 *>(q.xb + static_cast<int64_t>(ok ? j : 0) * kFusedKX) + 2 * xhalf;
    v[0] = src[0];
    v[1] = src[1];
    if (!ok) v[0] = v[1] = make_uint4(0u, 0u, 0u, 0u);
  };
  auto store_x = [&](char *img, const uint4 (&v)[2]) {
    const int xrow = tid >> 1, xhalf = tid & 1;
    *reinterpret_cast<uint4 *>(img + x_off(xrow, 2 * xhalf)) = v[0];
    *reinterpret_cast<uint4 *>(img + x_off(xrow, 2 * xhalf + 1)) = v[1];
  };
  auto load_srow = [&](int c, uint4 (&v)[2]) {
    const int xrow = tid >> 1, xhalf = tid & 1;
    const int j = c * RR + xrow;
    const bool ok = j < q.b;
    const uint4 *src = reinterpret_cast<const uint4 *>(q.srow + static_cast<int64_t>(ok ? j : 0) * kFusedSP) + 2 * xhalf;
    v[0] = src[0];
    v[1] = src[1];
    if (!ok) v[0] = v[1] = make_uint4(0u, 0u, 0u, 0u);
  };

  // ---- persistent accumulators ----
  f32x16 gw1[2][8];  // dW1 tiles: o-tiles 2w + a (the wave's features), i-tiles b = 0..7
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) gw1[a][b] = zero16();
  f32x16 gw0[2];     // dW0 tiles: features 64w + 32ft.., input columns 0..31
  gw0[0] = zero16();
  gw0[1] = zero16();
  f32x4 ghw[4];      // head dW: heads 4 (lane >> 4) + i, features 64w + 16j + (lane & 15)
#pragma unroll
  for (int j = 0; j < 4; ++j) ghw[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float gb1[2] = {0.f, 0.f}, gb0[2] = {0.f, 0.f};   // rs16-scattered bias grads per feature tile
  // loss-head partials of this lane's (row, head) pairs: heads 2k + (tid >> 7), k < KP
  constexpr int KP = NH > 1 ? NH / 2 : 1;
  float g_bh[KP], g_ls[KP], g_loss = 0.f;
#pragma unroll
  for (int k = 0; k < KP; ++k) g_bh[k] = g_ls[k] = 0.f;


  int chunk = blockIdx.x;
  {
    uint4 xv[2];
    load_x(chunk, xv);
    store_x(xnimg, xv);
  }
  __syncthreads();
  STAMP4(0);

  bf16x8 ring[C::P][NF];
  f32x16 acc[NF][4];
  for (; chunk < nchunks; chunk += G) {
    // ---- phase 1: a1 = relu(W0 x + b0) -> A1 image; the row scalars issued; W1 ring primed ----
    OPAQUE_LANE();
    uint4 sv[2];
    load_srow(chunk, sv);
    {
      // every operand issued up front (one wave per SIMD: no partner hides a load's latency)
      bf16x8 w0f[2][2], xb[2][4];
#pragma unroll
      for (int ft = 0; ft < 2; ++ft)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          w0f[ft][s] = *reinterpret_cast<const bf16x8 *>(N.w0b + (64 * w + 32 * ft + r) * kFusedKX + 16 * s + 8 * h);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int t = 0; t < 4; ++t) xb[s][t] = lds_b128(xnimg + x_off(32 * t + r, 2 * s + h));
#pragma unroll
      for (int ft0 = 0; ft0 < 2; ft0 += NF) {
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[f][t] = zero16();
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int f = 0; f < NF; ++f) acc[f][t] = mfma_v(w0f[ft0 + f][s], xb[s][t], acc[f][t]);
        if (ft0 + NF >= 2) ring_prime4<NF, C>(w_frag_base<H>(N.w1b, 2 * w, lane), ring);  // for phase 2
        drain_fence();
        store_act<NF>(img1, b0s, acc, w, ft0, r, h);
      }
    }
    STAMP4(1);
    __syncthreads();
    STAMP4(2);

    // ---- phase 2: a2 = W1 a1; the row scalars staged (the S region is free) ----
    OPAQUE_LANE();
    *reinterpret_cast<uint4 *>(simg + (tid >> 1) * 64 + 32 * (tid & 1)) = sv[0];
    *reinterpret_cast<uint4 *>(simg + (tid >> 1) * 64 + 32 * (tid & 1) + 16) = sv[1];
#pragma unroll
    for (int ft0 = 0; ft0 < 2; ft0 += NF) {
#pragma unroll
      for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[f][t] = zero16();
      pass4<NF, C>(w_frag_base<H>(N.w1b, 2 * w + ft0, lane), img1, r, h, ring, acc);
      if (ft0 + NF < 2) ring_prime4<NF, C>(w_frag_base<H>(N.w1b, 2 * w + ft0 + NF, lane), ring);
      // ---- phase 3: bias + ReLU -> A2 image ----
      OPAQUE_LANE();
      store_act<NF>(img2, b1s, acc, w, ft0, r, h);
    }
    STAMP4(3);
    __syncthreads();
    STAMP4(4);

    // ---- phase 4: head z = a2 . W_h^T on the 16x16x32 MFMA (wave w: rows 32w..32w+31 as two
    //      16-row tiles, lane -> head lane & 15), z staged in LDS, then the loss head over DENSE
    //      (row, head) pairs: lane -> row tid & 127 and heads 2k + (tid >> 7), k < KP (no padded
    //      head lanes, one row's scalar work once), the row sums on the row's lane of waves 0-1 ----
    OPAQUE_LANE();
    uint4 xc[2];
    load_x(chunk, xc);  // this chunk's states again, for the X image dW0 reads (phase 5)
    float *const zb = reinterpret_cast<float *>(dzimg);  // [128][16] f32: z -> log-prob; col 8: dlogp
    {
      const int n = lane & 15, qg = lane >> 4;
      f32x4 zacc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      {
        bf16x8 bh[H / 32], za[2][H / 32];
#pragma unroll
        for (int s = 0; s < H / 32; ++s) {
          bh[s] = lds_b128(whb + n * HeadImg<H>::PITCH + 2 * (32 * s + 8 * qg));
#pragma unroll
          for (int u = 0; u < 2; ++u) za[u][s] = lds_b128(img2 + img_off(32 * w + 16 * u + n, 4 * s + qg, PITCH));
        }
#pragma unroll
        for (int s = 0; s < H / 32; ++s)
#pragma unroll
          for (int u = 0; u < 2; ++u) zacc[u] = mfma16_v(za[u][s], bh[s], zacc[u]);
      }
      drain_fence();
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) zb[(32 * w + 16 * u + 4 * qg + i) * 16 + n] = zacc[u][i];
    }
    __syncthreads();
    OPAQUE_LANE();
    {
      const int row = tid & 127, hb = tid >> 7;
      const bool valid = chunk * RR + row < count;
      const float *const sp = reinterpret_cast<const float *>(simg) + row * kFusedSP;
      float dzv[KP];
      if constexpr (ACTOR) {
        float yk[KP], dk[KP], zk[KP];
#pragma unroll
        for (int k = 0; k < KP; ++k) zk[k] = zb[row * 16 + 2 * k + hb];  // all reads before the writes
#pragma unroll
        for (int k = 0; k < KP; ++k) {  // (row, head a): y, x - mu, the Normal log-prob
          const int a = 2 * k + hb;
          const bool on = a < A;
          float zz = zk[k];
          if (N.bh) zz += hbias[a];
          const float y = tanhf(zz);
          const float mu = q.omv * y;
          const float x = valid ? sp[a] : mu;
          const float d = x - mu;
          yk[k] = y;
          dk[k] = on ? d : 0.f;
          zb[row * 16 + a] = on ? ((-(d * d)) * (0.5f * hbias[48 + a]) - hbias[32 + a]) - kLogSqrt2Pi : 0.f;
        }
        __syncthreads();
        if (tid < RR) {  // the row's log-prob (row16_sum's tree; heads >= NH are its zero pads)
          float l[8];
#pragma unroll
          for (int a = 0; a < 8; ++a) l[a] = a < NH ? zb[row * 16 + a] : 0.f;
          const float logp = ((l[0] + l[1]) + (l[2] + l[3])) + ((l[4] + l[5]) + (l[6] + l[7]));
          const float old_lp = valid ? sp[A] : logp;
          const float adv = valid ? sp[A + 1] : 0.f;
          const float ratio = expf(logp - old_lp);
          const float s1 = ratio * adv;
          const float cl = ratio < q.clip_lo ? q.clip_lo : (ratio > q.clip_hi ? q.clip_hi : ratio);
          const float s2 = cl * adv;
          const float mn = (s1 != s1 || s2 != s2) ? (s1 + s2) : (s2 < s1 ? s2 : s1);
          const float gg = -q.inv_b;
          const float g1 = (s1 < s2) ? gg : (s1 == s2 ? gg * 0.5f : 0.f);
          const float g2 = (s2 < s1) ? gg : (s1 == s2 ? gg * 0.5f : 0.f);
          const bool inside = (ratio >= q.clip_lo) && (ratio <= q.clip_hi);
          const float dratio = g1 * adv + (inside ? g2 * adv : 0.f);
          zb[row * 16 + 8] = valid ? dratio * ratio : 0.f;
          if (valid) g_loss += mn;
        }
        __syncthreads();
        const float dlogp = zb[row * 16 + 8];
#pragma unroll
        for (int k = 0; k < KP; ++k) {
          const int a = 2 * k + hb;
          const bool on = a < A;
          const float h_ivar = hbias[48 + a];
          const float dmu = dlogp * (dk[k] * h_ivar);
          dzv[k] = on ? (dmu * q.omv) * (1.f - yk[k] * yk[k]) : 0.f;
          if (on && valid) {
            g_ls[k] += dlogp * ((dk[k] * dk[k]) * h_ivar - 1.f) - q.ent_coef * q.inv_ba;
            g_bh[k] += dzv[k];
          }
        }
      } else {
        float v = zb[row * 16];
        if (N.bh) v += hbias[0];
        const float vt = valid ? sp[A + 2] : v;
        const float diff = v - vt;
        const float ad = fabsf(diff);
        dzv[0] = tid < RR ? q.inv_b * (diff < -1.f ? -1.f : (diff > 1.f ? 1.f : diff)) : 0.f;
        if (tid < RR) {
          if (valid) g_loss += (ad < 1.f) ? 0.5f * ad * ad : (ad - 0.5f);
          g_bh[0] += dzv[0];
        }
      }
      __syncthreads();  // every z / log-prob / dlogp read done: the dz images take the region
      // dz images: row-major [128][16] and head-major [16][128 + 8], zeros in the padded heads
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        const int a = 2 * k + hb;
        if (a < NH) {
          *reinterpret_cast<uint16_t *>(dzimg + row * kDzRowBytes + 2 * a) = bf16_bits4(dzv[k]);
          *reinterpret_cast<uint16_t *>(dztimg + a * DZTP + 2 * row) = bf16_bits4(dzv[k]);
        }
      }
      if (tid < RR) {
#pragma unroll
        for (int a = NH; a < 16; ++a) {
          *reinterpret_cast<uint16_t *>(dzimg + row * kDzRowBytes + 2 * a) = 0;
          *reinterpret_cast<uint16_t *>(dztimg + a * DZTP + 2 * row) = 0;
        }
      }
    }
    STAMP4(5);
    __syncthreads();
    STAMP4(6);

    // ---- phase 5: the X image for dW0; head dW += dz^T a2 (own features); d2 = (dz . W_h) *
    //      ReLU'(a2) -> bias grad, D2 written over A2 in place (own columns: this wave's reads of
    //      them above precede the writes in its LDS order) ----
    OPAQUE_LANE();
    store_x(simg, xc);
    {
      // head dW and d2 operands all issued up front (the head dW MFMAs hide the d2 reads)
      bf16x8 af[RR / 32], bt[RR / 32][4], wht[2], dzb[4];
#pragma unroll
      for (int ks = 0; ks < RR / 32; ++ks) {
        af[ks] = lds_b128(dztimg + (lane & 15) * DZTP + 2 * (32 * ks + 8 * (lane >> 4)));
#pragma unroll
        for (int j = 0; j < 4; ++j) bt[ks][j] = tr_frag16(img2, PITCH, 32 * ks, 64 * w + 16 * j, lane);
      }
#pragma unroll
      for (int ft = 0; ft < 2; ++ft) wht[ft] = head_t_frag<H>(whb, 2 * w + ft, lane);
#pragma unroll
      for (int t = 0; t < 4; ++t) dzb[t] = lds_b128(dzimg + (32 * t + r) * kDzRowBytes + 16 * h);
#pragma unroll
      for (int ks = 0; ks < RR / 32; ++ks)
#pragma unroll
        for (int j = 0; j < 4; ++j) ghw[j] = mfma16_v(af[ks], bt[ks][j], ghw[j]);
      OPAQUE_LANE();
#pragma unroll
      for (int ft0 = 0; ft0 < 2; ft0 += NF) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int f = 0; f < NF; ++f) acc[f][t] = mfma_v(wht[ft0 + f], dzb[t], zero16());
        drain_fence();
        backward_in_place<NF>(img2, acc, gb1, w, ft0, lane);
      }
    }
    STAMP4(7);
    __syncthreads();
    STAMP4(8);

    // ---- phase 6a: dW1 += D2^T A1 over the chunk's 128 rows (8 k-steps of 16 rows, the next
    //      k-step's fragments read under the current one's MFMAs); the next chunk's states
    //      prefetched and parked in the (now free) dz region ----
    OPAQUE_LANE();
    {
      uint4 xn[2];
      load_x(chunk + G, xn);
      // fragments of k-step ks + 1 read under k-step ks's 16 MFMAs
      bf16x8 fa[2][2], fb[2][8];
#pragma unroll
      for (int a = 0; a < 2; ++a) fa[0][a] = tr_frag(img2, PITCH, 0, 64 * w + 32 * a, lane);
#pragma unroll
      for (int b = 0; b < 8; ++b) fb[0][b] = tr_frag(img1, PITCH, 0, 32 * b, lane);
#pragma unroll
      for (int ks = 0; ks < RR / 16; ++ks) {
        const int cu = ks & 1, nx = cu ^ 1;
        if (ks == RR / 16 - 2) ring_prime4<NF, C>(w_frag_base<H>(N.w1bt, 2 * w, lane), ring);  // for 6b
#pragma unroll
        for (int b = 0; b < 8; ++b) {
#pragma unroll
          for (int a = 0; a < 2; ++a) mfma_agpr(gw1[a][b], fa[cu][a], fb[cu][b]);
          if (ks + 1 < RR / 16) {
            if (b < 2) fa[nx][b] = tr_frag(img2, PITCH, 16 * (ks + 1), 64 * w + 32 * b, lane);
            fb[nx][b] = tr_frag(img1, PITCH, 16 * (ks + 1), 32 * b, lane);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      store_x(xnimg, xn);
    }
    STAMP4(9);

    // ---- phase 6b: d1 = (W1^T d2) * ReLU'(a1) -> bias grad, D1 over A1 in place (after every
    //      wave's dW1 reads of A1) ----
#pragma unroll
    for (int ft0 = 0; ft0 < 2; ft0 += NF) {
      OPAQUE_LANE();
#pragma unroll
      for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[f][t] = zero16();
      pass4<NF, C>(w_frag_base<H>(N.w1bt, 2 * w + ft0, lane), img2, r, h, ring, acc);
      if (ft0 + NF < 2) ring_prime4<NF, C>(w_frag_base<H>(N.w1bt, 2 * w + ft0 + NF, lane), ring);
      if (ft0 == 0) __syncthreads();  // every wave's dW1 reads of A1 done before D1 overwrites it
      OPAQUE_LANE();
      backward_in_place<NF>(img1, acc, gb0, w, ft0, lane);
    }

    // ---- phase 7: dW0 += D1^T X (the wave's own D1 columns; X staged in phase 5) ----
    OPAQUE_LANE();
    {
      bf16x8 xb[RR / 16], d1f[RR / 16][2];
#pragma unroll
      for (int ks = 0; ks < RR / 16; ++ks) {
        xb[ks] = tr_frag_x(simg, 16 * ks, lane);
#pragma unroll
        for (int ft = 0; ft < 2; ++ft) d1f[ks][ft] = tr_frag(img1, PITCH, 16 * ks, 64 * w + 32 * ft, lane);
      }
#pragma unroll
      for (int ks = 0; ks < RR / 16; ++ks)
#pragma unroll
        for (int ft = 0; ft < 2; ++ft) gw0[ft] = mfma_v(d1f[ks][ft], xb[ks], gw0[ft]);
    }
    __syncthreads();
    STAMP4(10);
  }

#undef OPAQUE_LANE
  // ================= epilogue: one partial-gradient slab per workgroup =================
  tid = tid0;
  lane = tid & 63;
  r = lane & 31;
  h = lane >> 5;
  float *slab = q.slabs + static_cast<int64_t>(blockIdx.x) * q.slab_stride;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int o0 = 32 * (2 * w + a), i0 = 32 * b;
#pragma unroll
      for (int e = 0; e < 16; ++e)
        slab[N.off_w1 + static_cast<int64_t>(o0 + reg_feature(e, h)) * H + i0 + r] = gw1[a][b][e];
    }
  if (r < q.din) {
#pragma unroll
    for (int ft = 0; ft < 2; ++ft)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        slab[N.off_w0 + static_cast<int64_t>(64 * w + 32 * ft + reg_feature(e, h)) * q.din + r] = gw0[ft][e];
  }
  if ((lane & 1) == 0) {
#pragma unroll
    for (int ft = 0; ft < 2; ++ft) {
      const int f = 64 * w + 32 * ft + rs16_feature(lane);
      if (N.b1) slab[N.off_b1 + f] = gb1[ft];
      if (N.b0) slab[N.off_b0 + f] = gb0[ft];
    }
  }
  const int na = ACTOR ? A : 1;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int a = 4 * (lane >> 4) + i;
      if (a < na) slab[N.off_wh + static_cast<int64_t>(a) * H + 64 * w + 16 * j + (lane & 15)] = ghw[j][i];
    }
  // head bias / log-std / loss partials: each wave's 64 lanes in a fixed xor-butterfly order,
  // then per head the two waves holding it (heads of parity hb on waves 2hb, 2hb + 1) in order
  float *red = reinterpret_cast<float *>(lds + L::RED);  // [4 waves][KP + 1][2]
  auto wsum = [](float v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v += __shfl_xor(v, m, 64);
    return v;
  };
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const float sb = wsum(g_bh[k]), sl = wsum(g_ls[k]);
    if (lane == 0) {
      red[(w * (KP + 1) + k) * 2] = sb;
      red[(w * (KP + 1) + k) * 2 + 1] = sl;
    }
  }
  {
    const float s = wsum(g_loss);
    if (lane == 0) red[(w * (KP + 1) + KP) * 2] = s;
  }
  __syncthreads();
  if (tid < na) {
    const int k = NH > 1 ? tid >> 1 : 0, hb = NH > 1 ? tid & 1 : 0;
    const float sb = red[((2 * hb) * (KP + 1) + k) * 2] + red[((2 * hb + 1) * (KP + 1) + k) * 2];
    const float sl = red[((2 * hb) * (KP + 1) + k) * 2 + 1] + red[((2 * hb + 1) * (KP + 1) + k) * 2 + 1];
    if (N.bh) slab[N.off_bh + tid] = sb;
    if (ACTOR) slab[q.off_logstd + tid] = sl;
  }
  if (tid == 0) {
    float s = 0.f;
#pragma unroll
    for (int v = 0; v < NW4; ++v) s += red[(v * (KP + 1) + KP) * 2];
    q.loss_part[2 * blockIdx.x + z] = s;
  }
  if constexpr (STAMP) {  // after every wave's slab stores have drained
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    STAMP4(11);
    t_acc[12] = __builtin_amdgcn_s_memrealtime() - t_real0;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (tid0 == 0) {
      uint64_t *dst = q.stamps + (static_cast<int64_t>(z) * gridDim.x + blockIdx.x) * kStampSlots;
#pragma unroll
      for (int k = 0; k < kStampSlots; ++k) dst[k] = t_acc[k];
    }
  }
#undef STAMP4
}

template <int CFG>
using CfgOf = typename std::conditional<CFG == 0, Cfg4<7, 1>,
                                        typename std::conditional<CFG == 1, Cfg4<3, 4>, Cfg4<7, 2>>::type>::type;

template <int NA, int CFG, bool STAMP>
__global__ __launch_bounds__(NT4, 1) void fused_update4_kernel(FusedArgs q) {
  __shared__ __attribute__((aligned(16))) char lds[Lds4::TOTAL];
  if (blockIdx.y == 0) body4<NA, true, 1, CfgOf<CFG>, STAMP>(q, q.net[0], lds);
  else body4<1, false, 1, CfgOf<CFG>, STAMP>(q, q.net[1], lds);
}

}  // namespace f4

bool fused_update4_ok(const FusedArgs &q) {
  return q.hidden == f4::H && q.act == PPO_ACT_RELU && q.act_dim >= 1 && q.act_dim <= kFusedMaxAct;
}

template <int CFG>
static void launch4_cfg(const FusedArgs &q, const TimRec &rec, hipStream_t st) {
  const dim3 grid(q.G, 2), block(f4::NT4);
  if (q.stamps) {  // diagnostic build: the headline head width only
    launch_k(rec, f4::fused_update4_kernel<6, CFG, true>, grid, block, 0, st, q);
    return;
  }
  if (q.act_dim <= 2) launch_k(rec, f4::fused_update4_kernel<2, CFG, false>, grid, block, 0, st, q);
  else if (q.act_dim <= 4) launch_k(rec, f4::fused_update4_kernel<4, CFG, false>, grid, block, 0, st, q);
  else if (q.act_dim <= 6) launch_k(rec, f4::fused_update4_kernel<6, CFG, false>, grid, block, 0, st, q);
  else launch_k(rec, f4::fused_update4_kernel<8, CFG, false>, grid, block, 0, st, q);
}

static const int g_f4_cfg = [] {
  const char *v = getenv("PPO_F4_CFG");
  return v ? atoi(v) : 0;
}();

int fused_update4_launch(const FusedArgs &q, const TimRec &rec, hipStream_t st) {
  PPO_REQUIRE(fused_update4_ok(q), "fused update (4 waves): ReLU, H = 256, act_dim <= 8 only");
  PPO_REQUIRE(q.G >= 1 && q.G <= kFusedMaxWG, "fused update: bad workgroup count %d", q.G);
  PPO_REQUIRE(!q.stamps || (q.act_dim > 4 && q.act_dim <= 6),
              "fused update (4 waves): phase stamps only for act_dim 5-6");
  if (g_f4_cfg == 1) launch4_cfg<1>(q, rec, st);
  else if (g_f4_cfg == 2) launch4_cfg<2>(q, rec, st);
  else launch4_cfg<0>(q, rec, st);
  PPO_LAUNCHED();
  return 0;
}

}  // namespace ppo
