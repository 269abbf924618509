// Windowed BiLSTM actor-critic on gfx950, behind the ppo_lstm_* C-ABI.
//
// Reference: models/lstm/lstm_actor.py:9-48 and lstm_critic.py:9-41 -- torch.nn.LSTM(O, Hf,
// num_layers, bidirectional=True, batch_first=True) over the (B, W, O) observation window, the
// activation on its outputs, then NetworkBlock MLPs (network_block_creator.py:24-86):
//   actor : features = act(Y.reshape(B, W*2Hf));  mean = tanh(MLP_mu(features));
//           std = 0.2 * exp(tanh(MLP_ls(features)))  -- shape (B, A): the reference's
//           repeat_interleave(std[None], B, 0) (lstm_actor.py:48) makes it (B, B, A), which
//           torch.distributions.Normal then cannot pair with a (B, A) mean; the engine returns
//           the per-row std the formula means (the std-shape fix SURVEY.md s0 asks for).
//   critic: one-layer BiLSTM, value = MLP_v(act(Y[:, W-1, :]))
// and the PPO losses of ppo.py:93-148 with that per-row std (Normal.log_prob / entropy).
//
// One LSTM layer, both directions in every launch (GemmBatch problem z = direction):
//   Gx = X W_ih^T + b_ih           one GEMM over the B*W rows          (gemm.h FWD, identity)
//   per step s (t = s forward, W-1-s reverse):
//     Gh = h_prev W_hh^T + b_hh    one GEMM over the B rows (skipped at s = 0: h_prev = 0)
//     lstm_cell_fwd_kernel         gates = Gh + Gx (torch: linear_hh(hx).add_(igates)),
//                                  i,f,o = sigmoid, g = tanh, c = f*c_prev + i*g, h = o*tanh(c);
//                                  keeps the gate activations (over Gx), c, h and h_prev
//   backward (BPTT), per step in reverse processing order:
//     dh_rec = dG(next step) W_hh  one GEMM over the B rows
//     lstm_cell_bwd_kernel         torch's elementwise backward forms (sigmoid: g*(1-y)*y,
//                                  tanh: g*(1-y*y)); dG overwrites the gate activations
//   dW_ih = dG^T X, dW_hh = dG^T H_prev (split-K slabs; bias grads = column sums of dG), and for
//   stacked layers dX = sum_d dG_d W_ih_d.
// GEMMs are the engine's MFMA templates (exact-f32 v_mfma_f32_32x32x2_f32 by default, bf16
// operands in PPO_PREC_BF16); the slabs reduce with reduce_slab_block in a fixed order.
// In bf16 mode the producers of the operands only GEMMs read -- the gathered states, h_prev and
// dG -- write them as bf16 (the RNE rounding the GEMM would apply while staging), so the
// weight-gradient, recurrent-gradient and input-gradient GEMMs move half the bytes; the bias
// gradients (column sums of dG) are then sums of those bf16 values.  The gate activations stay
// f32: stored as bf16 (measured, round 6) the sigmoid derivative y (1 - y) of a saturated gate
// loses its digits (bf16's spacing below 1 is 2^-8), which moved the BiLSTM weight gradients by
// 0.02-6.5 % (relative L2; latent 64, W = 3) in the bf16 emulation.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <new>
#include <vector>

#include "common.h"
#include "gemm.h"
#include "gemm_ops.h"
#include "reduce_slabs.h"
#include "timing.h"
#include "wide_gemm.h"
#include "wide_ops.h"

namespace ppo {
namespace lstm {

constexpr int kMaxA = 32;
constexpr int kSplits = 32;           // split-K slabs of the weight gradients (at most)
constexpr int64_t kAlign = 16;        // floats: every flat tensor starts 64-B aligned
constexpr int64_t kWsAlign = 64;

static inline int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

struct LstmLayer {
  int in;
  int64_t w_ih[2], w_hh[2], b_ih[2], b_hh[2];  // flat offsets, direction d
};
struct LstmNet {
  int layers, hidden;
  LstmLayer l[PPO_MAX_LAYERS];
};
struct MlpLayer {
  int in, out, act;
  int64_t w, b;  // b < 0: no bias
};
struct Mlp {
  int n;  // layers incl. the output layer
  MlpLayer l[PPO_MAX_LAYERS + 1];
};

// ---- kernels --------------------------------------------------------------------------------
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

struct CellArgs {
  float *g;            // [B*W][2][4H]: Gx in, gate activations out (dG in the backward)
  const float *gh;     // [B][2][4H] recurrent projection incl. b_hh (nullptr at the first step)
  const float *b_hh[2];
  float *c;            // [B*W][2H] cell states
  float *y;            // [B*W][2H] layer output h (step kernels: nullable, W16 only)
  float *hp;           // [B*W][2H] h_prev (zeros at each direction's first step)
  __bf16 *hp16;        // bf16 mode: h_prev as bf16 instead (the dW_hh GEMM's only operand use)
  float *feat;         // optional act(h): mode 1 -> [B*W][2H] (actor), mode 2 -> [B][2H] at t=W-1
  __bf16 *feat16;      // mode 1, nullable: act(h) as bf16 here instead of feat (bf16 ReLU nets:
                       // the actor MLPs' GEMMs read the features only as RNE bf16)
  int feat_mode, act;
  int b, w, h, s;
};

// One thread per (row, direction, 4 consecutive units): every tensor is read and written as
// float4 (H % 4 == 0, 16-B aligned buffers); per element the arithmetic of torch's LSTM cell.
__global__ __launch_bounds__(256) void lstm_cell_fwd_kernel(CellArgs q) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int H = q.h, W = q.w, H4 = H / 4;
  if (i >= static_cast<int64_t>(q.b) * 2 * H4) return;
  const int j = 4 * static_cast<int>(i % H4);
  const int d = static_cast<int>((i / H4) & 1);
  const int64_t b = i / (2 * H4);
  const bool first = q.s == 0;
  const int t = d == 0 ? q.s : W - 1 - q.s;
  const int tp = d == 0 ? t - 1 : t + 1;
  float *g = q.g + (b * W + t) * (8 * H) + d * (4 * H);
  float4 pre[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float4 hg = first ? *reinterpret_cast<const float4 *>(q.b_hh[d] + k * H + j)
                            : *reinterpret_cast<const float4 *>(q.gh + b * (8 * H) + d * (4 * H) + k * H + j);
    const float4 gx = *reinterpret_cast<const float4 *>(g + k * H + j);
    pre[k] = make_float4(hg.x + gx.x, hg.y + gx.y, hg.z + gx.z, hg.w + gx.w);
  }
  const int64_t o = (b * W + t) * (2 * H) + d * H + j;
  const int64_t op = (b * W + tp) * (2 * H) + d * H + j;
  const float4 cp4 = first ? make_float4(0.f, 0.f, 0.f, 0.f) : *reinterpret_cast<const float4 *>(q.c + op);
  const float4 hp4 = first ? make_float4(0.f, 0.f, 0.f, 0.f) : *reinterpret_cast<const float4 *>(q.y + op);
  const float *pr[4] = {&pre[0].x, &pre[1].x, &pre[2].x, &pre[3].x};
  const float cpv[4] = {cp4.x, cp4.y, cp4.z, cp4.w};
  float ig[4], fg[4], gg[4], og[4], c[4], h[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    ig[e] = sigmoidf_(pr[0][e]);
    fg[e] = sigmoidf_(pr[1][e]);
    gg[e] = tanhf(pr[2][e]);
    og[e] = sigmoidf_(pr[3][e]);
    c[e] = fg[e] * cpv[e] + ig[e] * gg[e];  // (forgetgate * cx).add_(ingate * cellgate)
    h[e] = og[e] * tanhf(c[e]);
  }
  *reinterpret_cast<float4 *>(g + j) = make_float4(ig[0], ig[1], ig[2], ig[3]);
  *reinterpret_cast<float4 *>(g + H + j) = make_float4(fg[0], fg[1], fg[2], fg[3]);
  *reinterpret_cast<float4 *>(g + 2 * H + j) = make_float4(gg[0], gg[1], gg[2], gg[3]);
  *reinterpret_cast<float4 *>(g + 3 * H + j) = make_float4(og[0], og[1], og[2], og[3]);
  *reinterpret_cast<float4 *>(q.c + o) = make_float4(c[0], c[1], c[2], c[3]);
  *reinterpret_cast<float4 *>(q.y + o) = make_float4(h[0], h[1], h[2], h[3]);
  if (q.hp16) {
    *reinterpret_cast<uint2 *>(q.hp16 + o) =
        make_uint2(pack_bf16x2(hp4.x, hp4.y), pack_bf16x2(hp4.z, hp4.w));
    // the next step's h_prev row as well: the W16 step kernel stages its A operand from it
    if (q.s + 1 < W) {
      const int tn = d == 0 ? t + 1 : t - 1;
      *reinterpret_cast<uint2 *>(q.hp16 + (b * W + tn) * (2 * H) + d * H + j) =
          make_uint2(pack_bf16x2(h[0], h[1]), pack_bf16x2(h[2], h[3]));
    }
  } else
    *reinterpret_cast<float4 *>(q.hp + o) = hp4;
  if (q.feat_mode == 1 && q.feat16) {
    *reinterpret_cast<uint2 *>(q.feat16 + o) =
        make_uint2(pack_bf16x2(act_forward(h[0], q.act), act_forward(h[1], q.act)),
                   pack_bf16x2(act_forward(h[2], q.act), act_forward(h[3], q.act)));
  } else if (q.feat_mode == 1 || (q.feat_mode == 2 && t == W - 1)) {
    float *f = q.feat_mode == 1 ? q.feat + o : q.feat + b * (2 * H) + d * H + j;
    *reinterpret_cast<float4 *>(f) = make_float4(act_forward(h[0], q.act), act_forward(h[1], q.act),
                                                 act_forward(h[2], q.act), act_forward(h[3], q.act));
  }
}

// ---- one forward step s > 0 in one launch (bf16 mode) ----------------------------------------
// The recurrent projection gh = h_prev W_hh^T + b_hh on MFMA with lstm_cell_fwd_kernel's cell in
// the epilogue, for both directions (blockIdx.z): the layered form writes gh ([B][2][4H] f32) in a
// GEMM and reads it back in the cell kernel.  A workgroup owns 64 rows x 64 hidden units and all
// four gates of them (a lane's accumulators hold i, f, g, o of the same (row, unit), so the cell
// needs no exchange).  Bitwise the layered result: the operands rounded to bf16 (RNE) as staged,
// the K order of gemm_bf16_kernel (k-steps of 16 in order into one v_mfma_f32_32x32x16_bf16
// accumulator), gh = acc + b_hh, then pre = gh + Gx and the same cell arithmetic.
constexpr int kStepUnits = 64, kStepBK = 32;
constexpr int kStepRowsMb = 128;  // rows per workgroup of the minibatch step launches
// their k-loop pipeline (lstm_step_fwd_body PIPE): 2, the LDS-DMA ring (default; measured
// against 1 on one box, alternating: forward steps 115.2 -> 100.5 ms per iteration, the main.py
// line 399.0 / 398.3 -> 384.2 / 383.4 ms, profiles/r06/lstm_pipe_*), or PPO_LSTM_STEP_PIPE=1, two
// register staging sets; read per call
static int lstm_step_pipe_env() {
  const char *v = getenv("PPO_LSTM_STEP_PIPE");
  return (v && atoi(v) == 1) ? 1 : 2;
}
struct StepArgs {
  CellArgs cell;
  const float *whh[2];  // W_hh per direction, [4H][H] f32 (torch layout)
  const __bf16 *whh16[2];  // W16 instantiation: the same rows as bf16 (the ctx's weight copy)
  // FX instantiation (layer 0): the input projection Gx = x_t W_ih^T + b_ih in the same launch,
  // from the bf16 window rows ([B*W][ldx], row b*W + t) and the W_ih images ([4H][ldx])
  const __bf16 *x16;
  const __bf16 *wih16[2];
  const float *b_ih[2];
  int ldx;
};

typedef __bf16 lstm_bf16x8 __attribute__((ext_vector_type(8)));
typedef float lstm_f32x16 __attribute__((ext_vector_type(16)));

// FX (W16 only): the step also computes its own input projection -- Gx of row t never goes to
// HBM.  Phase X accumulates x_t W_ih^T over the ldx k-columns (k-steps of 16 in order, one
// v_mfma_f32_32x32x16_bf16 accumulator per gate: wide_gemm.h's WK_F32 order over the same bf16
// operands), adds b_ih (its epilogue's f32 add) and keeps the result in registers; phase H is the
// recurrent projection as above (skipped at s = 0, where h_prev = c_prev = 0).  Bitwise the
// projection GEMM + step pair.
//
// ROWS rows x 64 units per workgroup, ROWS / 32 x 2 waves (a wave: 32 rows x 32 units x 4 gates).
// Every workgroup streams the whole 256 x K weight panel of its 64 units, so the panel traffic
// per launch is (b / ROWS) x 2 x 4H x K x 2 B: 128-row workgroups halve it against 64.
//
// PIPE: the k-loop's operand pipeline -- 0: one register staging set (load tile k+1 while tile k
// multiplies); 1: two register sets, loads two tiles ahead; 2 (W16): LDS-DMA ring
// (global_load_lds_dwordx4 straight into swizzled [rows][64] images, wide_gemm.h's RowImage
// layout), 3 stages of 64-deep k-tiles, no register staging.
template <bool W16, bool FX, int ROWS, int PIPE>
__device__ __forceinline__ void lstm_step_fwd_body(const StepArgs &q, int d) {
  static_assert(ROWS == 64 || ROWS == 128, "step rows");
  static_assert(PIPE < 2 || W16, "LDS-DMA from bf16 operands only");
  constexpr bool DMA = PIPE == 2;
  constexpr int NT = 4 * ROWS, RT = ROWS / 32;    // threads, row tiles
  // k-tile depth (64 for the register-prefetching loop measured: its two staging sets then need
  // 123 VGPRs of spill in lstm_step_fwdx_kernel)
  constexpr int BK = DMA ? 64 : kStepBK;
  constexpr int IPR = BK / 4;                     // 4-element staging items per operand row
  constexpr int NA = IPR * ROWS / NT, NB = 256 * IPR / NT;  // A / B staging items per thread
  constexpr int AP = DMA ? BK : BK + 8;           // bf16 image row pitch (16 B of padding unless
                                                  // swizzled)
  constexpr int AIMG = ROWS * AP, BIMG = 4 * kStepUnits * AP;
  constexpr int NSTG = DMA ? 3 : 2;
  __shared__ __attribute__((aligned(16))) __bf16 lds[NSTG * (AIMG + BIMG)];
  const CellArgs &c = q.cell;
  const int H = c.h, W = c.w;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int mt = wv % RT, ug = wv / RT;
  const int r0 = blockIdx.x * ROWS, j0 = blockIdx.y * kStepUnits;
  const int t = d == 0 ? c.s : W - 1 - c.s;
  const int tp = d == 0 ? t - 1 : t + 1;
  // f32 h_prev rows (+ row * W * 2H + k; the f32-staged instantiation only)
  const float *arow = W16 ? nullptr : c.y + static_cast<int64_t>(tp) * 2 * H + d * H;
  // W16: h_prev as bf16 from hp16's row t (the previous step wrote it there: bf16(h(tp)), the
  // rounding the f32 staging applies)
  const __bf16 *arow16 = W16 ? c.hp16 + static_cast<int64_t>(t) * 2 * H + d * H : nullptr;
  const int64_t lda = static_cast<int64_t>(W) * 2 * H;
  const float *wb = q.whh[d];
  const bool first = c.s == 0;

  // staging: A ROWS rows x 32 k (2 float4 per thread), B 256 rows (gate g: rows g*H + j0 .. +63)
  // x 32 k (NB float4 per thread); rows past b load row b-1 (clamped, results discarded).  W16:
  // the phase's bf16 operands (A rows at pa + row * pla, B rows at pb + n * plb)
  float4 va[DMA ? 1 : NA], vb[DMA ? 1 : NB];
  uint2 va16[DMA ? 1 : NA], vb16[DMA ? 1 : NB];
  const __bf16 *wb16 = W16 ? q.whh16[d] : nullptr;
  const __bf16 *pa = arow16, *pb = wb16;
  int64_t pla = lda, plb = H;
  auto gload = [&](int k0) {
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int e = tid + NT * u, rr = e / IPR, kk = (e % IPR) * 4;
      const int row = min(r0 + rr, c.b - 1);
      if constexpr (W16) va16[u] = *reinterpret_cast<const uint2 *>(pa + row * pla + k0 + kk);
      else va[u] = *reinterpret_cast<const float4 *>(arow + row * lda + k0 + kk);
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int e = tid + NT * u, nn = e / IPR, kk = (e % IPR) * 4;
      const int gate = nn / kStepUnits, jj = nn - gate * kStepUnits;
      if constexpr (W16) {
        vb16[u] = *reinterpret_cast<const uint2 *>(pb + static_cast<int64_t>(gate * H + j0 + jj) * plb + k0 + kk);
      } else {
        vb[u] = *reinterpret_cast<const float4 *>(wb + static_cast<int64_t>(gate * H + j0 + jj) * H + k0 + kk);
      }
    }
  };
  auto lstore = [&](int buf) {
    __bf16 *ai = lds + buf * (AIMG + BIMG), *bi = ai + AIMG;
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int e = tid + NT * u, rr = e / IPR, kk = (e % IPR) * 4;
      *reinterpret_cast<uint2 *>(ai + rr * AP + kk) =
          W16 ? va16[u] : make_uint2(pack_bf16x2(va[u].x, va[u].y), pack_bf16x2(va[u].z, va[u].w));
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int e = tid + NT * u, nn = e / IPR, kk = (e % IPR) * 4;
      *reinterpret_cast<uint2 *>(bi + nn * AP + kk) =
          W16 ? vb16[u] : make_uint2(pack_bf16x2(vb[u].x, vb[u].y), pack_bf16x2(vb[u].z, vb[u].w));
    }
  };

  lstm_f32x16 acc[4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[g][e] = 0.f;
  auto mfma_tile = [&](int cur) {
    const __bf16 *ai = lds + cur * (AIMG + BIMG), *bi = ai + AIMG;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const lstm_bf16x8 a = *reinterpret_cast<const lstm_bf16x8 *>(
          ai + (32 * mt + (lane & 31)) * AP + 16 * ks + 8 * (lane >> 5));
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const lstm_bf16x8 bv = *reinterpret_cast<const lstm_bf16x8 *>(
            bi + (g * kStepUnits + 32 * ug + (lane & 31)) * AP + 16 * ks + 8 * (lane >> 5));
        acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bv, acc[g], 0, 0, 0);
      }
    }
  };
  // W16: two register sets, tile i's loads in set i % 2 issued two tiles ahead of its LDS store
  // (one tile's MFMA + barrier more to land than a single set gives: the loop is load-latency
  // bound at two waves per SIMD); the same tiles in the same order
  uint2 sa0[PIPE == 1 ? NA : 1], sb0[PIPE == 1 ? NB : 1], sa1[PIPE == 1 ? NA : 1],
      sb1[PIPE == 1 ? NB : 1];
  auto gl16 = [&](int k0, uint2(&ra)[PIPE == 1 ? NA : 1], uint2(&rb)[PIPE == 1 ? NB : 1]) {
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int e = tid + NT * u, rr = e / IPR, kk = (e % IPR) * 4;
      const int row = min(r0 + rr, c.b - 1);
      ra[u] = *reinterpret_cast<const uint2 *>(pa + row * pla + k0 + kk);
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int e = tid + NT * u, nn = e / IPR, kk = (e % IPR) * 4;
      const int gate = nn / kStepUnits, jj = nn - gate * kStepUnits;
      rb[u] = *reinterpret_cast<const uint2 *>(pb + static_cast<int64_t>(gate * H + j0 + jj) * plb + k0 + kk);
    }
  };
  auto ls16 = [&](int buf, const uint2(&ra)[PIPE == 1 ? NA : 1], const uint2(&rb)[PIPE == 1 ? NB : 1]) {
    __bf16 *ai = lds + buf * (AIMG + BIMG), *bi = ai + AIMG;
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int e = tid + NT * u, rr = e / IPR, kk = (e % IPR) * 4;
      *reinterpret_cast<uint2 *>(ai + rr * AP + kk) = ra[u];
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int e = tid + NT * u, nn = e / IPR, kk = (e % IPR) * 4;
      *reinterpret_cast<uint2 *>(bi + nn * AP + kk) = rb[u];
    }
  };
  // PIPE 2: one stage = the A image (ROWS / 8 wave-instructions of 8 rows x 128 B) and the four
  // gates' 64-row B images (8 each); rows past b read row b-1 (clamped, results discarded)
  constexpr int NWV = NT / 64, NIA = ROWS / 8, NIB = 32, PER = (NIA + NIB) / NWV;
  static_assert((NIA + NIB) % NWV == 0, "uneven LDS-DMA split over the waves");
  auto dma_fill = [&](int buf, int k0) {
    __bf16 *ia = lds + buf * (AIMG + BIMG), *ib = ia + AIMG;
#pragma unroll
    for (int jj = 0; jj < PER; ++jj) {
      const int i = wv + NWV * jj;
      if (i < NIA) {
        const int row = 8 * i + (lane >> 3);
        const int lc = (lane & 7) ^ ((row >> 1) & 7);
        const int grow = min(r0 + row, c.b - 1);
        __builtin_amdgcn_global_load_lds(pa + grow * pla + k0 + 8 * lc,
                                         (wide::lds_void *)(ia + 512 * i), 16, 0, 0);
      } else {
        const int ibb = i - NIA, gate = ibb >> 3, row = 8 * (ibb & 7) + (lane >> 3);
        const int lc = (lane & 7) ^ ((row >> 1) & 7);
        __builtin_amdgcn_global_load_lds(pb + static_cast<int64_t>(gate * H + j0 + row) * plb + k0 + 8 * lc,
                                         (wide::lds_void *)(ib + 512 * ibb), 16, 0, 0);
      }
    }
  };
  auto mfma_dma = [&](int buf) {
    const __bf16 *ia = lds + buf * (AIMG + BIMG), *ib = ia + AIMG;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const lstm_bf16x8 a = wide::RowImage<ROWS, NWV>::frag(ia, 32 * mt, ks, lane);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const lstm_bf16x8 bv = wide::RowImage<64, NWV>::frag(ib + g * 64 * 64, 32 * ug, ks, lane);
        acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bv, acc[g], 0, 0, 0);
      }
    }
  };
  auto kloop = [&](int nk) {
    if constexpr (DMA) {
#pragma unroll
      for (int s2 = 0; s2 < NSTG - 1; ++s2)
        if (s2 < nk) dma_fill(s2, s2 * BK);
      int buf = 0;
      for (int kt = 0; kt < nk; ++kt) {
        // this wave's DMA of tile kt has landed (the younger tile may stay in flight), then every
        // wave's by the barrier; every wave is done reading buffer (kt - 1) % NSTG, refilled below
        wide::vm_wait_le<PER, NSTG - 2>(min(NSTG - 2, nk - 1 - kt));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (kt + NSTG - 1 < nk) dma_fill(buf == 0 ? NSTG - 1 : buf - 1, (kt + NSTG - 1) * BK);
        mfma_dma(buf);
        buf = buf + 1 == NSTG ? 0 : buf + 1;
      }
      __syncthreads();  // every wave's reads are done before the next phase refills the ring
    } else if constexpr (W16 && PIPE == 1) {
      gl16(0, sa0, sb0);
      if (nk > 1) gl16(BK, sa1, sb1);
      ls16(0, sa0, sb0);
      if (nk > 2) gl16(2 * BK, sa0, sb0);
      __syncthreads();
      for (int kt = 0; kt < nk; kt += 2) {
        mfma_tile(0);  // tile kt
        if (kt + 1 < nk) {
          ls16(1, sa1, sb1);
          if (kt + 3 < nk) gl16((kt + 3) * BK, sa1, sb1);
        }
        __syncthreads();
        if (kt + 1 >= nk) break;
        mfma_tile(1);  // tile kt + 1
        if (kt + 2 < nk) {
          ls16(0, sa0, sb0);
          if (kt + 4 < nk) gl16((kt + 4) * BK, sa0, sb0);
        }
        __syncthreads();
      }
    } else {
      gload(0);
      lstore(0);
      __syncthreads();
      int cur = 0;
      for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) gload((kt + 1) * BK);
        mfma_tile(cur);
        if (kt + 1 < nk) lstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
      }
    }
  };

  const int j = j0 + 32 * ug + (lane & 31);
  // FX phase X: Gx of the lane's (row, unit) for all four gates, + b_ih, held in gxr
  lstm_f32x16 gxr[4];
  if constexpr (FX) {
    pa = q.x16 + static_cast<int64_t>(t) * q.ldx;
    pla = static_cast<int64_t>(W) * q.ldx;
    pb = q.wih16[d];
    plb = q.ldx;
    kloop(q.ldx / BK);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float bi = q.b_ih[d][g * H + j];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        gxr[g][e] = acc[g][e] + bi;
        acc[g][e] = 0.f;
      }
    }
    pa = arow16;
    pla = lda;
    pb = wb16;
    plb = H;
  }
  if (!FX || !first) kloop(H / BK);

  // epilogue: C row (r&3) + 8 (r>>2) + 4 (lane>>5) of the wave's 32 rows, unit j = lane & 31.
  // Eight rows at a time, every load first and unconditional (rows past b read row b-1): a load
  // behind the row test made each row wait a memory round trip of its own.
  float bh[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bh[g] = c.b_hh[d][g * H + j];
#pragma unroll
  for (int e0 = 0; e0 < 16; e0 += 8) {
    float gx[8][4], cpv[8], hpv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u;
      const int64_t bb = r0 + 32 * mt + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      const int64_t bc = bb < c.b ? bb : c.b - 1;
      if constexpr (FX) {
#pragma unroll
        for (int k = 0; k < 4; ++k) gx[u][k] = gxr[k][e];
      } else {
        const float *g = c.g + (bc * W + t) * (8 * H) + d * (4 * H);
#pragma unroll
        for (int k = 0; k < 4; ++k) gx[u][k] = g[k * H + j];
      }
      const int64_t op = (bc * W + (first ? t : tp)) * (2 * H) + d * H + j;
      cpv[u] = first ? 0.f : c.c[op];
      if constexpr (!W16) hpv[u] = c.y[op];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u;
      const int64_t bb = r0 + 32 * mt + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      if (bb >= c.b) continue;
      float *g = c.g + (bb * W + t) * (8 * H) + d * (4 * H);
      float pre[4];
      if (FX && first) {  // lstm_cell_fwd_kernel's first step: b_hh + Gx
#pragma unroll
        for (int k = 0; k < 4; ++k) pre[k] = bh[k] + gx[u][k];
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) pre[k] = (acc[k][e] + bh[k]) + gx[u][k];  // gh.add_(igates)
      }
      const int64_t o = (bb * W + t) * (2 * H) + d * H + j;
      const float ig = sigmoidf_(pre[0]), fg = sigmoidf_(pre[1]), gg = tanhf(pre[2]),
                  og = sigmoidf_(pre[3]);
      const float cn = fg * cpv[u] + ig * gg;  // (forgetgate * cx).add_(ingate * cellgate)
      const float h = og * tanhf(cn);
      g[j] = ig;
      g[H + j] = fg;
      g[2 * H + j] = gg;
      g[3 * H + j] = og;
      c.c[o] = cn;
      if (c.y) c.y[o] = h;  // null: a one-layer net's minibatch step, where nothing reads h in f32
      if constexpr (W16) {
        // row t's h_prev is already there (FX, first step: zeros); h goes to the next step's row
        if (FX && first) c.hp16[o] = static_cast<__bf16>(0.f);
        if (c.s + 1 < W) {
          const int tn = d == 0 ? t + 1 : t - 1;
          c.hp16[(bb * W + tn) * (2 * H) + d * H + j] = static_cast<__bf16>(h);
        }
      } else if (c.hp16) {
        c.hp16[o] = static_cast<__bf16>(hpv[u]);
      } else {
        c.hp[o] = hpv[u];
      }
      if (c.feat_mode == 1) {
        if (c.feat16) c.feat16[o] = static_cast<__bf16>(act_forward(h, c.act));
        else c.feat[o] = act_forward(h, c.act);
      }
      else if (c.feat_mode == 2 && t == W - 1) c.feat[bb * (2 * H) + d * H + j] = act_forward(h, c.act);
    }
  }
}

template <bool W16, int PIPE>
__global__ __launch_bounds__(4 * kStepRowsMb) void lstm_step_fwd_kernel(StepArgs q) {
  lstm_step_fwd_body<W16, false, kStepRowsMb, PIPE>(q, blockIdx.z);
}
// the rollout's launches (1,024-row windows, 64-row workgroups: 8 x more of them than rows / 128
// would give): the same body under its own name, so the traffic / roofline rows of the minibatch
// kernel stay per-launch comparable
__global__ __launch_bounds__(256) void lstm_step_fwd_rollout_kernel(StepArgs q) {
  lstm_step_fwd_body<true, false, 64, 0>(q, blockIdx.z);
}
// the rollout's steps of BOTH nets in one launch (blockIdx.z = 2 net + direction): one step's
// 1,024 rows give a net 128 workgroups, half the CUs
struct StepArgs2 {
  StepArgs n[2];
};
__global__ __launch_bounds__(256) void lstm_step_fwd_rollout2_kernel(StepArgs2 q) {
  lstm_step_fwd_body<true, false, 64, 0>(q.n[blockIdx.z >> 1], blockIdx.z & 1);
}
// layer 0 with the input projection in the step (FX), minibatch launches
template <int PIPE>
__global__ __launch_bounds__(4 * kStepRowsMb) void lstm_step_fwdx_kernel(StepArgs q) {
  lstm_step_fwd_body<true, true, kStepRowsMb, PIPE>(q, blockIdx.z);
}

struct CellBwdArgs {
  float *g;            // gate activations in, dG out
  const float *c;
  const float *dy;     // [B*W][2H] gradient of the layer output (nullable rows handled by dy_mode)
  const float *dy2;    // mode 1, nullable: a second [B*W][2H] term, dy + dy2 (the actor's two MLPs)
  const float *dy_last;  // mode 2: [B][2H] gradient of h at t = W-1 only
  int dy_mode;         // 1: dy full, 2: dy_last
  const float *dh_rec; // [B][2H] recurrent gradient (nullptr at s = 0)
  float *dcarry;       // [B][2H] dc flowing to the previous forward step
  __bf16 *dg16;        // bf16 mode: dG written here as bf16 ([B*W][8H], g's layout) instead of g
  int b, w, h, s;
};

// float4 in and out as clang vectors (element access by constant index keeps them in registers;
// local float[4] arrays of the first float4 form were kept in scratch)
typedef float lstm_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ lstm_f4 ld4(const float *p) { return *reinterpret_cast<const lstm_f4 *>(p); }
__device__ __forceinline__ void st4(float *p, lstm_f4 v) { *reinterpret_cast<lstm_f4 *>(p) = v; }

__global__ __launch_bounds__(256) void lstm_cell_bwd_kernel(CellBwdArgs q) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int H = q.h, W = q.w, H4 = H / 4;
  if (i >= static_cast<int64_t>(q.b) * 2 * H4) return;
  const int j = 4 * static_cast<int>(i % H4);
  const int d = static_cast<int>((i / H4) & 1);
  const int64_t b = i / (2 * H4);
  const int t = d == 0 ? W - 1 - q.s : q.s;          // reverse of the forward processing order
  const bool first_fwd = d == 0 ? t == 0 : t == W - 1;
  const int tp = d == 0 ? t - 1 : t + 1;
  const int64_t o = (b * W + t) * (2 * H) + d * H + j;
  const int64_t r = b * (2 * H) + d * H + j;
  const lstm_f4 z4 = {0.f, 0.f, 0.f, 0.f};
  lstm_f4 dh4 = z4;
  if (q.dy_mode == 1) {
    dh4 = ld4(q.dy + o);
    if (q.dy2) dh4 = dh4 + ld4(q.dy2 + o);  // add_inplace's dy + dy2, at its one read
  } else if (t == W - 1) {
    dh4 = ld4(q.dy_last + r);
  }
  const lstm_f4 dr4 = q.s > 0 ? ld4(q.dh_rec + r) : z4;
  const lstm_f4 dc4 = q.s > 0 ? ld4(q.dcarry + r) : z4;
  float *g = q.g + (b * W + t) * (8 * H) + d * (4 * H);
  const lstm_f4 ig = ld4(g + j), fg = ld4(g + H + j), gg = ld4(g + 2 * H + j), og = ld4(g + 3 * H + j);
  const lstm_f4 c4 = ld4(q.c + o);
  const lstm_f4 cp4 = first_fwd ? z4 : ld4(q.c + (b * W + tp) * (2 * H) + d * H + j);
  lstm_f4 carry, di, df, dg, dout;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float dh = dh4[e];
    if (q.s > 0) dh += dr4[e];
    const float dc_in = q.s > 0 ? dc4[e] : 0.f;
    const float tc = tanhf(c4[e]);
    const float d_o = dh * tc;                          // hy = outgate * cy.tanh()
    const float d_tc = dh * og[e];
    const float dc = d_tc * (1.f - tc * tc) + dc_in;    // tanh_backward, + the next step's dcx
    const float d_f = dc * cp4[e], d_i = dc * gg[e], d_g = dc * ig[e];
    carry[e] = dc * fg[e];
    di[e] = (d_i * (1.f - ig[e])) * ig[e];              // sigmoid_backward: g * (1 - y) * y
    df[e] = (d_f * (1.f - fg[e])) * fg[e];
    dg[e] = d_g * (1.f - gg[e] * gg[e]);                // tanh_backward
    dout[e] = (d_o * (1.f - og[e])) * og[e];
  }
  st4(q.dcarry + r, carry);
  if (q.dg16) {
    __bf16 *g16 = q.dg16 + (b * W + t) * (8 * H) + d * (4 * H);
    const lstm_f4 gv[4] = {di, df, dg, dout};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      *reinterpret_cast<uint2 *>(g16 + k * H + j) =
          make_uint2(pack_bf16x2(gv[k][0], gv[k][1]), pack_bf16x2(gv[k][2], gv[k][3]));
    return;
  }
  st4(g + j, di);
  st4(g + H + j, df);
  st4(g + 2 * H + j, dg);
  st4(g + 3 * H + j, dout);
}

// The slab fold when every tensor is float4-aligned (the usual case): one thread per float4
// group, its S split loads issued up to 16 at a time, summed in reduce_slab_block's order -- chunk
// c holds splits [S c / 16, S (c + 1) / 16): two as (0 + v_a) + (0 + v_b), one as (0 + v) + 0,
// none as 0 + 0, the chunks added in order -- bitwise that kernel's result, with up to 16 loads in
// flight per thread instead of 2.
template <int S>
__global__ __launch_bounds__(256) void lstm_reduce_fast_kernel(float *__restrict__ grad,
                                                               const float *__restrict__ slabs,
                                                               int64_t total) {
  static_assert(S == 8 || S == 16 || S == 32, "split count");
  constexpr int PER = S / kRedChunks > 0 ? S / kRedChunks : 1;  // splits in a non-empty chunk
  constexpr int HALVES = S > 16 ? 2 : 1, CH = kRedChunks / HALVES;  // chunks per load batch
  const int64_t i = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 4;
  if (i >= total) return;
  const float *src = slabs + i;
  float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int half = 0; half < HALVES; ++half) {
    constexpr int NV = S / HALVES;
    float4 v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j)
      v[j] = *reinterpret_cast<const float4 *>(src + (NV * half + j) * total);
#pragma unroll
    for (int cc = 0; cc < CH; ++cc) {
      const int c = CH * half + cc;
      const int k0 = (S * c) / kRedChunks - NV * half, k1 = (S * (c + 1)) / kRedChunks - NV * half;
      float4 p;
      if (PER == 2) {
        const float4 a = v[k0], b = v[k0 + 1];
        p = make_float4((0.f + a.x) + (0.f + b.x), (0.f + a.y) + (0.f + b.y),
                        (0.f + a.z) + (0.f + b.z), (0.f + a.w) + (0.f + b.w));
      } else if (k1 > k0) {
        const float4 a = v[k0];
        p = make_float4((0.f + a.x) + 0.f, (0.f + a.y) + 0.f, (0.f + a.z) + 0.f, (0.f + a.w) + 0.f);
      } else {
        p = make_float4(0.f + 0.f, 0.f + 0.f, 0.f + 0.f, 0.f + 0.f);
      }
      out = (c == 0) ? p : make_float4(out.x + p.x, out.y + p.y, out.z + p.z, out.w + p.w);
    }
  }
  *reinterpret_cast<float4 *>(grad + i) = out;
}

// bf16 copy of the parameters, 4 per thread (the RNE rounding the GEMMs' staging applies)
__global__ __launch_bounds__(256) void lstm_params_bf16_kernel(const float *__restrict__ p,
                                                               __bf16 *__restrict__ o, int64_t n) {
  const int64_t i = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 4;
  if (i + 3 < n) {
    const float4 v = *reinterpret_cast<const float4 *>(p + i);
    *reinterpret_cast<uint2 *>(o + i) = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
  } else {
    for (int64_t k = i; k < n; ++k) o[k] = static_cast<__bf16>(p[k]);
  }
}

__global__ __launch_bounds__(kRedThreads) void lstm_reduce_kernel(ReduceArgs q) {
  (void)reduce_slab_block(q, blockIdx.x);
}

// xg16 (bf16 mode): the rows as bf16 instead of f32 (GEMM operands only), one (row, step) of O
// values per ld16-wide row; rows == nullptr: the states in order (the rollout's windows)
__global__ void lstm_gather_rows_kernel(const float *__restrict__ states,
                                        const int32_t *__restrict__ rows, int b, int din,
                                        float *__restrict__ xg, __bf16 *__restrict__ xg16, int o,
                                        int ld16) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= static_cast<int64_t>(b) * din) return;
  const int64_t j = i / din;
  const int64_t within = i - j * din;
  const float v = states[(rows ? static_cast<int64_t>(rows[j]) : j) * din + within];
  if (xg16) {
    const int64_t rw = j * (din / o) + within / o;  // row (j, t) of the [b*W][O] view
    xg16[rw * ld16 + within % o] = static_cast<__bf16>(v);
  } else {
    xg[i] = v;
  }
}

// The same gather four values a thread (O % 4 == 0: a float4 never straddles a step's O values,
// and the bf16 rows stay 8-B aligned)
__global__ void lstm_gather_rows4_kernel(const float *__restrict__ states,
                                         const int32_t *__restrict__ rows, int b, int din,
                                         float *__restrict__ xg, __bf16 *__restrict__ xg16, int o,
                                         int ld16) {
  const int64_t i = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 4;
  if (i >= static_cast<int64_t>(b) * din) return;
  const int64_t j = i / din;
  const int64_t within = i - j * din;
  const float4 v = *reinterpret_cast<const float4 *>(
      states + (rows ? static_cast<int64_t>(rows[j]) : j) * din + within);
  if (xg16) {
    const int64_t rw = j * (din / o) + within / o;
    *reinterpret_cast<uint2 *>(xg16 + rw * ld16 + within % o) =
        make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
  } else {
    *reinterpret_cast<float4 *>(xg + i) = v;
  }
}

// The layer-0 W_ih images of both nets and directions as bf16 [4H][ld16] (pad columns stay zero)
struct WihImages {
  const float *src[4];
  __bf16 *dst[4];
  int rows, in, ld16;
};
__global__ __launch_bounds__(256) void lstm_wih_image_kernel(WihImages q) {
  const int64_t per = static_cast<int64_t>(q.rows) * q.in;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= 4 * per) return;
  const int img = static_cast<int>(i / per);
  const int64_t e = i - img * per, r = e / q.in, c = e - r * q.in;
  q.dst[img][r * q.ld16 + c] = static_cast<__bf16>(q.src[img][e]);
}

// W_hh^T images [H][4H] bf16 of every net / layer / direction (the recurrent-gradient GEMM's
// k-inner B operand on the wide path); one thread per destination element
struct WhhTImages {
  const float *src[2 * 2 * PPO_MAX_LAYERS];
  __bf16 *dst[2 * 2 * PPO_MAX_LAYERS];
  int n, h;
};
__global__ __launch_bounds__(256) void lstm_whh_t_image_kernel(WhhTImages q) {
  const int64_t per = 4LL * q.h * q.h;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= q.n * per) return;
  const int img = static_cast<int>(i / per);
  const int64_t e = i - img * per, j = e / (4 * q.h), k = e - j * (4 * q.h);
  q.dst[img][e] = static_cast<__bf16>(q.src[img][k * q.h + j]);
}

__global__ void add_inplace_kernel(float *__restrict__ a, const float *__restrict__ b, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) a[i] += b[i];
}

// act_backward against the layer output, in place on dy (the feature activation of the LSTM
// outputs, lstm_actor.py:45 / lstm_critic.py:37)
__global__ void act_backward_inplace_kernel(float *__restrict__ dy, const float *__restrict__ y,
                                            int64_t n, int act) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) dy[i] = act_backward(dy[i], y[i], act);
}

// ---- heads ----------------------------------------------------------------------------------
struct HeadArgs {
  const float *mean;   // [B][A] tanh(MLP_mu)
  const float *u;      // [B][A] tanh(MLP_ls)
  const float *value;  // [B] critic output
  float *std_out;      // [B][A] (forward / policy step)
  // policy step
  const float *eps;
  uint64_t seed, offset;
  float *action, *logp_out, *value_out;
  // update
  const float *actions, *old_logp, *adv, *vt;
  const int32_t *rows;
  float *dzm, *dzs, *dv;  // [B][A], [B][A], [B]
  float *row_part;        // [B][3]: min(s1, s2), sum_a entropy, huber
  float clip_lo, clip_hi, ent_coef, inv_b, inv_ba;
  int b, a;
};

// Normal(mean, std) with std = 0.2 * exp(u) (lstm_actor.py:47): sample (torch.normal: eps*std +
// mean), log_prob summed over actions (ppo.py:26), critic value passthrough.
__global__ __launch_bounds__(256) void lstm_policy_head_kernel(HeadArgs q) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= q.b) return;
  const int A = q.a;
  float lp = 0.f;
  for (int k = 0; k < A; ++k) {
    const int64_t idx = static_cast<int64_t>(n) * A + k;
    const float mu = q.mean[idx];
    const float sd = 0.2f * expf(q.u[idx]);
    if (q.std_out) q.std_out[idx] = sd;
    if (!q.action) continue;
    const float e = q.eps ? q.eps[idx] : philox_normal_at(q.seed, q.offset + idx);
    const float x = e * sd + mu;
    q.action[idx] = x;
    const float d = x - mu;
    lp += (((-(d * d)) / (2.f * (sd * sd))) - logf(sd)) - kLogSqrt2Pi;
  }
  if (q.logp_out) q.logp_out[n] = lp;
  if (q.value_out) q.value_out[n] = q.value[n];
}

// ppo.py:108-135 per minibatch row: new log-prob, ratio, clipped surrogate, entropy, Huber; the
// gradients w.r.t. the two actor MLPs' pre-tanh outputs and the critic output.
__global__ __launch_bounds__(256) void lstm_update_head_kernel(HeadArgs q) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= q.b) return;
  const int A = q.a;
  const int64_t src = q.rows[n];
  float lp = 0.f, ent = 0.f;
  float mu[kMaxA], sd[kMaxA], dd[kMaxA], uv[kMaxA];
  for (int k = 0; k < A; ++k) {
    const int64_t idx = static_cast<int64_t>(n) * A + k;
    mu[k] = q.mean[idx];
    uv[k] = q.u[idx];  // kept: a reload behind the dz stores below waited for each of them
    sd[k] = 0.2f * expf(uv[k]);
    dd[k] = q.actions[src * A + k] - mu[k];
    const float ls = logf(sd[k]);
    lp += (((-(dd[k] * dd[k])) / (2.f * (sd[k] * sd[k]))) - ls) - kLogSqrt2Pi;
    ent += kEntropyConst + ls;
  }
  const float adv = q.adv[src];
  const float ratio = expf(lp - q.old_logp[src]);
  const float s1 = ratio * adv;
  const float cl = ratio < q.clip_lo ? q.clip_lo : (ratio > q.clip_hi ? q.clip_hi : ratio);
  const float s2 = cl * adv;
  const float mn = (s1 != s1 || s2 != s2) ? (s1 + s2) : (s2 < s1 ? s2 : s1);
  const float gg = -q.inv_b;
  const float g1 = (s1 < s2) ? gg : (s1 == s2 ? gg * 0.5f : 0.f);
  const float g2 = (s2 < s1) ? gg : (s1 == s2 ? gg * 0.5f : 0.f);
  const bool inside = (ratio >= q.clip_lo) && (ratio <= q.clip_hi);
  const float dratio = g1 * adv + (inside ? g2 * adv : 0.f);
  const float dlogp = dratio * ratio;
  for (int k = 0; k < A; ++k) {
    const int64_t idx = static_cast<int64_t>(n) * A + k;
    const float var = sd[k] * sd[k];
    const float dmu = dlogp * (dd[k] / var);
    // d/dstd of -(d^2)/(2 var) - log(std): d^2/std^3 - 1/std; entropy mean: -ent_coef/(B*A*std)
    const float dstd = dlogp * ((dd[k] * dd[k]) / (var * sd[k]) - 1.f / sd[k]) -
                       q.ent_coef * q.inv_ba / sd[k];
    const float du = dstd * sd[k];  // std = 0.2 * exp(u)
    const float uu = uv[k];
    q.dzm[idx] = dmu * (1.f - mu[k] * mu[k]);
    q.dzs[idx] = du * (1.f - uu * uu);
  }
  const float v = q.value[n];
  const float diff = v - q.vt[src];
  const float ad = fabsf(diff);
  q.dv[n] = q.inv_b * (diff < -1.f ? -1.f : (diff > 1.f ? 1.f : diff));
  q.row_part[3 * n] = mn;
  q.row_part[3 * n + 1] = ent;
  q.row_part[3 * n + 2] = (ad < 1.f) ? 0.5f * ad * ad : (ad - 0.5f);
}

// loss scalars: one block, fixed-order strided sums + tree (deterministic)
__global__ __launch_bounds__(256) void lstm_loss_kernel(const float *__restrict__ row_part, int b,
                                                        float inv_b, float inv_ba, float ent_coef,
                                                        float *__restrict__ loss_out) {
  __shared__ float red[3][256];
  const int tid = threadIdx.x;
  float s[3] = {0.f, 0.f, 0.f};
  for (int n = tid; n < b; n += 256)
    for (int k = 0; k < 3; ++k) s[k] += row_part[3 * n + k];
  for (int k = 0; k < 3; ++k) red[k][tid] = s[k];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w)
      for (int k = 0; k < 3; ++k) red[k][tid] += red[k][tid + w];
    __syncthreads();
  }
  if (tid == 0) {
    loss_out[0] = -(red[0][0] * inv_b) - (red[1][0] * inv_ba) * ent_coef;
    loss_out[1] = red[2][0] * inv_b;
  }
}

}  // namespace lstm
}  // namespace ppo

using namespace ppo;
using namespace ppo::lstm;

struct ppo_lstm_ctx {
  ppo_lstm_cfg cfg;
  int device;
  int prec;
  float ent_log_share;  // ppo_*_loss_entropy_share (logged actor loss only)
  LstmNet net[2];  // 0 actor, 1 critic
  Mlp mu, ls, vc;  // actor mean / logstd MLPs, critic MLP
  int64_t total, n_actor;
  std::vector<int64_t> offsets;  // torch parameters() order, actor then critic
  float *params;
  float *ws;
  int64_t rows;  // workspace rows
  // workspace views
  float *x;                          // [rows][W*O] gathered states
  float *g[2][PPO_MAX_LAYERS];       // [rows*W][8H]
  float *c[2][PPO_MAX_LAYERS], *y[2][PPO_MAX_LAYERS], *hp[2][PPO_MAX_LAYERS];  // [rows*W][2H]
  // bf16 mode: the GEMM-only operands as bf16 (gathered states, dG, h_prev)
  __bf16 *x16;                       // [rows*W + 128][ldx16] (pad columns zero)
  int ldx16;                         // round_up(O, 64): the wide GEMM's k extent
  __bf16 *wih16[2][2];               // layer-0 W_ih per net / direction, [4H][ldx16] bf16
  __bf16 *dg16[2][PPO_MAX_LAYERS];   // [(rows + 128)*W][8H] (128 rows: the wide GEMM's A tiles)
  __bf16 *whht16[2][PPO_MAX_LAYERS][2];  // W_hh^T per net / layer / direction, [H][4H] bf16
  __bf16 *hp16[2][PPO_MAX_LAYERS];   // [rows*W][2H]
  __bf16 *p16;                       // [total] bf16 copy of the parameters (minibatch steps)
  const __bf16 *w16;                 // p16 while a bf16 minibatch step runs (its GEMMs' weight
                                     // operands), else null
  float *gh, *dhrec, *dcarry;        // [rows][8H], [rows][2H], [rows][2H]
  float *dy[2], *tmp;                // [rows*W][2H]
  float *feat_a, *feat_c;            // [rows][W*2H], [rows][2H]
  __bf16 *feat16;                    // [rows][W*2H]: the actor features as bf16 (feat16_on())
  float *act_mu[PPO_MAX_LAYERS + 1], *act_ls[PPO_MAX_LAYERS + 1], *act_v[PPO_MAX_LAYERS + 1];
  float *dz[3][2];                   // ping-pong gradient buffers [rows][maxw]: mu, ls, critic
  float *slabs;                      // [kSplits][total] (the first `splits` used)
  int splits;                        // weight-gradient split-K slabs (PPO_LSTM_SPLITS)
  float *row_part;                   // [rows][3]
  int maxw;
  int fused_step;  // bf16 forward steps as lstm_step_fwd_kernel (ppo_lstm_fused_step)
  int rollout;     // inside forward_rollout: the step launches take the rollout kernel
  // forward_all's paired rollout steps: lstm_forward queues each net's step arguments (s > 0)
  // here instead of launching them, forward_all then launches both nets' step s together
  int defer_steps;
  int npend[2];
  StepArgs pend[2][16];
  Timing tim;
};

namespace {

// bf16 forward steps s > 0 as one recurrent-GEMM + cell launch (lstm_step_fwd_kernel);
// PPO_LSTM_FUSED_STEP=0 keeps the layered GEMM + cell pair
const int g_lstm_fused_step = [] {
  const char *v = getenv("PPO_LSTM_FUSED_STEP");
  return v ? atoi(v) : 1;
}();

// weight-gradient split-K slabs: PPO_LSTM_SPLITS = 8 | 16 | 32 (default 32).  Each split writes
// an f32 copy of every weight gradient that the fold reads back; fewer splits starve the
// weight-gradient GEMMs of workgroups instead (round 5, main.py line: 500 / 503 / 545 ms at 32 /
// 16 / 8).  Measured and dropped the same round: the backward step as one launch (recurrent
// gradient GEMM + cell, the forward step's decomposition) -- 136 us per step against 44 + 67 for
// the pair, its MFMA-layout epilogue touching the gates and states 4 B per lane.
const int g_lstm_splits = [] {
  const char *v = getenv("PPO_LSTM_SPLITS");
  const int n = v ? atoi(v) : 32;
  return (n == 8 || n == 16) ? n : 32;
}();

// PPO_LSTM_FUSEX=0: layer 0's input projection as its own GEMM (read per call: the bitwise test
// flips it)
bool lstm_fusex_env() {
  const char *v = getenv("PPO_LSTM_FUSEX");
  return !(v && atoi(v) == 0);
}

// bf16 mode, ReLU: the actor's features (act(h), [B][W*2H]) are stored only as bf16 -- the two
// actor MLPs' first-layer forward and weight-gradient GEMMs read them as RNE bf16 anyway, and the
// input gradient's ReLU' needs only their sign, which RNE keeps -- so the step kernels write, and
// those GEMMs read, half the bytes; bitwise the f32-stored form.  PPO_LSTM_FEAT16=0 keeps f32
// (read per call: the bitwise test flips it).
bool feat16_on(const ppo_lstm_ctx *x) {
  const char *v = getenv("PPO_LSTM_FEAT16");
  return x->prec == PPO_PREC_BF16 && x->cfg.activation == PPO_ACT_RELU &&
         (x->cfg.window * 2 * x->cfg.latent) % 4 == 0 && !(v && atoi(v) == 0);
}

struct TimingScope {
  explicit TimingScope(ppo_lstm_ctx *x) { g_tim = x->tim.on ? &x->tim : nullptr; }
  ~TimingScope() { g_tim = nullptr; }
};

void add_mlp(Mlp &m, int in, const ppo_lstm_cfg &c, int out, int final_act, int64_t &off,
             std::vector<int64_t> &offs) {
  m.n = c.n_hidden + 1;
  for (int l = 0; l < m.n; ++l) {
    MlpLayer &L = m.l[l];
    L.in = in;
    L.out = l < c.n_hidden ? c.hidden[l] : out;
    L.act = l < c.n_hidden ? c.activation : final_act;
    L.w = off;
    offs.push_back(off);
    off = align_up(off + static_cast<int64_t>(L.in) * L.out, kAlign);
    if (c.use_bias) {
      L.b = off;
      offs.push_back(off);
      off = align_up(off + L.out, kAlign);
    } else {
      L.b = -1;
    }
    in = L.out;
  }
}

void add_lstm(LstmNet &n, int layers, int in, int h, int64_t &off, std::vector<int64_t> &offs) {
  n.layers = layers;
  n.hidden = h;
  for (int l = 0; l < layers; ++l) {
    LstmLayer &L = n.l[l];
    L.in = l == 0 ? in : 2 * h;
    for (int d = 0; d < 2; ++d) {  // nn.LSTM order: w_ih, w_hh, b_ih, b_hh, then _reverse
      L.w_ih[d] = off;
      offs.push_back(off);
      off = align_up(off + 4LL * h * L.in, kAlign);
      L.w_hh[d] = off;
      offs.push_back(off);
      off = align_up(off + 4LL * h * h, kAlign);
      L.b_ih[d] = off;
      offs.push_back(off);
      off = align_up(off + 4LL * h, kAlign);
      L.b_hh[d] = off;
      offs.push_back(off);
      off = align_up(off + 4LL * h, kAlign);
    }
  }
}

int gemm_fwd(ppo_lstm_ctx *x, const GemmProblem *p, int np, int k, int rows, int max_n, int act,
             bool b_kn, hipStream_t st) {
  GemmBatch gb{};
  for (int i = 0; i < np; ++i) gb.p[i] = p[i];
  gb.k = k;
  gb.act = act;
  gb.prec = x->prec;
  return b_kn ? gemm_rows_fwd_kn(gb, np, rows, max_n, st)
              : gemm_rows_fwd_nk(gb, np, rows, max_n, st);
}

int gemm_dx(ppo_lstm_ctx *x, const GemmProblem *p, int np, int k, int rows, int max_n, int act,
            hipStream_t st) {
  GemmBatch gb{};
  for (int i = 0; i < np; ++i) gb.p[i] = p[i];
  gb.k = k;
  gb.act = act;
  gb.prec = x->prec;
  return gemm_rows_dx(gb, np, rows, max_n, st);
}

int gemm_partial(ppo_lstm_ctx *x, const GemmProblem *p, int np, int rows, int max_m, int max_n,
                 hipStream_t st) {
  GemmBatch gb{};
  for (int i = 0; i < np; ++i) gb.p[i] = p[i];
  gb.k = rows;
  gb.splits = x->splits;
  gb.slab_stride = x->total;
  gb.prec = x->prec;
  return gemm_wgrad_partial(gb, np, max_m, max_n, st);
}

// LSTM net z forward over xin [b*W][O] (batch-major rows); fills g/c/y/hp of every layer and the
// features of the top layer (actor: all steps, critic: t = W-1).
static const float *ih_bias(const ppo_lstm_ctx *x, const LstmLayer &L, int d) {
  return x->params + L.b_ih[d];
}

// xin16 (bf16 mode, nullable): the same rows as bf16, [b*W][ldx16] -- the input projection
// reads those.
int lstm_forward(ppo_lstm_ctx *x, int z, const float *xin, const __bf16 *xin16, int b,
                 hipStream_t st) {
  const LstmNet &N = x->net[z];
  const int H = N.hidden, W = x->cfg.window;
  const float *P = x->params;
  const bool b16 = x->prec == PPO_PREC_BF16;
  for (int l = 0; l < N.layers; ++l) {
    const LstmLayer &L = N.l[l];
    const float *in = l == 0 ? xin : x->y[z][l - 1];
    GemmProblem p[2] = {};
    for (int d = 0; d < 2; ++d) {
      p[d].a = in;
      p[d].lda = L.in;
      if (l == 0 && xin16) {
        // bf16 mode: the minibatch gather writes only the bf16 rows (xin holds no data then), so
        // the layered fallback below reads those too -- the same RNE-rounded operand the f32-staged
        // form would make, through the bf16-source FWD variant
        p[d].a16 = xin16;
        p[d].lda = x->ldx16;
      }
      p[d].b = P + L.w_ih[d];
      p[d].ldb = L.in;
      p[d].c = x->g[z][l] + d * 4 * H;
      p[d].ldc = 8 * H;
      p[d].bias = P + L.b_ih[d];
      p[d].m = b * W;
      p[d].n = 4 * H;
    }
    const bool fused_step = x->prec == PPO_PREC_BF16 && x->fused_step && H % kStepUnits == 0;
    // layer 0 of a bf16 step with the padded bf16 rows: the input projection inside each step's
    // launch (lstm_step_fwdx_kernel) instead of one Gx GEMM whose f32 output ([B*W][8H]) every
    // step reads back; PPO_LSTM_FUSEX=0 keeps the GEMM
    // step launch (the rollout's 1,024-row windows keep the GEMM: 5x the rows per launch fill the
    // GPU where one step's 1,024 rows do not)
    const bool fusex = fused_step && l == 0 && xin16 && x->w16 && !x->rollout &&
                       (4 * H) % 128 == 0 && x->ldx16 % 64 == 0 && lstm_fusex_env();
    if (fusex) {
      // no separate projection: lstm_step_fwdx_kernel below
    } else if (l == 0 && xin16 && x->w16 && (4 * H) % 128 == 0) {
      // the bf16 minibatch rows (padded to 64-deep k-tiles) through the wide path's LDS-DMA GEMM
      // into f32 Gx + b_ih: the same k-steps in the same order over the same bf16 operands (zeros
      // past O), the bias added as the layered epilogue adds it -- bitwise gemm_bf16_kernel's Gx
      wide::WideBatch wb{};
      for (int d = 0; d < 2; ++d) {
        wide::WideProblem &P = wb.p[d];
        P.a = xin16;
        P.lda = x->ldx16;
        P.b = x->wih16[z][d];
        P.ldb = x->ldx16;
        P.c = x->g[z][l] + d * 4 * H;
        P.ldc = 8 * H;
        P.bias = ih_bias(x, L, d);
        P.m = b * W;
        P.n = 4 * H;
        P.k = x->ldx16;
      }
      if (int rc = wide::run(wide::WK_F32, wb, 2, b * W, 4 * H, 0, st)) return rc;
    } else if (int rc = gemm_fwd(x, p, 2, L.in, b * W, 4 * H, PPO_ACT_IDENTITY, false, st)) {
      return rc;
    }
    for (int s = 0; s < W; ++s) {
      if ((s > 0 || fusex) && fused_step) {
        StepArgs a{};
        a.cell.g = x->g[z][l];
        a.cell.b_hh[0] = P + L.b_hh[0];
        a.cell.b_hh[1] = P + L.b_hh[1];
        a.cell.c = x->c[z][l];
        // the layer output h in f32 feeds only a stacked layer and the rollout's LSTM-output copy
        // (ppo_lstm_forward): a one-layer net's minibatch step (fusex) does not write it
        a.cell.y = (fusex && N.layers == 1) ? nullptr : x->y[z][l];
        a.cell.hp = x->hp[z][l];
        a.cell.hp16 = b16 ? x->hp16[z][l] : nullptr;
        const bool top = l == N.layers - 1;
        a.cell.feat_mode = top ? (z == 0 ? 1 : 2) : 0;
        a.cell.feat = z == 0 ? x->feat_a : x->feat_c;
        a.cell.feat16 = (top && z == 0 && feat16_on(x)) ? x->feat16 : nullptr;
        a.cell.act = x->cfg.activation;
        a.cell.b = b;
        a.cell.w = W;
        a.cell.h = H;
        a.cell.s = s;
        a.whh[0] = P + L.w_hh[0];
        a.whh[1] = P + L.w_hh[1];
        const dim3 grid(ceil_div(b, kStepRowsMb), H / kStepUnits, 2), block(4 * kStepRowsMb);
        const dim3 grid_r(ceil_div(b, 64), H / kStepUnits, 2);  // the rollout kernel's 64 rows
        if (fusex) {
          const int ldx = x->ldx16;
          for (int d = 0; d < 2; ++d) {
            a.whh16[d] = x->w16 + L.w_hh[d];
            a.wih16[d] = x->wih16[z][d];
            a.b_ih[d] = ih_bias(x, L, d);
          }
          a.x16 = xin16;
          a.ldx = ldx;
          const int pipe = lstm_step_pipe_env();
          TimRec rec{KC_LSTM, pipe == 2 ? "lstm_step_fwdx_kernel<2>" : "lstm_step_fwdx_kernel<1>", 0.0, 0.0};
          if (tim_active()) {
            const double kk = ldx + (s > 0 ? H : 0);
            rec.flops = 2.0 * 2 * b * 4.0 * H * kk;
            // W_ih (and W_hh) images and the bf16 rows in; gates / c (/ h unless one-layer) out (f32) and the next
            // row's bf16 h_prev; s > 0: the staged bf16 h_prev and c_prev in
            rec.bytes = 2.0 * 4 * H * ldx * 2 + 2.0 * b * ldx * 2 +
                        2.0 * b * H * (4.0 * (a.cell.y ? 6 : 5) + 2.0) +
                        (s > 0 ? 2.0 * 4 * H * H * 2 + 2.0 * b * H * (2.0 + 4.0) : 0.0);
          }
          if (pipe == 2) launch_k(rec, lstm_step_fwdx_kernel<2>, grid, block, 0, st, a);
          else launch_k(rec, lstm_step_fwdx_kernel<1>, grid, block, 0, st, a);
          PPO_LAUNCHED();
          continue;
        }
        // the launched instantiation's name (rocprof's, for the traffic table)
        TimRec rec{KC_LSTM,
                   x->w16 ? (x->rollout ? "lstm_step_fwd_rollout_kernel"
                                        : (lstm_step_pipe_env() == 2 ? "lstm_step_fwd_kernel<true, 2>"
                                                                     : "lstm_step_fwd_kernel<true, 1>"))
                          : "lstm_step_fwd_kernel<false, 0>",
                   0.0, 0.0};
        if (tim_active()) {
          rec.flops = 2.0 * 2 * b * 4.0 * H * H;
          // W_hh and h_prev once, Gx / c_prev / h_prev in, gates / c / h out (f32), h_prev out
          // (bf16 in bf16 mode); W16: W_hh and the staged h_prev in bf16, no f32 h_prev read
          rec.bytes = x->w16 ? 2.0 * 2 * 4.0 * H * H + 2.0 * b * H * (2.0 + 4.0 * (4 + 1 + 4 + 2) + 2.0)
                             : 4.0 * 2 * 4.0 * H * H +
                                   2.0 * b * H * (4.0 * (1 + 4 + 2 + 4 + 2) + (b16 ? 2.0 : 4.0));
        }
        if (x->w16) {
          a.whh16[0] = x->w16 + L.w_hh[0];
          a.whh16[1] = x->w16 + L.w_hh[1];
          if (x->rollout && x->defer_steps) {  // forward_all launches it with the other net's
            PPO_REQUIRE(x->npend[z] < 16, "ppo_lstm: too many deferred steps");
            x->pend[z][x->npend[z]++] = a;
            continue;
          }
          if (x->rollout) launch_k(rec, lstm_step_fwd_rollout_kernel, grid_r, dim3(256), 0, st, a);
          else if (lstm_step_pipe_env() == 2) launch_k(rec, lstm_step_fwd_kernel<true, 2>, grid, block, 0, st, a);
          else launch_k(rec, lstm_step_fwd_kernel<true, 1>, grid, block, 0, st, a);
        } else {
          launch_k(rec, lstm_step_fwd_kernel<false, 0>, grid, block, 0, st, a);
        }
        PPO_LAUNCHED();
        continue;
      }
      if (s > 0) {
        GemmProblem q[2] = {};
        for (int d = 0; d < 2; ++d) {
          const int tprev = d == 0 ? s - 1 : W - s;
          q[d].a = x->y[z][l] + static_cast<int64_t>(tprev) * 2 * H + d * H;
          q[d].lda = static_cast<int64_t>(W) * 2 * H;
          q[d].b = P + L.w_hh[d];
          q[d].ldb = H;
          q[d].c = x->gh + d * 4 * H;
          q[d].ldc = 8 * H;
          q[d].bias = P + L.b_hh[d];
          q[d].m = b;
          q[d].n = 4 * H;
        }
        if (int rc = gemm_fwd(x, q, 2, H, b, 4 * H, PPO_ACT_IDENTITY, false, st)) return rc;
      }
      CellArgs a{};
      a.g = x->g[z][l];
      a.gh = s > 0 ? x->gh : nullptr;
      a.b_hh[0] = P + L.b_hh[0];
      a.b_hh[1] = P + L.b_hh[1];
      a.c = x->c[z][l];
      a.y = x->y[z][l];
      a.hp = x->hp[z][l];
      a.hp16 = b16 ? x->hp16[z][l] : nullptr;
      const bool top = l == N.layers - 1;
      a.feat_mode = top ? (z == 0 ? 1 : 2) : 0;
      a.feat = z == 0 ? x->feat_a : x->feat_c;
      a.feat16 = (top && z == 0 && feat16_on(x)) ? x->feat16 : nullptr;
      a.act = x->cfg.activation;
      a.b = b;
      a.w = W;
      a.h = H;
      a.s = s;
      launch_k(TimRec{KC_LSTM, "lstm_cell_fwd_kernel", 0.0, 0.0}, lstm_cell_fwd_kernel,
               dim3(ceil_div(static_cast<int64_t>(b) * 2 * (H / 4), 256)), dim3(256), 0, st, a);
      PPO_LAUNCHED();
    }
  }
  return 0;
}

// MLP forward: m1 (and m2 on the same input, the actor's mean / logstd pair) over in [b][in0]
// in16 (nullable): the input rows as bf16 (the bf16 actor features), read instead of in
int mlp_forward(ppo_lstm_ctx *x, const Mlp *m[2], float *const *acts[2], int nm, const float *in,
                int b, hipStream_t st, const __bf16 *in16 = nullptr) {
  const float *P = x->params;
  for (int l = 0; l < m[0]->n; ++l) {
    GemmProblem p[2] = {};
    for (int k = 0; k < nm; ++k) {
      const MlpLayer &L = m[k]->l[l];
      p[k].a = l == 0 ? in : acts[k][l - 1];
      if (l == 0) p[k].a16 = in16;
      p[k].lda = L.in;
      p[k].b = P + L.w;
      p[k].ldb = L.in;
      p[k].c = acts[k][l];
      p[k].ldc = L.out;
      p[k].bias = L.b >= 0 ? P + L.b : nullptr;
      p[k].m = b;
      p[k].n = L.out;
    }
    const MlpLayer &L0 = m[0]->l[l];
    if (int rc = gemm_fwd(x, p, nm, L0.in, b, L0.out, L0.act, false, st)) return rc;
  }
  return 0;
}

// MLP backward from dz (gradient of the output layer's pre-activation, [b][out]); weight grads
// into the slabs, the input gradient (times act'(input) of the feature activation) into din.
// in16 (nullable): the input rows as bf16 -- the first layer's weight-gradient B operand and the
// input gradient's activation-derivative operand
int mlp_backward(ppo_lstm_ctx *x, const Mlp *m[2], float *const *acts[2], int nm, const float *in,
                 float *const *pp[2], float *din, int64_t ld_din, int feat_act, int b,
                 hipStream_t st, bool sum_din = true, const __bf16 *in16 = nullptr) {
  // pp[k]: the problem's two ping-pong buffers; pp[k][0] holds the output-layer gradient
  const float *P = x->params;
  float *cur[2] = {pp[0][0], nm == 2 ? pp[1][0] : nullptr};
  for (int l = m[0]->n - 1; l >= 0; --l) {
    GemmProblem p[2] = {};
    for (int k = 0; k < nm; ++k) {
      const MlpLayer &L = m[k]->l[l];
      p[k].a = cur[k];
      p[k].lda = L.out;
      p[k].b = l == 0 ? in : acts[k][l - 1];
      if (l == 0) p[k].b16 = in16;
      p[k].ldb = L.in;
      p[k].c = x->slabs + L.w;
      p[k].ldc = L.in;
      p[k].colsum = L.b >= 0 ? x->slabs + L.b : nullptr;
      p[k].m = L.out;
      p[k].n = L.in;
    }
    const MlpLayer &L0 = m[0]->l[l];
    if (int rc = gemm_partial(x, p, nm, b, L0.out, L0.in, st)) return rc;
    // dX = (dZ W) * act'(X): for l > 0 into the other ping-pong buffer; l == 0: the features
    GemmProblem q[2] = {};
    float *nxt[2] = {nullptr, nullptr};
    for (int k = 0; k < nm; ++k) {
      const MlpLayer &L = m[k]->l[l];
      q[k].a = cur[k];
      q[k].lda = L.out;
      q[k].b = P + L.w;
      q[k].ldb = L.in;
      if (l > 0) {
        nxt[k] = pp[k][(cur[k] == pp[k][0]) ? 1 : 0];
        q[k].c = nxt[k];
        q[k].ldc = L.in;
        q[k].aux = acts[k][l - 1];
      } else {
        q[k].c = k == 0 ? din : x->tmp;
        q[k].ldc = ld_din;
        q[k].aux = in;
        q[k].aux16 = in16;
      }
      q[k].m = b;
      q[k].n = L.in;
    }
    const int act = l > 0 ? m[0]->l[l - 1].act : feat_act;
    if (int rc = gemm_dx(x, q, nm, L0.out, b, L0.in, act, st)) return rc;
    // the two actor MLPs read the same features: sum their dX (sum_din = false: the consumer
    // adds x->tmp where it reads din, lstm_backward's dy2)
    if (l == 0 && nm == 2 && sum_din) {
      const int64_t n = static_cast<int64_t>(b) * ld_din;
      launch_k(TimRec{KC_LSTM, "add_inplace_kernel", 0.0, 0.0}, add_inplace_kernel,
               dim3(ceil_div(n, 256)), dim3(256), 0, st, din, x->tmp, n);
      PPO_LAUNCHED();
    }
    cur[0] = nxt[0];
    cur[1] = nxt[1];
  }
  return 0;
}

// BPTT of LSTM net z given dY of the top layer (actor: full [b*W][2H] in x->dy[0]; critic: the
// [b][2H] gradient of h at t = W-1 in x->dy[0]); weight grads into the slabs.
// xin16 (bf16 mode): the gathered rows as bf16; dG and h_prev then come from dg16 / hp16.
int lstm_backward(ppo_lstm_ctx *x, int z, const float *xin, const __bf16 *xin16, int b,
                  hipStream_t st, const float *dy2 = nullptr) {
  const LstmNet &N = x->net[z];
  const int H = N.hidden, W = x->cfg.window;
  const float *P = x->params;
  const bool b16 = x->prec == PPO_PREC_BF16;
  // the recurrent gradient on the wide path (W_hh^T images made by prep_w16); PPO_LSTM_DHREC=0
  // keeps gemm_bf16_kernel (the bitwise test's reference)
  const char *dv = getenv("PPO_LSTM_DHREC");
  const bool wide_rec = b16 && x->w16 && H % 64 == 0 && !(dv && atoi(dv) == 0);
  int cur = 0;
  for (int l = N.layers - 1; l >= 0; --l) {
    const LstmLayer &L = N.l[l];
    const bool top = l == N.layers - 1;
    for (int s = 0; s < W; ++s) {
      if (s > 0) {
        GemmProblem p[2] = {};
        for (int d = 0; d < 2; ++d) {
          const int tn = d == 0 ? W - s : s - 1;  // the step back-propagated at s - 1
          p[d].a = x->g[z][l] + static_cast<int64_t>(tn) * 8 * H + d * 4 * H;
          if (b16) p[d].a16 = x->dg16[z][l] + static_cast<int64_t>(tn) * 8 * H + d * 4 * H;
          if (b16 && x->w16) p[d].b16 = x->w16 + L.w_hh[d];
          p[d].lda = static_cast<int64_t>(W) * 8 * H;
          p[d].b = P + L.w_hh[d];
          p[d].ldb = H;
          p[d].c = x->dhrec + d * H;
          p[d].ldc = 2 * H;
          p[d].m = b;
          p[d].n = H;
        }
        if (wide_rec) {
          // the wide path's LDS-DMA GEMM over the same bf16 operands (dG rows k-inner, W_hh^T
          // images), the same k-steps of 16 in order: bitwise the layered dh_rec
          wide::WideBatch wb{};
          for (int d = 0; d < 2; ++d) {
            wide::WideProblem &Q = wb.p[d];
            Q.a = p[d].a16;
            Q.lda = p[d].lda;
            Q.b = x->whht16[z][l][d];
            Q.ldb = 4 * H;
            Q.c = p[d].c;
            Q.ldc = p[d].ldc;
            Q.m = b;
            Q.n = H;
            Q.k = 4 * H;
          }
          if (int rc = wide::run(wide::WK_F32, wb, 2, b, H, 0, st)) return rc;
        } else if (int rc = gemm_fwd(x, p, 2, 4 * H, b, H, PPO_ACT_IDENTITY, true, st)) {
          return rc;
        }
      }
      CellBwdArgs a{};
      a.g = x->g[z][l];
      a.c = x->c[z][l];
      a.dy_mode = (top && z == 1) ? 2 : 1;
      a.dy = x->dy[cur];
      a.dy2 = top ? dy2 : nullptr;  // the top layer's second dY term (the actor's log-std MLP)
      a.dy_last = x->dy[cur];
      a.dh_rec = s > 0 ? x->dhrec : nullptr;
      a.dcarry = x->dcarry;
      a.dg16 = b16 ? x->dg16[z][l] : nullptr;
      a.b = b;
      a.w = W;
      a.h = H;
      a.s = s;
      launch_k(TimRec{KC_LSTM, "lstm_cell_bwd_kernel", 0.0, 0.0}, lstm_cell_bwd_kernel,
               dim3(ceil_div(static_cast<int64_t>(b) * 2 * (H / 4), 256)), dim3(256), 0, st, a);
      PPO_LAUNCHED();
    }
    const float *in = l == 0 ? xin : x->y[z][l - 1];
    GemmProblem pi[2] = {}, ph[2] = {};
    for (int d = 0; d < 2; ++d) {
      pi[d].a = x->g[z][l] + d * 4 * H;
      if (b16) pi[d].a16 = x->dg16[z][l] + d * 4 * H;
      pi[d].lda = 8 * H;
      pi[d].b = in;
      pi[d].b16 = l == 0 ? xin16 : nullptr;
      pi[d].ldb = (l == 0 && xin16) ? x->ldx16 : L.in;
      pi[d].c = x->slabs + L.w_ih[d];
      pi[d].ldc = L.in;
      pi[d].colsum = x->slabs + L.b_ih[d];
      pi[d].m = 4 * H;
      pi[d].n = L.in;
      ph[d] = pi[d];
      ph[d].b = x->hp[z][l] + d * H;
      ph[d].b16 = b16 ? x->hp16[z][l] + d * H : nullptr;
      ph[d].ldb = 2 * H;
      ph[d].c = x->slabs + L.w_hh[d];
      ph[d].ldc = H;
      ph[d].colsum = x->slabs + L.b_hh[d];
      ph[d].n = H;
    }
    // bf16 mode, rows filling whole 64-row k-tiles: dW_ih (layer 0: the padded bf16 rows) and
    // dW_hh on the wide path's split-K WGRAD (LDS-DMA, both bf16 operands k-outer); dW_ih's
    // launch also sums dG's columns per split (wide_gemm.h acol) into the b_ih and b_hh slabs --
    // the same column sums gemm_bf16_kernel's COLSUM took, in its own fixed order
    const bool wide_w = b16 && xin16 && (static_cast<int64_t>(b) * W) % 64 == 0 &&
                        (4 * H) % 128 == 0 && H % 8 == 0;
    if (wide_w) {
      wide::WideBatch wb{};
      for (int d = 0; d < 2; ++d) {
        const bool ih = l == 0;  // layer 0: x16 is the k-outer bf16 B operand
        wide::WideProblem &Q = wb.p[d];
        Q.a = x->dg16[z][l] + d * 4 * H;
        Q.lda = 8 * H;
        Q.b = ih ? xin16 : nullptr;
        Q.ldb = x->ldx16;
        Q.c = x->slabs + L.w_ih[d];
        Q.ldc = L.in;
        Q.m = 4 * H;
        Q.n = L.in;
        Q.k = b * W;
        Q.slab_stride = x->total;
        Q.acol = x->slabs + L.b_ih[d];
        Q.acol2 = x->slabs + L.b_hh[d];
      }
      wb.splits = x->splits;
      if (l == 0) {
        if (int rc = wide::run(wide::WK_WGRAD, wb, 2, 4 * H, L.in, b * W, st)) return rc;
      } else {  // stacked layers' f32 inputs: the bf16-source GEMM, bias partials for both
        for (int d = 0; d < 2; ++d) pi[d].colsum2 = x->slabs + L.b_hh[d];
        if (int rc = gemm_partial(x, pi, 2, b * W, 4 * H, L.in, st)) return rc;
      }
      for (int d = 0; d < 2; ++d) {
        wide::WideProblem &Q = wb.p[d];
        Q.b = x->hp16[z][l] + d * H;
        Q.ldb = 2 * H;
        Q.c = x->slabs + L.w_hh[d];
        Q.ldc = H;
        Q.n = H;
        Q.acol = Q.acol2 = nullptr;
      }
      if (int rc = wide::run(wide::WK_WGRAD, wb, 2, 4 * H, H, b * W, st)) return rc;
    } else {
      if (int rc = gemm_partial(x, pi, 2, b * W, 4 * H, L.in, st)) return rc;
      if (int rc = gemm_partial(x, ph, 2, b * W, 4 * H, H, st)) return rc;
    }
    if (l > 0) {  // dY of the layer below = sum_d dG_d W_ih_d (no activation between layers)
      const int nxt = cur ^ 1;
      for (int d = 0; d < 2; ++d) {
        GemmProblem p{};
        p.a = x->g[z][l] + d * 4 * H;
        if (b16) p.a16 = x->dg16[z][l] + d * 4 * H;
        if (b16 && x->w16 && L.in % 4 == 0) p.b16 = x->w16 + L.w_ih[d];
        p.lda = 8 * H;
        p.b = P + L.w_ih[d];
        p.ldb = L.in;
        p.c = d == 0 ? x->dy[nxt] : x->tmp;
        p.ldc = L.in;
        p.m = b * W;
        p.n = L.in;
        if (int rc = gemm_fwd(x, &p, 1, 4 * H, b * W, L.in, PPO_ACT_IDENTITY, true, st)) return rc;
      }
      const int64_t n = static_cast<int64_t>(b) * W * L.in;
      launch_k(TimRec{KC_LSTM, "add_inplace_kernel", 0.0, 0.0}, add_inplace_kernel,
               dim3(ceil_div(n, 256)), dim3(256), 0, st, x->dy[nxt], x->tmp, n);
      PPO_LAUNCHED();
      cur = nxt;
    }
  }
  return 0;
}

int check_rows(ppo_lstm_ctx *x, int b) {
  PPO_REQUIRE(b >= 0 && b <= x->rows, "ppo_lstm: %d rows exceed the workspace (%lld)", b,
              static_cast<long long>(x->rows));
  PPO_REQUIRE(x->params != nullptr, "ppo_lstm: parameters not bound (ppo_lstm_bind_params)");
  return 0;
}

int forward_all(ppo_lstm_ctx *x, const float *xin, const __bf16 *xin16, int b, hipStream_t st) {
  // the rollout (one-layer nets, W16 step kernels): both nets' projections and first steps, then
  // each step s of both nets as one launch (lstm_step_fwd_rollout2_kernel) -- the same per-net
  // launches' work in stream order, so bitwise the same; PPO_LSTM_PAIR_STEPS=0 launches per net
  const int H = x->cfg.latent, W = x->cfg.window;
  const char *pv = getenv("PPO_LSTM_PAIR_STEPS");
  const bool pair = x->rollout && x->w16 && x->fused_step && x->prec == PPO_PREC_BF16 &&
                    H % kStepUnits == 0 && x->net[0].layers == 1 && x->net[1].layers == 1 &&
                    W <= 16 && !(pv && atoi(pv) == 0);
  struct DeferScope {
    ppo_lstm_ctx *x;
    ~DeferScope() { x->defer_steps = 0; }
  } defer_scope{x};
  x->defer_steps = pair ? 1 : 0;
  x->npend[0] = x->npend[1] = 0;
  if (int rc = lstm_forward(x, 0, xin, xin16, b, st)) return rc;
  if (int rc = lstm_forward(x, 1, xin, xin16, b, st)) return rc;
  x->defer_steps = 0;
  PPO_REQUIRE(x->npend[0] == x->npend[1], "ppo_lstm: paired rollout steps %d / %d", x->npend[0],
              x->npend[1]);
  for (int i = 0; i < x->npend[0]; ++i) {
    StepArgs2 a2{};
    a2.n[0] = x->pend[0][i];
    a2.n[1] = x->pend[1][i];
    TimRec rec{KC_LSTM, "lstm_step_fwd_rollout2_kernel", 0.0, 0.0};
    launch_k(rec, lstm_step_fwd_rollout2_kernel, dim3(ceil_div(b, 64), H / kStepUnits, 4),
             dim3(256), 0, st, a2);
    PPO_LAUNCHED();
  }
  const Mlp *am[2] = {&x->mu, &x->ls};
  float *const *aa[2] = {x->act_mu, x->act_ls};
  if (int rc = mlp_forward(x, am, aa, 2, x->feat_a, b, st, feat16_on(x) ? x->feat16 : nullptr))
    return rc;
  const Mlp *cm[2] = {&x->vc, nullptr};
  float *const *ca[2] = {x->act_v, nullptr};
  return mlp_forward(x, cm, ca, 1, x->feat_c, b, st);
}

}  // namespace

extern "C" int ppo_lstm_ctx_create(const ppo_lstm_cfg *cfg, int device, ppo_lstm_ctx **out) {
  PPO_REQUIRE(cfg != nullptr && out != nullptr, "ppo_lstm_ctx_create: null argument");
  const ppo_lstm_cfg &c = *cfg;
  PPO_REQUIRE(c.obs_dim > 0 && c.window > 0 && c.act_dim > 0 && c.act_dim <= kMaxA,
              "ppo_lstm_ctx_create: bad obs/window/act (%d, %d, %d)", c.obs_dim, c.window,
              c.act_dim);
  PPO_REQUIRE(c.latent > 0 && c.latent % 4 == 0 && c.latent <= 1024,
              "ppo_lstm_ctx_create: latent size %d must be a multiple of 4 in [4, 1024]", c.latent);
  PPO_REQUIRE(c.actor_layers >= 1 && c.actor_layers <= PPO_MAX_LAYERS,
              "ppo_lstm_ctx_create: %d feature-extractor layers", c.actor_layers);
  PPO_REQUIRE(c.n_hidden >= 1 && c.n_hidden <= PPO_MAX_LAYERS,
              "ppo_lstm_ctx_create: %d hidden layers", c.n_hidden);
  PPO_REQUIRE(c.activation >= PPO_ACT_RELU && c.activation <= PPO_ACT_ELU,
              "ppo_lstm_ctx_create: activation %d", c.activation);
  PPO_REQUIRE(c.max_rows > 0, "ppo_lstm_ctx_create: max_rows %d", c.max_rows);
  for (int l = 0; l < c.n_hidden; ++l)
    PPO_REQUIRE(c.hidden[l] > 0 && c.hidden[l] <= 4096, "ppo_lstm_ctx_create: hidden width %d",
                c.hidden[l]);
  ppo_lstm_ctx *x = new (std::nothrow) ppo_lstm_ctx();
  PPO_REQUIRE(x != nullptr, "ppo_lstm_ctx_create: out of host memory");
  x->cfg = c;
  x->device = device;
  x->prec = PPO_PREC_F32;
  x->ent_log_share = 1.f;
  x->fused_step = g_lstm_fused_step;
  x->rollout = 0;
  x->splits = g_lstm_splits;
  const int H = c.latent, W = c.window, O = c.obs_dim, A = c.act_dim;
  int64_t off = 0;
  // LSTMActor.parameters(): feature_extractor, actor, actor_logstd (lstm_actor.py:12-38)
  add_lstm(x->net[0], c.actor_layers, O, H, off, x->offsets);
  add_mlp(x->mu, W * 2 * H, c, A, PPO_ACT_TANH, off, x->offsets);
  add_mlp(x->ls, W * 2 * H, c, A, PPO_ACT_TANH, off, x->offsets);
  x->n_actor = off;
  // LSTMCritic.parameters(): feature_extractor.0 (one layer), network (lstm_critic.py:19-31)
  add_lstm(x->net[1], 1, O, H, off, x->offsets);
  add_mlp(x->vc, 2 * H, c, 1, PPO_ACT_IDENTITY, off, x->offsets);
  x->total = off;
  int maxw = std::max(A, 1);
  for (int l = 0; l < c.n_hidden; ++l) maxw = std::max(maxw, c.hidden[l]);
  x->maxw = maxw;
  const int64_t R = c.max_rows;
  x->rows = R;
  // workspace carve-out
  int64_t need = 0;
  auto take = [&](int64_t n) {
    const int64_t at = need;
    need = align_up(need + n, kWsAlign);
    return at;
  };
  const int64_t o_x = take(R * W * O);
  // bf16 buffers: half the floats; the gathered rows padded to the wide GEMM's 64-deep k-tiles
  // and 128-row tiles (its A operand reads whole tiles)
  const int ldx16 = static_cast<int>(align_up(O, 64));
  const int64_t o_x16 = take(((R * W + 128) * ldx16 + 1) / 2);
  int64_t o_wih16[2][2];
  for (int z = 0; z < 2; ++z)
    for (int d = 0; d < 2; ++d) o_wih16[z][d] = take((4LL * H * ldx16 + 1) / 2);
  const int64_t o_p16 = take((x->total + 1) / 2);
  int64_t o_g[2][PPO_MAX_LAYERS], o_c[2][PPO_MAX_LAYERS], o_y[2][PPO_MAX_LAYERS],
      o_hp[2][PPO_MAX_LAYERS], o_dg16[2][PPO_MAX_LAYERS], o_hp16[2][PPO_MAX_LAYERS],
      o_whht16[2][PPO_MAX_LAYERS][2];
  for (int z = 0; z < 2; ++z)
    for (int l = 0; l < x->net[z].layers; ++l) {
      o_g[z][l] = take(R * W * 8 * H);
      o_c[z][l] = take(R * W * 2 * H);
      o_y[z][l] = take(R * W * 2 * H);
      o_hp[z][l] = take(R * W * 2 * H);
      o_dg16[z][l] = take((R + 128) * W * 4 * H);
      for (int d = 0; d < 2; ++d) o_whht16[z][l][d] = take(2LL * H * H);
      o_hp16[z][l] = take(R * W * H);
    }
  const int64_t o_gh = take(R * 8 * H), o_dhrec = take(R * 2 * H), o_dcarry = take(R * 2 * H);
  const int64_t o_dy0 = take(R * W * 2 * H), o_dy1 = take(R * W * 2 * H);
  const int64_t o_tmp = take(R * std::max<int64_t>(W * 2 * H, maxw));
  const int64_t o_fa = take(R * W * 2 * H), o_fc = take(R * 2 * H);
  const int64_t o_f16 = take(R * W * H);
  int64_t o_mu[PPO_MAX_LAYERS + 1], o_ls[PPO_MAX_LAYERS + 1], o_v[PPO_MAX_LAYERS + 1];
  for (int l = 0; l <= c.n_hidden; ++l) {
    o_mu[l] = take(R * x->mu.l[l].out);
    o_ls[l] = take(R * x->ls.l[l].out);
    o_v[l] = take(R * x->vc.l[l].out);
  }
  int64_t o_dz[3][2];
  for (int k = 0; k < 3; ++k)
    for (int p = 0; p < 2; ++p) o_dz[k][p] = take(R * maxw);
  const int64_t o_slabs = take(kSplits * x->total);
  const int64_t o_rp = take(R * 3);
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc(&x->ws, sizeof(float) * std::max<int64_t>(need, 1));
  if (e != hipSuccess) {
    set_error("ppo_lstm_ctx_create: hipMalloc(%lld floats) failed: %s",
              static_cast<long long>(need), hipGetErrorString(e));
    delete x;
    return PPO_EHIP;
  }
  float *w = x->ws;
  x->x = w + o_x;
  x->x16 = reinterpret_cast<__bf16 *>(w + o_x16);
  x->ldx16 = ldx16;
  for (int z = 0; z < 2; ++z)
    for (int d = 0; d < 2; ++d) x->wih16[z][d] = reinterpret_cast<__bf16 *>(w + o_wih16[z][d]);
  x->p16 = reinterpret_cast<__bf16 *>(w + o_p16);
  for (int z = 0; z < 2; ++z)
    for (int l = 0; l < x->net[z].layers; ++l) {
      x->g[z][l] = w + o_g[z][l];
      x->c[z][l] = w + o_c[z][l];
      x->y[z][l] = w + o_y[z][l];
      x->hp[z][l] = w + o_hp[z][l];
      x->dg16[z][l] = reinterpret_cast<__bf16 *>(w + o_dg16[z][l]);
      for (int d = 0; d < 2; ++d)
        x->whht16[z][l][d] = reinterpret_cast<__bf16 *>(w + o_whht16[z][l][d]);
      x->hp16[z][l] = reinterpret_cast<__bf16 *>(w + o_hp16[z][l]);
    }
  x->gh = w + o_gh;
  x->dhrec = w + o_dhrec;
  x->dcarry = w + o_dcarry;
  x->dy[0] = w + o_dy0;
  x->dy[1] = w + o_dy1;
  x->tmp = w + o_tmp;
  x->feat_a = w + o_fa;
  x->feat_c = w + o_fc;
  x->feat16 = reinterpret_cast<__bf16 *>(w + o_f16);
  for (int l = 0; l <= c.n_hidden; ++l) {
    x->act_mu[l] = w + o_mu[l];
    x->act_ls[l] = w + o_ls[l];
    x->act_v[l] = w + o_v[l];
  }
  for (int k = 0; k < 3; ++k)
    for (int p = 0; p < 2; ++p) x->dz[k][p] = w + o_dz[k][p];
  x->slabs = w + o_slabs;
  // the alignment padding between tensors is never written by a GEMM: zero slabs reduce to 0;
  // the padded bf16 rows / images keep zero pad columns (only their first O are ever written)
  e = hipMemset(x->slabs, 0, sizeof(float) * kSplits * x->total);
  if (e == hipSuccess) e = hipMemset(x->x16, 0, sizeof(__bf16) * (R * W + 128) * ldx16);
  for (int z = 0; z < 2 && e == hipSuccess; ++z)
    for (int d = 0; d < 2 && e == hipSuccess; ++d)
      e = hipMemset(x->wih16[z][d], 0, sizeof(__bf16) * 4LL * H * ldx16);
  if (e != hipSuccess) {
    set_error("ppo_lstm_ctx_create: hipMemset failed: %s", hipGetErrorString(e));
    (void)hipFree(x->ws);
    delete x;
    return PPO_EHIP;
  }
  x->row_part = w + o_rp;
  *out = x;
  return 0;
}

extern "C" int ppo_lstm_ctx_destroy(ppo_lstm_ctx *x) {
  if (!x) return 0;
  (void)timing_enable(x->tim, 0, 0);
  for (int i = 0; i < 2 * x->tim.capacity; ++i) (void)hipEventDestroy(x->tim.ev[i]);
  delete[] x->tim.ev;
  delete[] x->tim.cls;
  delete[] x->tim.kname;
  delete[] x->tim.flops;
  delete[] x->tim.bytes;
  if (x->ws) (void)hipFree(x->ws);
  delete x;
  return 0;
}

extern "C" int ppo_lstm_param_layout(const ppo_lstm_ctx *x, int64_t *offsets, int max_tensors,
                                     int64_t *total, int64_t *n_actor) {
  PPO_REQUIRE(x != nullptr, "ppo_lstm_param_layout: null ctx");
  const int n = static_cast<int>(x->offsets.size());
  if (offsets)
    for (int i = 0; i < std::min(n, max_tensors); ++i) offsets[i] = x->offsets[i];
  if (total) *total = x->total;
  if (n_actor) *n_actor = x->n_actor;
  return n;
}

extern "C" int ppo_lstm_bind_params(ppo_lstm_ctx *x, float *params_d) {
  PPO_REQUIRE(x != nullptr && params_d != nullptr, "ppo_lstm_bind_params: null argument");
  PPO_REQUIRE(reinterpret_cast<uintptr_t>(params_d) % 64 == 0,
              "ppo_lstm_bind_params: parameter buffer must be 64-B aligned");
  x->params = params_d;
  return 0;
}

extern "C" int ppo_lstm_loss_entropy_share(ppo_lstm_ctx *x, float share) {
  PPO_REQUIRE(x != nullptr, "ppo_lstm_loss_entropy_share: null ctx");
  x->ent_log_share = share;
  return 0;
}

extern "C" int ppo_lstm_set_precision(ppo_lstm_ctx *x, int prec) {
  PPO_REQUIRE(x != nullptr, "ppo_lstm_set_precision: null ctx");
  PPO_REQUIRE(prec == PPO_PREC_F32 || prec == PPO_PREC_BF16, "ppo_lstm_set_precision: %d", prec);
  x->prec = prec;
  return 0;
}

// bf16 mode: the LSTM GEMMs read a bf16 copy of the parameters made once per call (the rounding
// their staging applied to the f32 masters per workgroup) and layer 0's W_ih as padded images for
// the wide projection (bwd: and the W_hh^T images of the recurrent-gradient GEMM); x->w16 is
// cleared again when the caller's W16Scope ends
struct W16Scope {
  ppo_lstm_ctx *x;
  ~W16Scope() { x->w16 = nullptr; }
};
int prep_w16(ppo_lstm_ctx *x, hipStream_t st, bool bwd) {
  if (x->prec != PPO_PREC_BF16) return 0;
  const int H = x->cfg.latent, O = x->cfg.obs_dim;
  launch_k(TimRec{KC_GATHER, "lstm_params_bf16_kernel", 0.0, 6.0 * x->total},
           lstm_params_bf16_kernel, dim3(ceil_div(x->total, 4 * 256)), dim3(256), 0, st,
           x->params, x->p16, x->total);
  PPO_LAUNCHED();
  x->w16 = x->p16;
  WihImages wi{};  // the input projection's B operands, at the padded row stride
  int k = 0;
  for (int z = 0; z < 2; ++z)
    for (int d = 0; d < 2; ++d, ++k) {
      wi.src[k] = x->params + x->net[z].l[0].w_ih[d];
      wi.dst[k] = x->wih16[z][d];
    }
  wi.rows = 4 * H;
  wi.in = O;
  wi.ld16 = x->ldx16;
  launch_k(TimRec{KC_GATHER, "lstm_wih_image_kernel", 0.0, 4.0 * 4 * H * O * 6.0},
           lstm_wih_image_kernel, dim3(ceil_div(4LL * 4 * H * O, 256)), dim3(256), 0, st, wi);
  PPO_LAUNCHED();
  if (!bwd || H % 64 != 0) return 0;
  WhhTImages wt{};
  for (int z = 0; z < 2; ++z)
    for (int l = 0; l < x->net[z].layers; ++l)
      for (int d = 0; d < 2; ++d, ++wt.n) {
        wt.src[wt.n] = x->params + x->net[z].l[l].w_hh[d];
        wt.dst[wt.n] = x->whht16[z][l][d];
      }
  wt.h = H;
  launch_k(TimRec{KC_GATHER, "lstm_whh_t_image_kernel", 0.0, 0.0}, lstm_whh_t_image_kernel,
           dim3(ceil_div(wt.n * 4LL * H * H, 256)), dim3(256), 0, st, wt);
  PPO_LAUNCHED();
  return 0;
}

// rows of [W*O] state windows -> xg (f32) or xg16 (bf16, padded stride); rows == nullptr: in order
int gather_rows(ppo_lstm_ctx *x, const float *states, const int32_t *rows, int b, float *xg,
                __bf16 *xg16, hipStream_t st) {
  const int O = x->cfg.obs_dim, din = x->cfg.window * O;
  const int64_t n = static_cast<int64_t>(b) * din;
  if (O % 4 == 0 && reinterpret_cast<uintptr_t>(states) % 16 == 0) {
    launch_k(TimRec{KC_GATHER, "lstm_gather_rows4_kernel", 0.0, 0.0}, lstm_gather_rows4_kernel,
             dim3(ceil_div(n / 4, 256)), dim3(256), 0, st, states, rows, b, din, xg, xg16, O,
             x->ldx16);
  } else {
    launch_k(TimRec{KC_GATHER, "lstm_gather_rows_kernel", 0.0, 0.0}, lstm_gather_rows_kernel,
             dim3(ceil_div(n, 256)), dim3(256), 0, st, states, rows, b, din, xg, xg16, O,
             x->ldx16);
  }
  PPO_LAUNCHED();
  return 0;
}

// The rollout's forward (policy step / forward) in bf16 mode on the minibatch step's operands:
// the parameter images, the window rows as padded bf16 (the gather kernel, rows in order), the
// wide projection and the W16 step kernels -- the same arithmetic as the layered f32-staged form
// (RNE-rounded operands, the same k order), so rollout and update forwards stay bitwise equal
int forward_rollout(ppo_lstm_ctx *x, const float *state_d, int n, hipStream_t st) {
  if (x->prec != PPO_PREC_BF16) return forward_all(x, state_d, nullptr, n, st);
  W16Scope w16_scope{x};
  struct RolloutScope {
    ppo_lstm_ctx *x;
    ~RolloutScope() { x->rollout = 0; }
  } rollout_scope{x};
  x->rollout = 1;
  if (int rc = prep_w16(x, st, false)) return rc;
  if (int rc = gather_rows(x, state_d, nullptr, n, nullptr, x->x16, st)) return rc;
  return forward_all(x, state_d, x->x16, n, st);
}

extern "C" int ppo_lstm_forward(ppo_lstm_ctx *x, const float *state_d, int n, float *mean_d,
                                float *std_d, float *value_d, float *actor_lstm_out_d,
                                float *critic_lstm_out_d, void *stream) {
  PPO_REQUIRE(x != nullptr && state_d != nullptr, "ppo_lstm_forward: null argument");
  if (int rc = check_rows(x, n)) return rc;
  if (n == 0) return 0;
  PPO_HIP_TRY(hipSetDevice(x->device));
  TimingScope ts(x);
  hipStream_t st = as_stream(stream);
  if (int rc = forward_rollout(x, state_d, n, st)) return rc;
  const int A = x->cfg.act_dim, W = x->cfg.window;
  const int64_t yb = sizeof(float) * static_cast<int64_t>(n) * W * 2 * x->cfg.latent;
  if (actor_lstm_out_d)
    PPO_HIP_TRY(hipMemcpyAsync(actor_lstm_out_d, x->y[0][x->net[0].layers - 1], yb,
                               hipMemcpyDeviceToDevice, st));
  if (critic_lstm_out_d)
    PPO_HIP_TRY(hipMemcpyAsync(critic_lstm_out_d, x->y[1][0], yb, hipMemcpyDeviceToDevice, st));
  const int nl = x->cfg.n_hidden;
  if (mean_d)
    PPO_HIP_TRY(hipMemcpyAsync(mean_d, x->act_mu[nl], sizeof(float) * static_cast<int64_t>(n) * A,
                               hipMemcpyDeviceToDevice, st));
  HeadArgs h{};
  h.mean = x->act_mu[nl];
  h.u = x->act_ls[nl];
  h.value = x->act_v[nl];
  h.std_out = std_d;
  h.value_out = value_d;
  h.b = n;
  h.a = A;
  launch_k(TimRec{KC_POLICY_HEAD, "lstm_policy_head_kernel", 0.0, 0.0}, lstm_policy_head_kernel,
           dim3(ceil_div(n, 256)), dim3(256), 0, st, h);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_lstm_policy_step(ppo_lstm_ctx *x, const float *state_d, int n,
                                    const float *eps_d, uint64_t seed, uint64_t offset,
                                    float *action_d, float *logp_d, float *value_d, void *stream) {
  PPO_REQUIRE(x != nullptr && state_d != nullptr, "ppo_lstm_policy_step: null argument");
  PPO_REQUIRE(action_d != nullptr || logp_d == nullptr,
              "ppo_lstm_policy_step: logp needs the action buffer");
  if (int rc = check_rows(x, n)) return rc;
  if (n == 0) return 0;
  PPO_HIP_TRY(hipSetDevice(x->device));
  TimingScope ts(x);
  hipStream_t st = as_stream(stream);
  if (int rc = forward_rollout(x, state_d, n, st)) return rc;
  const int nl = x->cfg.n_hidden;
  HeadArgs h{};
  h.mean = x->act_mu[nl];
  h.u = x->act_ls[nl];
  h.value = x->act_v[nl];
  h.eps = eps_d;
  h.seed = seed;
  h.offset = offset;
  h.action = action_d;
  h.logp_out = logp_d;
  h.value_out = value_d;
  h.b = n;
  h.a = x->cfg.act_dim;
  launch_k(TimRec{KC_POLICY_HEAD, "lstm_policy_head_kernel", 0.0, 0.0}, lstm_policy_head_kernel,
           dim3(ceil_div(n, 256)), dim3(256), 0, st, h);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_lstm_minibatch_grad(ppo_lstm_ctx *x, const float *states_d,
                                       const float *actions_d, const float *logp_d,
                                       const float *adv_d, const float *vt_d,
                                       const int32_t *rows_d, int b, float *grad_d, float *loss_d,
                                       float clip_lo, float clip_hi, float entropy_coef,
                                       float inv_b, float inv_ba, void *stream) {
  PPO_REQUIRE(x != nullptr && states_d && actions_d && logp_d && adv_d && vt_d && rows_d && grad_d,
              "ppo_lstm_minibatch_grad: null argument");
  if (int rc = check_rows(x, b)) return rc;
  PPO_REQUIRE(b > 0, "ppo_lstm_minibatch_grad: empty minibatch");
  PPO_HIP_TRY(hipSetDevice(x->device));
  TimingScope ts(x);
  hipStream_t st = as_stream(stream);
  const ppo_lstm_cfg &c = x->cfg;
  const int W = c.window, A = c.act_dim, H = c.latent, nl = c.n_hidden;
  W16Scope w16_scope{x};
  if (int rc = prep_w16(x, st, true)) return rc;
  // bf16 mode: the gathered rows only feed GEMMs, so they are staged as bf16
  // (rows of O values at a stride of ldx16, a multiple of 64: the wide GEMM's k-tiles)
  const __bf16 *x16 = x->prec == PPO_PREC_BF16 ? x->x16 : nullptr;
  if (int rc = gather_rows(x, states_d, rows_d, b, x->x, const_cast<__bf16 *>(x16), st)) return rc;
  if (int rc = forward_all(x, x->x, x16, b, st)) return rc;
  HeadArgs h{};
  h.mean = x->act_mu[nl];
  h.u = x->act_ls[nl];
  h.value = x->act_v[nl];
  h.actions = actions_d;
  h.old_logp = logp_d;
  h.adv = adv_d;
  h.vt = vt_d;
  h.rows = rows_d;
  h.dzm = x->dz[0][0];
  h.dzs = x->dz[1][0];
  h.dv = x->dz[2][0];
  h.row_part = x->row_part;
  h.clip_lo = clip_lo;
  h.clip_hi = clip_hi;
  h.ent_coef = entropy_coef;
  h.inv_b = inv_b;
  h.inv_ba = inv_ba;
  h.b = b;
  h.a = A;
  launch_k(TimRec{KC_UPDATE_HEAD, "lstm_update_head_kernel", 0.0, 0.0}, lstm_update_head_kernel,
           dim3(ceil_div(b, 256)), dim3(256), 0, st, h);
  PPO_LAUNCHED();
  if (loss_d) {
    launch_k(TimRec{KC_REDUCE, "lstm_loss_kernel", 0.0, 0.0}, lstm_loss_kernel, dim3(1),
             dim3(256), 0, st, x->row_part, b, inv_b, inv_ba, entropy_coef * x->ent_log_share,
             loss_d);
    PPO_LAUNCHED();
  }
  {  // critic: MLP, then BiLSTM (the gradient of h at t = W-1 lands in dy[0])
    const Mlp *cm[2] = {&x->vc, nullptr};
    float *const *ca[2] = {x->act_v, nullptr};
    float *const *pp[2] = {x->dz[2], nullptr};
    if (int rc = mlp_backward(x, cm, ca, 1, x->feat_c, pp, x->dy[0], 2 * H, c.activation, b, st))
      return rc;
    if (int rc = lstm_backward(x, 1, x->x, x16, b, st)) return rc;
  }
  {  // actor: both MLPs into one feature gradient, then BiLSTM
    const Mlp *am[2] = {&x->mu, &x->ls};
    float *const *aa[2] = {x->act_mu, x->act_ls};
    float *const *pp[2] = {x->dz[0], x->dz[1]};
    if (int rc = mlp_backward(x, am, aa, 2, x->feat_a, pp, x->dy[0],
                              static_cast<int64_t>(W) * 2 * H, c.activation, b, st, false,
                              feat16_on(x) ? x->feat16 : nullptr))
      return rc;
    if (int rc = lstm_backward(x, 0, x->x, x16, b, st, x->tmp)) return rc;
  }
  // slabs -> flat gradient, tensor by tensor in a fixed split order
  ReduceArgs r{};
  int ns = 0;
  for (size_t i = 0; i < x->offsets.size(); ++i) {
    PPO_REQUIRE(ns < kMaxSegs, "ppo_lstm_minibatch_grad: too many tensors (%zu)", x->offsets.size());
    ReduceSeg &g = r.seg[ns++];
    g.dst = x->offsets[i];
    g.len = (i + 1 < x->offsets.size() ? x->offsets[i + 1] : x->total) - x->offsets[i];
    g.src = x->slabs + x->offsets[i];
    g.stride = x->total;
    g.nsplit = x->splits;
  }
  r.nseg = ns;
  r.total = x->total;
  r.grad = grad_d;
  bool aligned = x->total % 4 == 0 && reinterpret_cast<uintptr_t>(x->slabs) % 16 == 0 &&
                 reinterpret_cast<uintptr_t>(grad_d) % 16 == 0;
  for (size_t i = 0; i < x->offsets.size(); ++i) aligned = aligned && x->offsets[i] % 4 == 0;
  if (aligned) {
    const TimRec rec{KC_REDUCE, "reduce_slabs_kernel", 0.0, 4.0 * (x->splits + 1.0) * x->total};
    const dim3 grid(ceil_div(x->total, 4 * 256));
    if (x->splits == 8)
      launch_k(rec, lstm_reduce_fast_kernel<8>, grid, dim3(256), 0, st, grad_d, x->slabs, x->total);
    else if (x->splits == 16)
      launch_k(rec, lstm_reduce_fast_kernel<16>, grid, dim3(256), 0, st, grad_d, x->slabs, x->total);
    else
      launch_k(rec, lstm_reduce_fast_kernel<32>, grid, dim3(256), 0, st, grad_d, x->slabs, x->total);
  } else
    launch_k(TimRec{KC_REDUCE, "reduce_slabs_kernel", 0.0, 0.0}, lstm_reduce_kernel,
             dim3(ceil_div(x->total, kRedParams)), dim3(kRedThreads), 0, st, r);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_lstm_timing(ppo_lstm_ctx *x, int enable, int capacity) {
  PPO_REQUIRE(x != nullptr, "ppo_lstm_timing: null ctx");
  return timing_enable(x->tim, enable, capacity);
}

extern "C" int ppo_lstm_timing_kernel(ppo_lstm_ctx *x, int index, const char **name, int *kclass,
                                      double *total_ms, int64_t *launches, double *flops,
                                      double *bytes) {
  PPO_REQUIRE(x != nullptr, "ppo_lstm_timing_kernel: null ctx");
  return timing_read_kernel(x->tim, index, name, kclass, total_ms, launches, flops, bytes);
}

extern "C" int ppo_lstm_fused_step(ppo_lstm_ctx *x, int enable) {
  PPO_REQUIRE(x != nullptr, "ppo_lstm_fused_step: null ctx");
  if (enable < 0) return x->fused_step;
  x->fused_step = enable != 0;
  return 0;
}
