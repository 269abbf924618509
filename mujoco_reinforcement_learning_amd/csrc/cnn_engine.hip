// Pixel-observation actor-critic (BASELINE.json configs[4]: dm_control cheetah-run, 84x84x3
// frames, 1024 envs) on gfx950, behind the ppo_cnn_* C-ABI (include/ppo_engine.h).
//
// The reference has no pixel / CNN path (running_dm_control.py:56-91 is a state-observation
// humanoid), so the model is this engine's declaration: per net the Nature-DQN
// encoder (csrc/conv.h: three implicit-GEMM convolutions on MFMA, ReLU, torch CHW flatten ->
// 3136 features) followed by the reference's NetworkBlock heads (network_block_creator.py:24-86):
//   actor : mean = omv * tanh(MLP_mu(features)), std = exp(actor_logstd)  (models/linear/actor.py)
//   critic: value = MLP_v(features)                                        (models/critic.py)
// and the PPO minibatch of ppo.py:108-135 (Normal log-prob, clipped surrogate, entropy, Huber).
//
// Minibatch (both nets per launch, blockIdx.z = net):
//   conv FWD x3 (pixels gathered through the minibatch rows) -> a1, a2 (HWC), features (CHW f32)
//   MLP forward (gemm.h; actor and critic share launches when their layer shapes agree)
//   cnn_update_head_kernel: log-prob, ratio, clipped surrogate, Huber -> dz (actor head, critic
//     output), per-split log-std and loss partials
//   MLP backward (split-K slabs; the input gradient of layer 0 times relu'(features) is the
//     encoder's output gradient, CHW)
//   conv L3 WGRAD + DGRAD, L2 WGRAD + DGRAD, L1 WGRAD (per-split slabs)
//   reduce_slabs_kernel: every slab -> the flat gradient in a fixed order (deterministic)
#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "common.h"
#include "conv.h"
#include "conv_pixel.h"
#include "conv_lds.h"
#include "gemm.h"
#include "gemm_ops.h"
#include "reduce_slabs.h"
#include "timing.h"

namespace ppo {
namespace cnn {

using namespace conv;

constexpr int kMaxA = 32;
constexpr int kMlpSplits = 32;        // split-K slabs of the MLP weight gradients (max)
constexpr int kConvMaxSplits = 256;   // split-K slabs of a conv weight gradient (max)
constexpr int kHeadSplits = 256;      // row blocks of the update head (log-std / loss partials)
constexpr int64_t kAlign = 16;        // floats: every flat tensor starts 64-B aligned
constexpr int64_t kWsAlign = 64;

static inline int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

struct MlpLayer {
  int in, out, act;
  int64_t w, b;  // b < 0: no bias
};
struct Mlp {
  int n;  // layers incl. the output layer
  MlpLayer l[PPO_MAX_LAYERS + 1];
};
struct ConvParams {
  int64_t w, b;  // torch-order weight [co][ci][k][k] and bias offsets
};

// ---- heads ------------------------------------------------------------------------------------
struct HeadArgs {
  const float *ya;       // actor head output tanh(z) [B][A]
  const float *vc;       // critic output [B]
  const float *logstd;   // [A]
  float omv;
  int b, a;
  // policy step
  const float *eps;
  uint64_t seed, offset;
  const uint64_t *offset_base;
  float *action, *logp_out, *value_out, *mean_out;
  // update
  const int32_t *rows;
  const float *actions, *old_logp, *adv, *vt;
  float *dza, *dzc;      // d(actor head pre-activation) [B][A], d(critic output) [B]
  float *ls_part;        // [splits][A]
  float *loss_part;      // [splits][2]
  int splits;
  float clip_lo, clip_hi, ent_coef, inv_b, inv_ba;
};

// ppo.py:22-26 per env row (torch formulas of policy_head_kernel): mean = omv * tanh(z);
// action = eps * std + mean; logp = sum_a (-(x - mu)^2) / (2 var) - log(std) - log(sqrt(2 pi)).
__global__ __launch_bounds__(256) void cnn_policy_head_kernel(HeadArgs q) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= q.b) return;
  const int A = q.a;
  const uint64_t off = q.offset + (q.offset_base ? *q.offset_base : 0);
  float lp = 0.f;
  for (int k = 0; k < A; ++k) {
    const int64_t idx = static_cast<int64_t>(n) * A + k;
    const float mu = q.omv * q.ya[idx];
    if (q.mean_out) q.mean_out[idx] = mu;
    if (!q.action) continue;
    const float sd = expf(q.logstd[k]);
    const float e = q.eps ? q.eps[idx] : philox_normal_at(q.seed, off + idx);
    const float x = e * sd + mu;  // torch.normal: randn * std, then + mean (two roundings)
    q.action[idx] = x;
    const float d = x - mu;
    lp += ((-(d * d)) / (2.f * (sd * sd)) - logf(sd)) - kLogSqrt2Pi;
  }
  if (q.logp_out) q.logp_out[n] = lp;
  if (q.value_out) q.value_out[n] = q.vc[n];
}

// ppo.py:108-135 per minibatch row; block s owns rows [s*B/S, (s+1)*B/S) and writes its fixed-
// order partial sums of d(loss)/d(actor_logstd) and of the two loss terms.
__global__ __launch_bounds__(256) void cnn_update_head_kernel(HeadArgs q) {
  __shared__ float s_sd[kMaxA], s_lsd[kMaxA], s_var[kMaxA];
  __shared__ float red[256][kMaxA + 2];
  const int tid = threadIdx.x, A = q.a;
  if (tid < A) {
    const float sd = expf(q.logstd[tid]);
    s_sd[tid] = sd;
    s_lsd[tid] = logf(sd);
    s_var[tid] = sd * sd;
  }
  __syncthreads();
  const int j0 = static_cast<int>((static_cast<int64_t>(blockIdx.x) * q.b) / q.splits);
  const int j1 = static_cast<int>((static_cast<int64_t>(blockIdx.x + 1) * q.b) / q.splits);
  float ls[kMaxA];
#pragma unroll
  for (int k = 0; k < kMaxA; ++k) ls[k] = 0.f;
  float la = 0.f, lc = 0.f;
  for (int j = j0 + tid; j < j1; j += 256) {
    const int64_t sr = q.rows[j];
    float lp = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxA; ++k) {
      if (k >= A) break;
      const float mu = q.omv * q.ya[static_cast<int64_t>(j) * A + k];
      const float d = q.actions[sr * A + k] - mu;
      lp += ((-(d * d)) / (2.f * s_var[k]) - s_lsd[k]) - kLogSqrt2Pi;
    }
    const float adv = q.adv[sr];
    const float ratio = expf(lp - q.old_logp[sr]);
    const float s1 = ratio * adv;
    const float cl = ratio < q.clip_lo ? q.clip_lo : (ratio > q.clip_hi ? q.clip_hi : ratio);
    const float s2 = cl * adv;
    const float mn = (s1 != s1 || s2 != s2) ? (s1 + s2) : (s2 < s1 ? s2 : s1);
    const float gg = -q.inv_b;
    const float g1 = (s1 < s2) ? gg : (s1 == s2 ? gg * 0.5f : 0.f);
    const float g2 = (s2 < s1) ? gg : (s1 == s2 ? gg * 0.5f : 0.f);
    const bool inside = (ratio >= q.clip_lo) && (ratio <= q.clip_hi);
    const float dlogp = (g1 * adv + (inside ? g2 * adv : 0.f)) * ratio;
#pragma unroll
    for (int k = 0; k < kMaxA; ++k) {
      if (k >= A) break;
      const int64_t idx = static_cast<int64_t>(j) * A + k;
      const float y = q.ya[idx];
      const float d = q.actions[sr * A + k] - q.omv * y;
      const float dmu = dlogp * (d / s_var[k]);
      q.dza[idx] = (dmu * q.omv) * (1.f - y * y);
      ls[k] += dlogp * ((d * d) / s_var[k] - 1.f) - q.ent_coef * q.inv_ba;
    }
    la += mn;
    const float v = q.vc[j];
    const float diff = v - q.vt[sr];
    const float ad = fabsf(diff);
    lc += (ad < 1.f) ? 0.5f * ad * ad : (ad - 0.5f);
    q.dzc[j] = q.inv_b * (diff < -1.f ? -1.f : (diff > 1.f ? 1.f : diff));
  }
#pragma unroll
  for (int k = 0; k < kMaxA; ++k)
    if (k < A) red[tid][k] = ls[k];
  red[tid][A] = la;
  red[tid][A + 1] = lc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w)
      for (int k = 0; k < A + 2; ++k) red[tid][k] += red[tid + w][k];
    __syncthreads();
  }
  if (tid < A) q.ls_part[static_cast<int64_t>(blockIdx.x) * A + tid] = red[0][tid];
  if (tid == 0) {
    q.loss_part[2 * blockIdx.x] = red[0][A];
    q.loss_part[2 * blockIdx.x + 1] = red[0][A + 1];
  }
}

__global__ __launch_bounds__(kRedThreads) void cnn_reduce_kernel(ReduceArgs q) {
  (void)reduce_slab_block(q, blockIdx.x);
}

// ---- synthetic pixel VecEnv (bench / test harness) ----------------------------------------------
__device__ __forceinline__ uint32_t mix32(uint32_t seed, uint32_t t, uint32_t n, uint32_t i) {
  uint32_t h = (i * 0x9E3779B1u) ^ (t * 0x85EBCA77u + n * 0xC2B2AE3Du + seed * 0x27D4EB2Fu);
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

struct PixelArgs {
  uint32_t seed;
  int t, n, h, w, c, a;
  const float *action;
  uint8_t *out;
  const float *base_reward;
  const uint8_t *base_term;
  double *reward_out;
  uint8_t *term_out;
};

// thread = 4 consecutive bytes of one frame (H*W*C % 4 == 0); threads of unit 0 also write the
// env's reward / termination
__global__ __launch_bounds__(256) void pixel_env_step_kernel(PixelArgs p) {
  const int frame = p.h * p.w * p.c;
  const int units = frame / 4;
  const int64_t g = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (g >= static_cast<int64_t>(p.n) * units) return;
  const int n = static_cast<int>(g / units), u = static_cast<int>(g % units);
  int qa[kMaxA];
#pragma unroll
  for (int j = 0; j < kMaxA; ++j) {
    qa[j] = 0;
    if (j < p.a && p.action) {
      const float f = floorf(p.action[static_cast<int64_t>(n) * p.a + j] * 8.f);
      qa[j] = static_cast<int>(f < -64.f ? -64.f : (f > 63.f ? 63.f : f));
    }
  }
  uint32_t word = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int i = 4 * u + e;
    const int ch = i % p.c, pix = i / p.c, x = pix % p.w, y = pix / p.w;
    const uint32_t hsh = mix32(p.seed, static_cast<uint32_t>(p.t), static_cast<uint32_t>(n),
                               static_cast<uint32_t>(i));
    int j = (2 * ch + ((x + y) & 1)) % p.a;
    int qv = 0;
#pragma unroll
    for (int k = 0; k < kMaxA; ++k)
      if (k == j) qv = qa[k];
    word |= ((hsh + static_cast<uint32_t>(qv)) & 255u) << (8 * e);
  }
  reinterpret_cast<uint32_t *>(p.out + static_cast<int64_t>(n) * frame)[u] = word;
  if (u == 0 && p.reward_out && p.action && p.t >= 1) {
    double ctrl = 0.0;
    for (int j = 0; j < p.a; ++j) {
      const double av = p.action[static_cast<int64_t>(n) * p.a + j];
      ctrl = ctrl + av * av;
    }
    const int64_t r = static_cast<int64_t>(p.t - 1) * p.n + n;
    p.reward_out[n] = static_cast<double>(p.base_reward[r]) - 0.01 * ctrl;
    p.term_out[n] = p.base_term[r];
  }
}

}  // namespace cnn
}  // namespace ppo

using namespace ppo;
using namespace ppo::cnn;

struct ppo_cnn_ctx {
  ppo_cnn_cfg cfg;
  int device;
  int prec;
  float ent_log_share;  // ppo_*_loss_entropy_share (logged actor loss only)
  ConvParams conv[2][3];   // per net, per encoder layer
  int64_t logstd_off;
  Mlp mlp[2];              // actor mean MLP, critic MLP (input: 3136 features)
  int64_t total, n_actor;
  std::vector<int64_t> offsets;  // torch parameters() order, actor then critic
  float *params;
  const uint64_t *rng_counter;
  float *ws;
  int64_t rows;
  // workspace views (per net z)
  float *wpack[2][3];                 // packed conv weights [co][(ky kx) ci]
  __bf16 *wdg[2][2];                  // bf16 W'^T of L2 / L3 for dgrad_lds_kernel (conv_lds.h)
  __bf16 *wfw[2][2];                  // bf16 W' of L2 / L3 for fwd_lds_kernel
  void *a1[2], *a2[2];                // encoder activations (bf16 or f32, HWC)
  float *feat[2];                     // [rows][3136] CHW
  float *act[2][PPO_MAX_LAYERS + 1];  // MLP layer outputs [rows][out]
  float *dz[2][2];                    // MLP ping-pong gradients [rows][maxw]
  float *dfeat[2];                    // [rows][3136] gradient at the L3 pre-activation (CHW)
  float *dz2[2], *dz1[2];             // gradients at the L2 / L1 pre-activations (HWC)
  float *mlp_slabs;                   // [kMlpSplits][total]
  float *cslab[2][3];                 // conv slabs [kConvMaxSplits][cout*kdim + cout (aligned)]
  int64_t cslab_stride[3];
  int cslab_splits_last[3];           // split counts of the last encoder backward
  float *ls_part, *loss_part;         // [kHeadSplits][A], [kHeadSplits][2]
  int maxw;
  Timing tim;
};

namespace {

struct TimingScope {
  explicit TimingScope(ppo_cnn_ctx *x) { g_tim = x->tim.on ? &x->tim : nullptr; }
  ~TimingScope() { g_tim = nullptr; }
};

void add_mlp(Mlp &m, int in, const ppo_cnn_cfg &c, int out, int final_act, bool bias, int64_t &off,
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
    if (bias) {
      L.b = off;
      offs.push_back(off);
      off = align_up(off + L.out, kAlign);
    } else {
      L.b = -1;
    }
    in = L.out;
  }
}

template <class G>
void add_conv(ConvParams &cp, int64_t &off, std::vector<int64_t> &offs) {
  cp.w = off;
  offs.push_back(off);
  off = align_up(off + static_cast<int64_t>(G::cout) * G::kdim, kAlign);
  cp.b = off;
  offs.push_back(off);
  off = align_up(off + G::cout, kAlign);
}

template <class G>
int64_t slab_floats() { return align_up(static_cast<int64_t>(G::cout) * G::kdim + G::cout, 4); }

int check_rows(const ppo_cnn_ctx *x, int b) {
  PPO_REQUIRE(x != nullptr, "ppo_cnn: null ctx");
  PPO_REQUIRE(b >= 0 && b <= x->rows, "ppo_cnn: %d rows exceed the workspace (%lld)", b,
              static_cast<long long>(x->rows));
  PPO_REQUIRE(x->params != nullptr, "ppo_cnn: parameters not bound (ppo_cnn_bind_params)");
  return 0;
}

// ---- encoder launches ---------------------------------------------------------------------------
template <class G, int MODE>
TimRec conv_rec(const char *name, int nimg, int nets) {
  // algorithmic FLOPs: every (output position, tap, cin, cout) product once -- the same
  // 2 * P * COUT * KS^2 * CIN per image for FWD, DGRAD (border taps excluded) and WGRAD
  const double p = static_cast<double>(nimg) * nets;
  const double fl = 2.0 * p * G::P * G::cout * G::kdim;
  // bytes: the layer input and the product's other tensor once (f32 upper bound)
  const double by =
      p * 4.0 * (static_cast<double>(G::PIN) * G::cin + static_cast<double>(G::P) * G::cout);
  return TimRec{KC_CONV, tim_active() ? name : nullptr, fl, by};
}

// The LDS-staged bf16 kernels (conv_pixel.h, conv_lds.h): their algorithmic bytes per image, both
// nets -- every tensor once at its stored width (u8 frames read once for both nets, bf16
// activations, f32 gradients); the frame / input of a product read once.
template <class G, int MODE>
TimRec lds_rec(const char *name, int nimg) {
  TimRec r = conv_rec<G, MODE>(name, nimg, 2);
  const double in = static_cast<double>(G::PIN) * G::cin, out = static_cast<double>(G::P) * G::cout;
  const bool pixel = G::cin == 3;
  double per;
  if (MODE == MODE_FWD)
    per = pixel ? in + 2 * 2 * out : 2 * (2 * in + (G::P == L3::P ? 4 : 2) * out);
  else if (MODE == MODE_WGRAD)
    per = pixel ? in + 2 * 4 * out : 2 * (2 * in + 4 * out);
  else
    per = 2 * (4 * out + 2 * in + 4 * in);  // dz, relu' operand, the input gradient
  r.bytes = static_cast<double>(nimg) * per;
  return r;
}

template <class G, int MODE, typename TIN, typename TOUT, bool BF, bool DZCHW, bool OUTCHW, int WM,
          int WN, int TM, int TN>
int launch_conv(const ConvArgs &a, int nets, hipStream_t st) {
  constexpr int BM = 32 * TM * WM, BN = 32 * TN * WN, BK = 32;
  constexpr int NCLS = MODE == MODE_DGRAD ? G::s * G::s : 1;
  const int M = MODE == MODE_FWD ? a.nimg * G::P
              : MODE == MODE_DGRAD ? a.nimg * G::hq * G::wq : G::cout;
  const int N = MODE == MODE_FWD ? G::cout : MODE == MODE_DGRAD ? G::cin : G::kdim;
  if (M == 0) return 0;
  if constexpr (MODE == MODE_WGRAD) {
    const int64_t per_split = ceil_div(static_cast<int64_t>(a.nimg) * G::P, a.splits);
    PPO_REQUIRE(per_split / G::P + 2 <= kWgradMaxFrames,
                "conv wgrad: %lld positions per split span more than %d frames",
                static_cast<long long>(per_split), kWgradMaxFrames);
  }
  const int tiles = ceil_div(M, BM) * ceil_div(N, BN);
  // DGRAD: (tile, class) in x; WGRAD: (split, tile) in x
  dim3 grid(tiles * NCLS * (MODE == MODE_WGRAD ? a.splits : 1), 1, nets);
  const char *name = nullptr;
  if (tim_active())
    name = intern_name("conv_kernel<%dx%dx%d k%d s%d, %s, %s, %d>", G::hin, G::win, G::cin, G::k,
                       G::s, MODE == MODE_FWD ? "fwd" : MODE == MODE_DGRAD ? "dgrad" : "wgrad",
                       BF ? "bf16" : "f32", G::cout);
  launch_k(conv_rec<G, MODE>(name, a.nimg, nets),
           conv_kernel<G, MODE, TIN, TOUT, BF, DZCHW, OUTCHW, WM, WN, TM, TN, BK>, grid,
           dim3(64 * WM * WN), 0, st, a);
  PPO_LAUNCHED();
  return 0;
}

// Tile shapes: FWD / DGRAD 256 rows x N (N = 32: 4 waves of 64x32; N = 64: 4 waves of 64x64);
// WGRAD COUT x 128 columns (COUT = 32: 4 waves of 32x32; 64: 4 waves of 32x64).
template <class G, int MODE, typename TIN, typename TOUT, bool BF, bool DZCHW, bool OUTCHW>
int run_conv(const ConvArgs &a, int nets, hipStream_t st) {
  if constexpr (MODE == MODE_WGRAD) {
    if constexpr (G::cout == 32)
      return launch_conv<G, MODE, TIN, TOUT, BF, DZCHW, OUTCHW, 1, 4, 1, 1>(a, nets, st);
    else
      return launch_conv<G, MODE, TIN, TOUT, BF, DZCHW, OUTCHW, 2, 2, 1, 2>(a, nets, st);
  } else {
    constexpr int N = MODE == MODE_FWD ? G::cout : G::cin;
    if constexpr (N == 32)
      return launch_conv<G, MODE, TIN, TOUT, BF, DZCHW, OUTCHW, 4, 1, 2, 1>(a, nets, st);
    else
      return launch_conv<G, MODE, TIN, TOUT, BF, DZCHW, OUTCHW, 4, 1, 2, 2>(a, nets, st);
  }
}

// The bf16 pixel layer through the space-to-depth kernels (conv_pixel.h); PPO_PIXEL_S2D=0 keeps
// it on the implicit-GEMM conv_kernel (the A/B baseline).
static const int g_pix_s2d = [] {
  const char *v = getenv("PPO_PIXEL_S2D");
  return v ? atoi(v) : 1;
}();

PixArgs pix_args(ppo_cnn_ctx *x, const uint8_t *frames, const int32_t *rows, int b) {
  PixArgs p{};
  p.frames = frames;
  p.rows = rows;
  p.nimg = b;
  for (int z = 0; z < 2; ++z) {
    p.w[z] = x->params + x->conv[z][0].w;
    p.bias[z] = x->params + x->conv[z][0].b;
  }
  return p;
}

int pixel_forward(ppo_cnn_ctx *x, const uint8_t *frames, const int32_t *rows, int b, hipStream_t st) {
  if (b == 0) return 0;
  PixArgs p = pix_args(x, frames, rows, b);
  for (int z = 0; z < 2; ++z) p.out[z] = static_cast<__bf16 *>(x->a1[z]);
  launch_k(lds_rec<L1, MODE_FWD>("pixel_fwd_kernel", b), pixel_fwd_kernel,
           dim3(std::min(b, 512)), dim3(kPixFwdThreads), 0, st, p);
  PPO_LAUNCHED();
  return 0;
}

int pixel_wgrad(ppo_cnn_ctx *x, const uint8_t *frames, const int32_t *rows, int b, int splits,
                hipStream_t st) {
  PixArgs p = pix_args(x, frames, rows, b);
  for (int z = 0; z < 2; ++z) {
    p.dz[z] = x->dz1[z];
    p.slab[z] = x->cslab[z][0];
  }
  p.slab_stride = x->cslab_stride[0];
  p.splits = splits;
  launch_k(lds_rec<L1, MODE_WGRAD>("pixel_wgrad_kernel", b), pixel_wgrad_kernel,
           dim3(splits), dim3(kPixWgThreads), 0, st, p);
  PPO_LAUNCHED();
  return 0;
}

// The bf16 input gradients of L2 / L3 through dgrad_lds_kernel (conv_lds.h); PPO_CONV_LDS=0
// keeps them on the implicit-GEMM conv_kernel.
static const int g_conv_lds = [] {
  const char *v = getenv("PPO_CONV_LDS");
  return v ? atoi(v) : 1;
}();

template <class D>
int dgrad_lds(ppo_cnn_ctx *x, int l, const float *const dz[2], const void *const xin[2],
              float *const dout[2], int b, hipStream_t st) {
  // W'^T of both nets: packed by lds_pack (the weights of this minibatch's forward)
  if (b == 0) return 0;
  DgArgs q{};
  for (int z = 0; z < 2; ++z) {
    q.wt[z] = x->wdg[z][l - 1];
    q.dz[z] = dz[z];
    q.xin[z] = static_cast<const __bf16 *>(xin[z]);
    q.dout[z] = dout[z];
  }
  q.nimg = b;
  using G = std::conditional_t<D::S == 2, L2, L3>;
  launch_k(lds_rec<G, MODE_DGRAD>(D::S == 2 ? "dgrad_lds_kernel<L2>" : "dgrad_lds_kernel<L3>", b),
           dgrad_lds_kernel<D>, dim3(std::min(b, 256)), dim3(512), 0, st, q);
  PPO_LAUNCHED();
  return 0;
}

template <class D>
int pack_fw(ppo_cnn_ctx *x, int l, hipStream_t st) {
  launch_k(TimRec{KC_CONV, "fw_pack_kernel", 0.0, 0.0}, fw_pack_kernel<D>,
           dim3(ceil_div(2LL * D::CO * D::KD, 256)), dim3(256), 0, st,
           x->params + x->conv[0][l].w, x->params + x->conv[1][l].w, x->wfw[0][l - 1],
           x->wfw[1][l - 1]);
  PPO_LAUNCHED();
  return 0;
}

template <class D>
int pack_dg(ppo_cnn_ctx *x, int l, hipStream_t st) {
  launch_k(TimRec{KC_CONV, "dg_pack_kernel", 0.0, 0.0}, dg_pack_kernel<D>,
           dim3(ceil_div(2LL * D::N * D::KD, 256)), dim3(256), 0, st,
           x->params + x->conv[0][l].w, x->params + x->conv[1][l].w, x->wdg[0][l - 1],
           x->wdg[1][l - 1]);
  PPO_LAUNCHED();
  return 0;
}

template <class D>
int fwd_lds(ppo_cnn_ctx *x, int l, const void *const xin[2], void *const out[2], int b,
            hipStream_t st) {
  if (b == 0) return 0;
  FwArgs q{};
  for (int z = 0; z < 2; ++z) {
    q.wp[z] = x->wfw[z][l - 1];
    q.bias[z] = x->params + x->conv[z][l].b;
    q.xin[z] = static_cast<const __bf16 *>(xin[z]);
    q.out[z] = out[z];
  }
  q.nimg = b;
  using G = std::conditional_t<D::S == 2, L2, L3>;
  launch_k(lds_rec<G, MODE_FWD>(D::S == 2 ? "fwd_lds_kernel<L2>" : "fwd_lds_kernel<L3>", b),
           fwd_lds_kernel<D>, dim3(std::min(b, 256)), dim3(512), 0, st, q);
  PPO_LAUNCHED();
  return 0;
}

template <class D>
int wgrad_lds(ppo_cnn_ctx *x, int l, const void *const xin[2], const float *const dz[2], int b,
              int splits, hipStream_t st) {
  FwArgs q{};
  for (int z = 0; z < 2; ++z) {
    q.xin[z] = static_cast<const __bf16 *>(xin[z]);
    q.dz[z] = dz[z];
    q.slab[z] = x->cslab[z][l];
  }
  q.slab_stride = x->cslab_stride[l];
  q.splits = splits;
  q.nimg = b;
  using G = std::conditional_t<D::S == 2, L2, L3>;
  launch_k(lds_rec<G, MODE_WGRAD>(D::S == 2 ? "wgrad_lds_kernel<L2>" : "wgrad_lds_kernel<L3>", b),
           wgrad_lds_kernel<D>, dim3(splits), dim3(512), 0, st, q);
  PPO_LAUNCHED();
  return 0;
}

int pack_conv(ppo_cnn_ctx *x, hipStream_t st) {
  if (x->prec == PPO_PREC_BF16 && g_conv_lds) {
    if (int rc = pack_fw<L2F>(x, 1, st)) return rc;
    if (int rc = pack_fw<L3F>(x, 2, st)) return rc;
    if (int rc = pack_dg<L2D>(x, 1, st)) return rc;
    if (int rc = pack_dg<L3D>(x, 2, st)) return rc;
    if (g_pix_s2d) return 0;  // no conv_kernel reads the f32 pack
  }
  PackArgs p{};
  const int co[3] = {L1::cout, L2::cout, L3::cout}, ci[3] = {L1::cin, L2::cin, L3::cin},
            ks[3] = {L1::k, L2::k, L3::k};
  int64_t most = 0;
  for (int l = 0; l < 3; ++l)
    for (int z = 0; z < 2; ++z) {
      const int i = 2 * l + z;
      p.src[i] = x->params + x->conv[z][l].w;
      p.dst[i] = x->wpack[z][l];
      p.cout[i] = co[l];
      p.cin[i] = ci[l];
      p.k[i] = ks[l];
      most = std::max<int64_t>(most, static_cast<int64_t>(co[l]) * ci[l] * ks[l] * ks[l]);
    }
  launch_k(TimRec{KC_CONV, "conv_pack_kernel", 0.0, 0.0}, conv_pack_kernel,
           dim3(ceil_div(most, 256), 6), dim3(256), 0, st, p);
  PPO_LAUNCHED();
  return 0;
}

template <typename TACT, bool BF>
int encoder_forward_t(ppo_cnn_ctx *x, const uint8_t *frames, const int32_t *rows, int b,
                      hipStream_t st) {
  ConvArgs a{};
  a.nimg = b;
  for (int z = 0; z < 2; ++z) {
    a.net[z].in = frames;
    a.net[z].w = x->wpack[z][0];
    a.net[z].bias = x->params + x->conv[z][0].b;
    a.net[z].out = x->a1[z];
  }
  a.rows = rows;
  if (BF && g_pix_s2d) {
    if (int rc = pixel_forward(x, frames, rows, b, st)) return rc;
  } else if (int rc = run_conv<L1, MODE_FWD, uint8_t, TACT, BF, false, false>(a, 2, st)) {
    return rc;
  }
  a.rows = nullptr;
  for (int z = 0; z < 2; ++z) {
    a.net[z].in = x->a1[z];
    a.net[z].w = x->wpack[z][1];
    a.net[z].bias = x->params + x->conv[z][1].b;
    a.net[z].out = x->a2[z];
  }
  if (BF && g_conv_lds) {
    const void *xin[2] = {x->a1[0], x->a1[1]};
    void *const out[2] = {x->a2[0], x->a2[1]};
    if (int rc = fwd_lds<L2F>(x, 1, xin, out, b, st)) return rc;
  } else if (int rc = run_conv<L2, MODE_FWD, TACT, TACT, BF, false, false>(a, 2, st)) {
    return rc;
  }
  for (int z = 0; z < 2; ++z) {
    a.net[z].in = x->a2[z];
    a.net[z].w = x->wpack[z][2];
    a.net[z].bias = x->params + x->conv[z][2].b;
    a.net[z].out = x->feat[z];
  }
  if (BF && g_conv_lds) {
    const void *xin[2] = {x->a2[0], x->a2[1]};
    void *const out[2] = {x->feat[0], x->feat[1]};
    return fwd_lds<L3F>(x, 2, xin, out, b, st);
  }
  return run_conv<L3, MODE_FWD, TACT, float, BF, false, true>(a, 2, st);
}

template <typename TACT, bool BF>
int encoder_backward_t(ppo_cnn_ctx *x, const uint8_t *frames, const int32_t *rows, int b,
                       hipStream_t st) {
  auto splits_for = [](int64_t k) {
    return static_cast<int>(std::min<int64_t>(kConvMaxSplits, std::max<int64_t>(1, k / 8192)));
  };
  ConvArgs a{};
  a.nimg = b;
  // L3: dz = dfeat (CHW)
  for (int z = 0; z < 2; ++z) {
    a.net[z] = ConvNet{};
    a.net[z].in = x->a2[z];
    a.net[z].w = x->wpack[z][2];
    a.net[z].dz = x->dfeat[z];
    a.net[z].dout = x->dz2[z];
    a.net[z].slab = x->cslab[z][2];
    a.net[z].has_bias = 1;
  }
  a.splits = splits_for(static_cast<int64_t>(b) * L3::P);
  a.slab_stride = x->cslab_stride[2];
  if (BF && g_conv_lds) {
    a.splits = std::max(1, std::min(kConvMaxSplits, b));
    const void *xin[2] = {x->a2[0], x->a2[1]};
    const float *dz[2] = {x->dfeat[0], x->dfeat[1]};
    if (int rc = wgrad_lds<L3F>(x, 2, xin, dz, b, a.splits, st)) return rc;
  } else if (int rc = run_conv<L3, MODE_WGRAD, TACT, TACT, BF, true, false>(a, 2, st)) {
    return rc;
  }
  if (BF && g_conv_lds) {
    const float *dz[2] = {x->dfeat[0], x->dfeat[1]};
    const void *xin[2] = {x->a2[0], x->a2[1]};
    float *const dout[2] = {x->dz2[0], x->dz2[1]};
    if (int rc = dgrad_lds<L3D>(x, 2, dz, xin, dout, b, st)) return rc;
  } else if (int rc = run_conv<L3, MODE_DGRAD, TACT, TACT, BF, true, false>(a, 2, st)) {
    return rc;
  }
  const int s3 = a.splits;
  // L2: dz = dz2 (HWC)
  for (int z = 0; z < 2; ++z) {
    a.net[z].in = x->a1[z];
    a.net[z].w = x->wpack[z][1];
    a.net[z].dz = x->dz2[z];
    a.net[z].dout = x->dz1[z];
    a.net[z].slab = x->cslab[z][1];
  }
  a.splits = splits_for(static_cast<int64_t>(b) * L2::P);
  a.slab_stride = x->cslab_stride[1];
  if (BF && g_conv_lds) {
    a.splits = std::max(1, std::min(kConvMaxSplits, b));
    const void *xin[2] = {x->a1[0], x->a1[1]};
    const float *dz[2] = {x->dz2[0], x->dz2[1]};
    if (int rc = wgrad_lds<L2F>(x, 1, xin, dz, b, a.splits, st)) return rc;
  } else if (int rc = run_conv<L2, MODE_WGRAD, TACT, TACT, BF, false, false>(a, 2, st)) {
    return rc;
  }
  if (BF && g_conv_lds) {
    const float *dz[2] = {x->dz2[0], x->dz2[1]};
    const void *xin[2] = {x->a1[0], x->a1[1]};
    float *const dout[2] = {x->dz1[0], x->dz1[1]};
    if (int rc = dgrad_lds<L2D>(x, 1, dz, xin, dout, b, st)) return rc;
  } else if (int rc = run_conv<L2, MODE_DGRAD, TACT, TACT, BF, false, false>(a, 2, st)) {
    return rc;
  }
  const int s2 = a.splits;
  // L1: pixels through the minibatch rows, dz = dz1
  for (int z = 0; z < 2; ++z) {
    a.net[z].in = frames;
    a.net[z].w = x->wpack[z][0];
    a.net[z].dz = x->dz1[z];
    a.net[z].dout = nullptr;
    a.net[z].slab = x->cslab[z][0];
  }
  a.rows = rows;
  a.splits = splits_for(static_cast<int64_t>(b) * L1::P);
  a.slab_stride = x->cslab_stride[0];
  if (BF && g_pix_s2d) {
    if (int rc = pixel_wgrad(x, frames, rows, b, a.splits, st)) return rc;
  } else if (int rc = run_conv<L1, MODE_WGRAD, uint8_t, TACT, BF, false, false>(a, 2, st)) {
    return rc;
  }
  // remember the split counts for the reduction
  x->cslab_splits_last[0] = a.splits;
  x->cslab_splits_last[1] = s2;
  x->cslab_splits_last[2] = s3;
  return 0;
}

int encoder_forward(ppo_cnn_ctx *x, const uint8_t *frames, const int32_t *rows, int b,
                    hipStream_t st) {
  if (int rc = pack_conv(x, st)) return rc;
  return x->prec == PPO_PREC_BF16 ? encoder_forward_t<__bf16, true>(x, frames, rows, b, st)
                                  : encoder_forward_t<float, false>(x, frames, rows, b, st);
}

int encoder_backward(ppo_cnn_ctx *x, const uint8_t *frames, const int32_t *rows, int b,
                     hipStream_t st) {
  return x->prec == PPO_PREC_BF16 ? encoder_backward_t<__bf16, true>(x, frames, rows, b, st)
                                  : encoder_backward_t<float, false>(x, frames, rows, b, st);
}

// ---- MLP heads (gemm.h) ---------------------------------------------------------------------------
// Forward of both MLPs (net z reads x->feat[z]); layers of equal shape share a launch.
int mlp_forward(ppo_cnn_ctx *x, int b, hipStream_t st) {
  const float *P = x->params;
  for (int l = 0; l < x->mlp[0].n; ++l) {
    GemmProblem p[2] = {};
    for (int z = 0; z < 2; ++z) {
      const MlpLayer &L = x->mlp[z].l[l];
      p[z].a = l == 0 ? x->feat[z] : x->act[z][l - 1];
      p[z].lda = L.in;
      p[z].b = P + L.w;
      p[z].ldb = L.in;
      p[z].c = x->act[z][l];
      p[z].ldc = L.out;
      p[z].bias = L.b >= 0 ? P + L.b : nullptr;
      p[z].m = b;
      p[z].n = L.out;
    }
    const MlpLayer &LA = x->mlp[0].l[l], &LC = x->mlp[1].l[l];
    const bool same = LA.in == LC.in && LA.out == LC.out && LA.act == LC.act;
    for (int z = 0; z < (same ? 1 : 2); ++z) {
      GemmBatch gb{};
      gb.p[0] = p[z];
      if (same) gb.p[1] = p[1];
      gb.k = x->mlp[z].l[l].in;
      gb.act = x->mlp[z].l[l].act;
      gb.prec = x->prec;
      if (int rc = gemm_rows_fwd_nk(gb, same ? 2 : 1, b, x->mlp[z].l[l].out, st))
        return rc;
    }
  }
  return 0;
}

// Backward of both MLPs from x->dz[z][0] (gradient at the output layer's pre-activation): weight
// gradients into the MLP slabs, the input gradient times relu'(features) into x->dfeat[z].
int mlp_backward(ppo_cnn_ctx *x, int b, int splits, hipStream_t st) {
  const float *P = x->params;
  float *cur[2] = {x->dz[0][0], x->dz[1][0]};
  for (int l = x->mlp[0].n - 1; l >= 0; --l) {
    GemmProblem pw[2] = {}, px[2] = {};
    float *nxt[2] = {nullptr, nullptr};
    for (int z = 0; z < 2; ++z) {
      const MlpLayer &L = x->mlp[z].l[l];
      pw[z].a = cur[z];
      pw[z].lda = L.out;
      pw[z].b = l == 0 ? x->feat[z] : x->act[z][l - 1];
      pw[z].ldb = L.in;
      pw[z].c = x->mlp_slabs + L.w;
      pw[z].ldc = L.in;
      pw[z].colsum = L.b >= 0 ? x->mlp_slabs + L.b : nullptr;
      pw[z].m = L.out;
      pw[z].n = L.in;
      px[z].a = cur[z];
      px[z].lda = L.out;
      px[z].b = P + L.w;
      px[z].ldb = L.in;
      if (l > 0) {
        nxt[z] = x->dz[z][cur[z] == x->dz[z][0] ? 1 : 0];
        px[z].c = nxt[z];
        px[z].aux = x->act[z][l - 1];
      } else {
        px[z].c = x->dfeat[z];
        px[z].aux = x->feat[z];
      }
      px[z].ldc = L.in;
      px[z].m = b;
      px[z].n = L.in;
    }
    const MlpLayer &LA = x->mlp[0].l[l], &LC = x->mlp[1].l[l];
    const bool same = LA.in == LC.in && LA.out == LC.out;
    for (int z = 0; z < (same ? 1 : 2); ++z) {
      GemmBatch gw{};
      gw.p[0] = pw[z];
      if (same) gw.p[1] = pw[1];
      gw.k = b;
      gw.splits = splits;
      gw.slab_stride = x->total;
      gw.prec = x->prec;
      if (int rc = gemm_wgrad_partial(gw, same ? 2 : 1, x->mlp[z].l[l].out, x->mlp[z].l[l].in, st))
        return rc;
      GemmBatch gx{};
      gx.p[0] = px[z];
      if (same) gx.p[1] = px[1];
      gx.k = x->mlp[z].l[l].out;
      gx.act = l > 0 ? x->mlp[z].l[l - 1].act : PPO_ACT_RELU;  // the encoder's output ReLU
      gx.prec = x->prec;
      if (int rc = gemm_rows_dx(gx, same ? 2 : 1, b, x->mlp[z].l[l].in, st))
        return rc;
    }
    cur[0] = nxt[0];
    cur[1] = nxt[1];
  }
  return 0;
}

int forward_all(ppo_cnn_ctx *x, const uint8_t *frames, const int32_t *rows, int b, hipStream_t st) {
  if (int rc = encoder_forward(x, frames, rows, b, st)) return rc;
  return mlp_forward(x, b, st);
}

}  // namespace

// ============================================================================================
// C-ABI
// ============================================================================================
extern "C" int ppo_cnn_ctx_create(const ppo_cnn_cfg *cfg, int device, ppo_cnn_ctx **out) {
  PPO_REQUIRE(cfg != nullptr && out != nullptr, "ppo_cnn_ctx_create: null argument");
  const ppo_cnn_cfg &c = *cfg;
  PPO_REQUIRE(c.height == L1::hin && c.width == L1::win && c.channels == L1::cin,
              "ppo_cnn_ctx_create: frames %dx%dx%d; the compiled encoder takes %dx%dx%d",
              c.height, c.width, c.channels, L1::hin, L1::win, L1::cin);
  PPO_REQUIRE(c.act_dim >= 1 && c.act_dim <= kMaxA, "ppo_cnn_ctx_create: act_dim %d", c.act_dim);
  PPO_REQUIRE(c.n_hidden >= 0 && c.n_hidden <= PPO_MAX_LAYERS, "ppo_cnn_ctx_create: %d hidden layers",
              c.n_hidden);
  PPO_REQUIRE(c.activation >= PPO_ACT_RELU && c.activation <= PPO_ACT_ELU,
              "ppo_cnn_ctx_create: activation %d", c.activation);
  PPO_REQUIRE(c.max_rows > 0, "ppo_cnn_ctx_create: max_rows %d", c.max_rows);
  for (int l = 0; l < c.n_hidden; ++l)
    PPO_REQUIRE(c.hidden[l] > 0 && c.hidden[l] <= 4096 && c.hidden[l] % 4 == 0,
                "ppo_cnn_ctx_create: hidden width %d (multiple of 4 in [4, 4096])", c.hidden[l]);
  ppo_cnn_ctx *x = new (std::nothrow) ppo_cnn_ctx();
  PPO_REQUIRE(x != nullptr, "ppo_cnn_ctx_create: out of host memory");
  x->cfg = c;
  x->device = device;
  x->prec = PPO_PREC_F32;
  x->ent_log_share = 1.f;
  const int A = c.act_dim;
  int64_t off = 0;
  // actor: actor_logstd (the module's own parameter comes first in parameters()), encoder, MLP
  x->logstd_off = off;
  x->offsets.push_back(off);
  off = align_up(off + A, kAlign);
  add_conv<L1>(x->conv[0][0], off, x->offsets);
  add_conv<L2>(x->conv[0][1], off, x->offsets);
  add_conv<L3>(x->conv[0][2], off, x->offsets);
  add_mlp(x->mlp[0], kFeatures, c, A, PPO_ACT_TANH, c.use_bias != 0, off, x->offsets);
  x->n_actor = off;
  // critic: encoder, MLP (the reference critic's layers always have biases, critic.py:20)
  add_conv<L1>(x->conv[1][0], off, x->offsets);
  add_conv<L2>(x->conv[1][1], off, x->offsets);
  add_conv<L3>(x->conv[1][2], off, x->offsets);
  add_mlp(x->mlp[1], kFeatures, c, 1, PPO_ACT_IDENTITY, true, off, x->offsets);
  x->total = off;
  int maxw = std::max(A, 1);
  for (int l = 0; l < c.n_hidden; ++l) maxw = std::max(maxw, c.hidden[l]);
  x->maxw = maxw;
  const int64_t R = c.max_rows;
  x->rows = R;
  x->cslab_stride[0] = slab_floats<L1>();
  x->cslab_stride[1] = slab_floats<L2>();
  x->cslab_stride[2] = slab_floats<L3>();
  int64_t need = 0;
  auto take = [&](int64_t n) {
    const int64_t at = need;
    need = align_up(need + n, kWsAlign);
    return at;
  };
  int64_t o_wdg[2][2], o_wfw[2][2], o_pack[2][3], o_a1[2], o_a2[2], o_feat[2], o_act[2][PPO_MAX_LAYERS + 1], o_dz[2][2],
      o_dfeat[2], o_dz2[2], o_dz1[2], o_cslab[2][3];
  const int64_t ksz[3] = {static_cast<int64_t>(L1::cout) * L1::kdim,
                          static_cast<int64_t>(L2::cout) * L2::kdim,
                          static_cast<int64_t>(L3::cout) * L3::kdim};
  for (int z = 0; z < 2; ++z) {
    for (int l = 0; l < 3; ++l) o_pack[z][l] = take(ksz[l]);
    o_wdg[z][0] = take(L2D::N * L2D::KD / 2);  // bf16
    o_wdg[z][1] = take(L3D::N * L3D::KD / 2);
    o_wfw[z][0] = take(L2F::CO * L2F::KD / 2);
    o_wfw[z][1] = take(L3F::CO * L3F::KD / 2);
    o_a1[z] = take(R * L1::P * L1::cout);  // f32-sized (bf16 uses half)
    o_a2[z] = take(R * L2::P * L2::cout);
    o_feat[z] = take(R * kFeatures);
    for (int l = 0; l < x->mlp[z].n; ++l) o_act[z][l] = take(R * x->mlp[z].l[l].out);
    o_dz[z][0] = take(R * maxw);
    o_dz[z][1] = take(R * maxw);
    o_dfeat[z] = take(R * kFeatures);
    o_dz2[z] = take(R * L2::P * L2::cout);
    o_dz1[z] = take(R * L1::P * L1::cout);
    for (int l = 0; l < 3; ++l) o_cslab[z][l] = take(kConvMaxSplits * x->cslab_stride[l]);
  }
  const int64_t o_mslab = take(kMlpSplits * x->total);
  const int64_t o_ls = take(static_cast<int64_t>(kHeadSplits) * A);
  const int64_t o_loss = take(static_cast<int64_t>(kHeadSplits) * 2);
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc(&x->ws, sizeof(float) * std::max<int64_t>(need, 1));
  if (e == hipSuccess) e = hipMemset(x->ws, 0, sizeof(float) * std::max<int64_t>(need, 1));
  if (e != hipSuccess) {
    set_error("ppo_cnn_ctx_create: allocating %lld floats of workspace failed: %s",
              static_cast<long long>(need), hipGetErrorString(e));
    if (x->ws) (void)hipFree(x->ws);
    delete x;
    return PPO_EHIP;
  }
  float *w = x->ws;
  for (int z = 0; z < 2; ++z) {
    for (int l = 0; l < 3; ++l) {
      x->wpack[z][l] = w + o_pack[z][l];
      if (l < 2) x->wdg[z][l] = reinterpret_cast<__bf16 *>(w + o_wdg[z][l]);
      if (l < 2) x->wfw[z][l] = reinterpret_cast<__bf16 *>(w + o_wfw[z][l]);
      x->cslab[z][l] = w + o_cslab[z][l];
    }
    x->a1[z] = w + o_a1[z];
    x->a2[z] = w + o_a2[z];
    x->feat[z] = w + o_feat[z];
    for (int l = 0; l < x->mlp[z].n; ++l) x->act[z][l] = w + o_act[z][l];
    x->dz[z][0] = w + o_dz[z][0];
    x->dz[z][1] = w + o_dz[z][1];
    x->dfeat[z] = w + o_dfeat[z];
    x->dz2[z] = w + o_dz2[z];
    x->dz1[z] = w + o_dz1[z];
  }
  x->mlp_slabs = w + o_mslab;
  x->ls_part = w + o_ls;
  x->loss_part = w + o_loss;
  *out = x;
  return 0;
}

extern "C" int ppo_cnn_ctx_destroy(ppo_cnn_ctx *x) {
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

extern "C" int ppo_cnn_param_layout(const ppo_cnn_ctx *x, int64_t *offsets, int max_tensors,
                                    int64_t *total, int64_t *n_actor) {
  PPO_REQUIRE(x != nullptr, "ppo_cnn_param_layout: null ctx");
  const int n = static_cast<int>(x->offsets.size());
  if (offsets)
    for (int i = 0; i < std::min(n, max_tensors); ++i) offsets[i] = x->offsets[i];
  if (total) *total = x->total;
  if (n_actor) *n_actor = x->n_actor;
  return n;
}

extern "C" int ppo_cnn_bind_params(ppo_cnn_ctx *x, float *params_d) {
  PPO_REQUIRE(x != nullptr && params_d != nullptr, "ppo_cnn_bind_params: null argument");
  PPO_REQUIRE(reinterpret_cast<uintptr_t>(params_d) % 64 == 0,
              "ppo_cnn_bind_params: parameter buffer must be 64-B aligned");
  x->params = params_d;
  return 0;
}

extern "C" int ppo_cnn_loss_entropy_share(ppo_cnn_ctx *x, float share) {
  PPO_REQUIRE(x != nullptr, "ppo_cnn_loss_entropy_share: null ctx");
  x->ent_log_share = share;
  return 0;
}

extern "C" int ppo_cnn_set_precision(ppo_cnn_ctx *x, int prec) {
  PPO_REQUIRE(x != nullptr, "ppo_cnn_set_precision: null ctx");
  PPO_REQUIRE(prec == PPO_PREC_F32 || prec == PPO_PREC_BF16, "ppo_cnn_set_precision: %d", prec);
  x->prec = prec;
  return 0;
}

extern "C" int ppo_cnn_set_rng_counter(ppo_cnn_ctx *x, const uint64_t *counter_d) {
  PPO_REQUIRE(x != nullptr, "ppo_cnn_set_rng_counter: null ctx");
  x->rng_counter = counter_d;
  return 0;
}

extern "C" int ppo_cnn_forward(ppo_cnn_ctx *x, const uint8_t *frames_d, int n, float *mean_d,
                               float *value_d, float *feat_actor_d, float *feat_critic_d,
                               void *stream) {
  if (int rc = check_rows(x, n)) return rc;
  PPO_REQUIRE(frames_d != nullptr, "ppo_cnn_forward: null frames");
  if (n == 0) return 0;
  PPO_HIP_TRY(hipSetDevice(x->device));
  hipStream_t st = as_stream(stream);
  TimingScope ts(x);
  if (int rc = forward_all(x, frames_d, nullptr, n, st)) return rc;
  const int64_t fb = sizeof(float) * static_cast<int64_t>(n) * kFeatures;
  if (feat_actor_d) PPO_HIP_TRY(hipMemcpyAsync(feat_actor_d, x->feat[0], fb, hipMemcpyDeviceToDevice, st));
  if (feat_critic_d) PPO_HIP_TRY(hipMemcpyAsync(feat_critic_d, x->feat[1], fb, hipMemcpyDeviceToDevice, st));
  HeadArgs h{};
  h.ya = x->act[0][x->mlp[0].n - 1];
  h.vc = x->act[1][x->mlp[1].n - 1];
  h.logstd = x->params + x->logstd_off;
  h.omv = x->cfg.output_max_value;
  h.b = n;
  h.a = x->cfg.act_dim;
  h.mean_out = mean_d;
  h.value_out = value_d;
  launch_k(TimRec{KC_POLICY_HEAD, "cnn_policy_head_kernel", 0.0, 0.0}, cnn_policy_head_kernel,
           dim3(ceil_div(n, 256)), dim3(256), 0, st, h);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_cnn_policy_step(ppo_cnn_ctx *x, const uint8_t *frames_d, int n,
                                   const float *eps_d, uint64_t seed, uint64_t offset,
                                   float *action_d, float *logp_d, float *value_d, float *mean_d,
                                   void *stream) {
  if (int rc = check_rows(x, n)) return rc;
  PPO_REQUIRE(frames_d != nullptr, "ppo_cnn_policy_step: null frames");
  PPO_REQUIRE(action_d != nullptr || logp_d == nullptr,
              "ppo_cnn_policy_step: logp needs the action buffer");
  if (n == 0) return 0;
  PPO_HIP_TRY(hipSetDevice(x->device));
  hipStream_t st = as_stream(stream);
  TimingScope ts(x);
  if (int rc = forward_all(x, frames_d, nullptr, n, st)) return rc;
  HeadArgs h{};
  h.ya = x->act[0][x->mlp[0].n - 1];
  h.vc = x->act[1][x->mlp[1].n - 1];
  h.logstd = x->params + x->logstd_off;
  h.omv = x->cfg.output_max_value;
  h.b = n;
  h.a = x->cfg.act_dim;
  h.eps = eps_d;
  h.seed = seed;
  h.offset = offset;
  h.offset_base = x->rng_counter;
  h.action = action_d;
  h.logp_out = logp_d;
  h.value_out = value_d;
  h.mean_out = mean_d;
  launch_k(TimRec{KC_POLICY_HEAD, "cnn_policy_head_kernel", 0.0, 0.0}, cnn_policy_head_kernel,
           dim3(ceil_div(n, 256)), dim3(256), 0, st, h);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_cnn_minibatch_grad(ppo_cnn_ctx *x, const uint8_t *frames_d,
                                      const float *actions_d, const float *logp_d,
                                      const float *adv_d, const float *vt_d,
                                      const int32_t *rows_d, int b, float *grad_d, float *loss_d,
                                      float clip_lo, float clip_hi, float entropy_coef,
                                      float inv_b, float inv_ba, void *stream) {
  if (int rc = check_rows(x, b)) return rc;
  PPO_REQUIRE(frames_d && actions_d && logp_d && adv_d && vt_d && rows_d && grad_d,
              "ppo_cnn_minibatch_grad: null argument");
  PPO_REQUIRE(b > 0, "ppo_cnn_minibatch_grad: empty minibatch");
  PPO_HIP_TRY(hipSetDevice(x->device));
  hipStream_t st = as_stream(stream);
  TimingScope ts(x);
  const int A = x->cfg.act_dim;
  if (int rc = forward_all(x, frames_d, rows_d, b, st)) return rc;
  const int head_splits = std::min(kHeadSplits, std::max(1, b / 64));
  HeadArgs h{};
  h.ya = x->act[0][x->mlp[0].n - 1];
  h.vc = x->act[1][x->mlp[1].n - 1];
  h.logstd = x->params + x->logstd_off;
  h.omv = x->cfg.output_max_value;
  h.b = b;
  h.a = A;
  h.rows = rows_d;
  h.actions = actions_d;
  h.old_logp = logp_d;
  h.adv = adv_d;
  h.vt = vt_d;
  h.dza = x->dz[0][0];
  h.dzc = x->dz[1][0];
  h.ls_part = x->ls_part;
  h.loss_part = x->loss_part;
  h.splits = head_splits;
  h.clip_lo = clip_lo;
  h.clip_hi = clip_hi;
  h.ent_coef = entropy_coef;
  h.inv_b = inv_b;
  h.inv_ba = inv_ba;
  launch_k(TimRec{KC_UPDATE_HEAD, "cnn_update_head_kernel", 0.0, 0.0}, cnn_update_head_kernel,
           dim3(head_splits), dim3(256), 0, st, h);
  PPO_LAUNCHED();
  const int mlp_splits = std::min(kMlpSplits, std::max(1, b / 512));
  if (int rc = mlp_backward(x, b, mlp_splits, st)) return rc;
  if (int rc = encoder_backward(x, frames_d, rows_d, b, st)) return rc;

  // slabs -> flat gradient in ascending tensor order, each in a fixed split order
  ReduceArgs r{};
  int ns = 0;
  auto seg = [&](int64_t dst, int64_t len, const float *src, int64_t stride, int nsplit) {
    ReduceSeg &g = r.seg[ns++];
    g.dst = dst;
    g.len = len;
    g.src = src;
    g.stride = stride;
    g.nsplit = nsplit;
  };
  const int64_t ksz[3] = {static_cast<int64_t>(L1::cout) * L1::kdim,
                          static_cast<int64_t>(L2::cout) * L2::kdim,
                          static_cast<int64_t>(L3::cout) * L3::kdim};
  const int cout[3] = {L1::cout, L2::cout, L3::cout};
  for (int z = 0; z < 2; ++z) {
    if (z == 0) seg(x->logstd_off, A, x->ls_part, A, head_splits);
    for (int l = 0; l < 3; ++l) {
      const int ns_l = x->cslab_splits_last[l];
      seg(x->conv[z][l].w, ksz[l], x->cslab[z][l], x->cslab_stride[l], ns_l);
      seg(x->conv[z][l].b, cout[l], x->cslab[z][l] + ksz[l], x->cslab_stride[l], ns_l);
    }
    for (int l = 0; l < x->mlp[z].n; ++l) {
      const MlpLayer &L = x->mlp[z].l[l];
      seg(L.w, static_cast<int64_t>(L.out) * L.in, x->mlp_slabs + L.w, x->total, mlp_splits);
      if (L.b >= 0) seg(L.b, L.out, x->mlp_slabs + L.b, x->total, mlp_splits);
    }
  }
  PPO_REQUIRE(ns <= kMaxSegs, "ppo_cnn_minibatch_grad: %d tensors exceed the reduction table", ns);
  r.nseg = ns;
  r.total = x->total;
  r.grad = grad_d;
  r.loss_part = x->loss_part;
  r.loss_splits = head_splits;
  r.inv_b = inv_b;
  r.logstd = x->params + x->logstd_off;
  r.act_dim = A;
  r.ent_coef = entropy_coef * x->ent_log_share;
  r.loss_out = loss_d;
  launch_k(TimRec{KC_REDUCE, "reduce_slabs_kernel", 0.0, 0.0}, cnn_reduce_kernel,
           dim3(ceil_div(x->total, kRedParams)), dim3(kRedThreads), 0, st, r);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_cnn_timing(ppo_cnn_ctx *x, int enable, int capacity) {
  PPO_REQUIRE(x != nullptr, "ppo_cnn_timing: null ctx");
  return timing_enable(x->tim, enable, capacity);
}

extern "C" int ppo_cnn_timing_kernel(ppo_cnn_ctx *x, int index, const char **name, int *kclass,
                                     double *total_ms, int64_t *launches, double *flops,
                                     double *bytes) {
  PPO_REQUIRE(x != nullptr, "ppo_cnn_timing_kernel: null ctx");
  return timing_read_kernel(x->tim, index, name, kclass, total_ms, launches, flops, bytes);
}

extern "C" int ppo_synthetic_pixel_step(uint32_t seed, int t, const float *action_d, int n, int h,
                                        int w, int c, int a, uint8_t *frames_out_d,
                                        const float *base_reward_d, const uint8_t *base_term_d,
                                        double *reward_out_d, uint8_t *term_out_d, void *stream) {
  PPO_REQUIRE(frames_out_d != nullptr, "ppo_synthetic_pixel_step: null frames");
  PPO_REQUIRE(n >= 0 && h > 0 && w > 0 && c > 0 && (h * w * c) % 4 == 0 && a >= 1 && a <= kMaxA,
              "ppo_synthetic_pixel_step: bad shape");
  PPO_REQUIRE(!reward_out_d || (base_reward_d && base_term_d && term_out_d && action_d && t >= 1),
              "ppo_synthetic_pixel_step: rewards need the base streams, an action and t >= 1");
  if (n == 0) return 0;
  FreeTimingScope ts;
  PixelArgs p{};
  p.seed = seed;
  p.t = t;
  p.n = n;
  p.h = h;
  p.w = w;
  p.c = c;
  p.a = a;
  p.action = action_d;
  p.out = frames_out_d;
  p.base_reward = base_reward_d;
  p.base_term = base_term_d;
  p.reward_out = reward_out_d;
  p.term_out = term_out_d;
  const int64_t threads = static_cast<int64_t>(n) * (h * w * c / 4);
  launch_k(TimRec{KC_ENV, "pixel_env_step_kernel", 0.0, static_cast<double>(n) * h * w * c},
           pixel_env_step_kernel, dim3(ceil_div(threads, 256)), dim3(256), 0, as_stream(stream), p);
  PPO_LAUNCHED();
  return 0;
}
