// Fused rollout policy step for precision mode bf16 (SURVEY.md s8(a) A1-A4 in one launch):
// observation-window push + per-sample standardisation (running_gym_sequential_vectorized.py:
// 53-58, 61-92), actor and critic forward (network_block_creator.py:74-86, linear/actor.py:
// 25-30, critic.py:22-25), Normal sampling and log-prob (ppo_agent.py:27-43, ppo.py:22-26).
//
// grid = (ceil(N / 64), nets): blockIdx.y is the net (0 actor, 1 critic), one workgroup = 64
// envs of one net, 8 waves, wave w owning hidden features 32w..32w+31 -- the same LDS images,
// weight ring and MFMA maps as the fused update kernel (fused_common.h), so a rollout step and
// the update's forward compute identical bf16-operand products.  The head width is compile-time
// (actor: act_dim padded to 2/4/6/8 with zero head rows; critic: 1).
//
// Window length 1 (every MLP config): the pushed window is the new observation itself, so both
// nets' workgroups standardise the same values independently and only the actor's (the critic's
// on a value-only call) write the window and the state.  The standardisation is the A1 kernels' f64 loop (same order, bit-
// identical states).
#include <type_traits>

#include "fused_common.h"
#include "fused_policy.h"

namespace ppo {

using namespace fu;

constexpr int kPolicyXsPitch = 33;  // f32 state staging pitch (floats)

template <int H>
struct PolicyLds {
  static constexpr int PITCH = 2 * H;
  static constexpr int X = 0;                                   // bf16 [64][32]
  static constexpr int A1 = X + R * 64;                         // bf16 [64][H]
  static constexpr int A2 = A1 + R * PITCH;                     // bf16 [64][H]
  static constexpr int WH = A2 + R * PITCH;                     // bf16 head image [16][H + 8]
  static constexpr int BIAS = WH + HeadImg<H>::BYTES;           // f32 b0[H], b1[H]
  static constexpr int HS = BIAS + 2 * H * 4;                   // f32 head bias[8], logstd[8]
  static constexpr int XS = HS + 16 * 4;                        // f32 [64][33] standardised states
  static constexpr int TOTAL = XS + R * kPolicyXsPitch * 4;
  static_assert(TOTAL <= 163840, "LDS budget");
};

template <int H, int ACT, int NH, bool ACTOR, bool STAMP = false>
__device__ __forceinline__ void policy_body(const PolicyFusedArgs &q, const FusedNet &N,
                                            char *lds) {
  // STAMP (diagnostic build): wave 0 records s_memtime at each phase boundary
  uint64_t tst[8];
#define PSTAMP(k)                                      \
  if constexpr (STAMP) {                               \
    tst[k] = __builtin_amdgcn_s_memtime();             \
  }
  PSTAMP(0);
  using L = PolicyLds<H>;
  char *const ximg = lds + L::X;
  char *const a1img = lds + L::A1;
  char *const a2img = lds + L::A2;
  char *const whb = lds + L::WH;
  float *const bias = reinterpret_cast<float *>(lds + L::BIAS);
  float *const hs = reinterpret_cast<float *>(lds + L::HS);
  float *const xs = reinterpret_cast<float *>(lds + L::XS);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int row0 = blockIdx.x * R;
  const int A = q.act_dim;
  const int O = q.obs_dim;

  // ---- stage head (bf16 image) / bias parameters ----
  stage_head_image<H>(whb, N.wh, ACTOR ? A : 1, tid, NT);
  for (int i = tid; i < 2 * H; i += NT) {
    const float *b = i < H ? N.b0 : N.b1;
    bias[i] = b ? b[i % H] : 0.f;
  }
  if (tid < 8) hs[tid] = (tid < (ACTOR ? A : 1) && N.bh) ? N.bh[tid] : 0.f;
  if (ACTOR && tid >= 8 && tid < 16) hs[tid] = (tid - 8 < A) ? q.logstd[tid - 8] : 0.f;

  PSTAMP(1);
  // the window / state writer: the actor's workgroups, or the critic's on a value-only call
  const bool writer = ACTOR || !q.do_actor;
  // ---- observe (A1): thread per env row, the A1 kernels' f64 loops ----
  if (tid < R) {
    const int env = row0 + tid;
    float *dst = xs + tid * kPolicyXsPitch;
    if (env < q.n) {
      const double *src = q.obs_d ? q.obs_d + static_cast<int64_t>(env) * O
                                  : q.window_d + static_cast<int64_t>(env) * O;  // W = 1
      double x[kFusedKX];
#pragma unroll
      for (int f = 0; f < kFusedKX; ++f) x[f] = f < O ? src[f] : 0.0;
#pragma unroll
      for (int f = 0; f < kFusedKX; ++f) dst[f] = (!q.normalize && f < O) ? static_cast<float>(x[f]) : 0.f;
      if (q.normalize) {
        for (int sl = 0; sl < q.tab.count; ++sl) {
          const int lo = q.tab.edge[sl], hi = q.tab.edge[sl + 1];
          const int cnt = hi - lo;
          if (cnt <= 0) continue;
          double sum = 0.0;
#pragma unroll
          for (int f = 0; f < kFusedKX; ++f)
            if (f >= lo && f < hi) sum += x[f];
          const double mean = sum / cnt;
          double csum = 0.0;
#pragma unroll
          for (int f = 0; f < kFusedKX; ++f)
            if (f >= lo && f < hi) csum += x[f] - mean;
          const double cmean = csum / cnt;
          double ss = 0.0;
#pragma unroll
          for (int f = 0; f < kFusedKX; ++f)
            if (f >= lo && f < hi) {
              const double d = (x[f] - mean) - cmean;
              ss += d * d;
            }
          double sd = sqrt(ss / (cnt - 1));  // cnt == 1 -> NaN, as torch.std
          if (sd == 0.0) sd = 1.0;
#pragma unroll
          for (int f = 0; f < kFusedKX; ++f)
            if (f >= lo && f < hi) dst[f] = static_cast<float>((x[f] - mean) / sd);
        }
      }
      if (writer && q.obs_d) {
        double *wrow = q.window_d + static_cast<int64_t>(env) * O;
#pragma unroll
        for (int f = 0; f < kFusedKX; ++f)
          if (f < O) wrow[f] = x[f];
      }
    } else {
#pragma unroll
      for (int f = 0; f < kFusedKX; ++f) dst[f] = 0.f;
    }
  }
  __syncthreads();
  PSTAMP(2);
  // states -> rollout buffer (writer workgroups; coalesced) and the bf16 X image
  if (writer) {
    for (int idx = tid; idx < R * O; idx += NT) {
      const int lrow = idx / O, e = idx - lrow * O, env = row0 + lrow;
      if (env < q.n) q.state_d[static_cast<int64_t>(env) * O + e] = xs[lrow * kPolicyXsPitch + e];
    }
  }
  for (int idx = tid; idx < R * 16; idx += NT) {
    const int xr = idx >> 4, c2 = (idx & 15) * 2;
    *reinterpret_cast<uint32_t *>(ximg + x_off(xr, c2 >> 3) + 2 * (c2 & 7)) =
        pack2(xs[xr * kPolicyXsPitch + c2], xs[xr * kPolicyXsPitch + c2 + 1]);
  }
  __syncthreads();
  PSTAMP(3);

  // ---- L0: a1 = act(W0 x + b0) -> A1 image ----
  bf16x8 ring[PD + 1];
  wring_prime<H>(w_frag_base<H>(N.w1b, w, lane), ring);
  {
    f32x16 acc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 af = *reinterpret_cast<const bf16x8 *>(N.w0b + (32 * w + r) * kFusedKX + 16 * s + 8 * h);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        acc[t] = mfma(af, lds_b128(ximg + x_off(32 * t + r, 2 * s + h)), acc[t]);
    }
    mfma_drain(acc);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * w + 8 * g + 4 * h;
      const float4 bv = *reinterpret_cast<const float4 *>(bias + f0);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const float y0 = act_forward(acc[t][4 * g] + bv.x, ACT);
        const float y1 = act_forward(acc[t][4 * g + 1] + bv.y, ACT);
        const float y2 = act_forward(acc[t][4 * g + 2] + bv.z, ACT);
        const float y3 = act_forward(acc[t][4 * g + 3] + bv.w, ACT);
        *reinterpret_cast<uint2 *>(a1img + img_off(32 * t + r, 4 * w + g, L::PITCH) + 8 * h) =
            make_uint2(pack2(y0, y1), pack2(y2, y3));
      }
    }
  }
  __syncthreads();
  PSTAMP(4);

  // ---- L1: a2 = act(W1 a1 + b1) -> A2 image (bf16: the head's operand) ----
  {
    f32x16 a2[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) a2[t][e] = 0.f;
    mlp_pass<H>(w_frag_base<H>(N.w1b, w, lane), a1img, r, h, ring, a2);
    PSTAMP(5);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * w + 8 * g + 4 * h;
      const float4 bv = *reinterpret_cast<const float4 *>(bias + H + f0);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        *reinterpret_cast<uint2 *>(a2img + img_off(32 * t + r, 4 * w + g, L::PITCH) + 8 * h) =
            make_uint2(pack2(act_forward(a2[t][4 * g] + bv.x, ACT), act_forward(a2[t][4 * g + 1] + bv.y, ACT)),
                       pack2(act_forward(a2[t][4 * g + 2] + bv.z, ACT), act_forward(a2[t][4 * g + 3] + bv.w, ACT)));
    }
  }
  __syncthreads();
  PSTAMP(6);

  // ---- heads: z = a2 . W_h^T on the 16x16x32 MFMA (the update kernel's bf16 products); waves w
  //      and w + 4 form the same 16-row tile and split its rows: lane -> head n = lane & 15, rows
  //      16 (w & 3) + 4 (lane >> 4) + 2 (w >> 2) + {0, 1} ----
  {
    const int n = lane & 15, qg = lane >> 4, tile = w & 3, half = w >> 2;
    // K split between the wave pair (the update kernel's head order): half 0 sums k-steps
    // 0..H/64-1, half 1 the rest; partners swap their kept rows through the free A1 region
    f32x4 zacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = half * (H / 64); s < (half + 1) * (H / 64); ++s)
      zacc = mfma16(lds_b128(a2img + img_off(16 * tile + n, 4 * s + qg, L::PITCH)),
                    lds_b128(whb + n * HeadImg<H>::PITCH + 2 * (32 * s + 8 * qg)), zacc);
    asm volatile("s_nop 15" : "+v"(zacc));
    float *const xch = reinterpret_cast<float *>(a1img);  // [8 waves][64 lanes][2]
    *reinterpret_cast<float2 *>(xch + 2 * (w * 64 + lane)) =
        half ? make_float2(zacc[0], zacc[1]) : make_float2(zacc[2], zacc[3]);
    __syncthreads();
    const float2 px = *reinterpret_cast<const float2 *>(xch + 2 * ((w ^ (NW / 2)) * 64 + lane));
    const float zr[2] = {(half ? zacc[2] : zacc[0]) + px.x, (half ? zacc[3] : zacc[1]) + px.y};
    if constexpr (ACTOR) {
      const bool act_lane = n < A;
      const float sd = act_lane ? expf(hs[8 + n]) : 1.f;
      const float lsd = act_lane ? logf(sd) : 0.f;
      const float i2var = 1.f / (2.f * (sd * sd));
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int env = row0 + 16 * tile + 4 * qg + 2 * half + i;
        float lp = 0.f;
        if (act_lane && env < q.n) {
          float zz = zr[i];
          if (N.bh) zz += hs[n];
          const float mu = q.omv * tanhf(zz);
          const int64_t idx = static_cast<int64_t>(env) * A + n;
          const float e = q.eps ? q.eps[idx]
                                : philox_normal_at(q.seed, q.offset + (q.offset_base ? *q.offset_base : 0) + idx);
          const float x = e * sd + mu;  // torch.normal: randn*std then + mean (two roundings)
          if (q.action) q.action[idx] = x;
          if (q.mean) q.mean[idx] = mu;
          const float d = x - mu;
          lp = ((-(d * d)) * i2var - lsd) - kLogSqrt2Pi;
        }
        // Normal.log_prob(...).sum(1): fixed xor tree over the 16 head lanes (pads are 0), the
        // same tree as the update kernel's loss head
        const float s = row16_sum(lp);
        if (n == 0 && env < q.n && q.logp) q.logp[env] = s;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int env = row0 + 16 * tile + 4 * qg + 2 * half + i;
        if (n == 0 && env < q.n && q.value) q.value[env] = N.bh ? zr[i] + hs[0] : zr[i];
      }
    }
  }
  PSTAMP(7);
  if constexpr (STAMP) {
    if (tid == 0 && blockIdx.x < 128) {
      uint64_t *dst = q.stamps + (static_cast<int64_t>(blockIdx.y) * 128 + blockIdx.x) * 11;
#pragma unroll
      for (int k = 0; k < 7; ++k) dst[k] = tst[k + 1] - tst[k];
      dst[9] = tst[7] - tst[0];
      dst[10] = tst[0];
    }
  }
#undef PSTAMP
}

template <int H, int ACT, int NA, bool STAMP = false>
__global__ __launch_bounds__(NT, 1) void policy_fused_kernel(PolicyFusedArgs q) {
  __shared__ __attribute__((aligned(16))) char lds[PolicyLds<H>::TOTAL];
  // y = 0 actor, y = 1 critic when both run; a single-net call launches one row of workgroups
  const bool actor = q.do_actor && blockIdx.y == 0;
  if (actor) policy_body<H, ACT, NA, true, STAMP>(q, q.net[0], lds);
  else policy_body<H, ACT, 1, false, STAMP>(q, q.net[1], lds);
}

int policy_fused_launch(const PolicyFusedArgs &q, const TimRec &rec, hipStream_t st) {
  PPO_REQUIRE(q.hidden == 256, "fused policy: hidden width %d not compiled", q.hidden);
  PPO_REQUIRE(q.act_dim >= 1 && q.act_dim <= kFusedMaxAct, "fused policy: act_dim %d", q.act_dim);
  PPO_REQUIRE(q.window == 1 && q.obs_dim <= kFusedKX, "fused policy: needs W = 1, O <= %d",
              kFusedKX);
  PPO_REQUIRE(q.do_actor || q.do_critic, "fused policy: nothing requested");
  const dim3 grid(ceil_div(q.n, R), (q.do_actor && q.do_critic) ? 2 : 1);
  auto go = [&](auto kernel) { launch_k(rec, kernel, grid, dim3(NT), 0, st, q); };
  const int na = q.act_dim <= 2 ? 2 : q.act_dim <= 4 ? 4 : q.act_dim <= 6 ? 6 : 8;
  if (q.stamps) {  // diagnostic build: ReLU, padded head width 6 (HalfCheetah) only
    PPO_REQUIRE(q.act == PPO_ACT_RELU && na == 6, "policy stamps: ReLU with A in (4, 6] only");
    go(policy_fused_kernel<256, PPO_ACT_RELU, 6, true>);
    PPO_LAUNCHED();
    return 0;
  }
  auto by_na = [&](auto act_tag) {
    constexpr int ACTV = decltype(act_tag)::value;
    if (na == 2) go(policy_fused_kernel<256, ACTV, 2>);
    else if (na == 4) go(policy_fused_kernel<256, ACTV, 4>);
    else if (na == 6) go(policy_fused_kernel<256, ACTV, 6>);
    else go(policy_fused_kernel<256, ACTV, 8>);
  };
  if (q.act == PPO_ACT_RELU) by_na(std::integral_constant<int, PPO_ACT_RELU>{});
  else if (q.act == PPO_ACT_TANH) by_na(std::integral_constant<int, PPO_ACT_TANH>{});
  else by_na(std::integral_constant<int, PPO_ACT_ELU>{});
  PPO_LAUNCHED();
  return 0;
}

}  // namespace ppo
