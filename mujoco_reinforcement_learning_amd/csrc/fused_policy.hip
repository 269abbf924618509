// Fused rollout policy step for precision mode bf16 (SURVEY.md s8(a) A1-A4 in one launch):
// observation-window push + per-sample standardisation (running_gym_sequential_vectorized.py:
// 53-58, 61-92), actor and critic forward (network_block_creator.py:74-86, linear/actor.py:
// 25-30, critic.py:22-25), Normal sampling and log-prob (ppo_agent.py:27-43, ppo.py:22-26).
//
// grid = (ceil(N / RP), nets): blockIdx.y is the net (0 actor, 1 critic), one workgroup = RP = 32
// envs of one net (256 workgroups at N = 4096: every CU busy), 8 waves, wave w owning hidden
// features 32w..32w+31 -- the same LDS images, weight ring and MFMA maps as the fused update
// kernel (fused_common.h) on one 32-row tile instead of two, so a rollout step and the update's
// forward compute identical bf16-operand products.  The head width is compile-time
// (actor: act_dim padded to 2/4/6/8 with zero head rows; critic: 1).
//
// Window length 1 (every MLP config): the pushed window is the new observation itself, so both
// nets' workgroups standardise the same values independently and only the actor's (the critic's
// on a value-only call) write the window and the state.  The standardisation is the A1 kernels' f64 loop (same order, bit-
// identical states).
#include <type_traits>

#include "fused_common.h"
#include "fused_policy.h"
#include "row_stats.h"

namespace ppo {

using namespace fu;

constexpr int kPolicyXsPitch = 33;  // f64 observation staging pitch (doubles)
constexpr int RP = 32;              // envs per workgroup (one 32-row MFMA tile)
constexpr int NTP = RP / 32;        // row tiles per workgroup

template <int H>
struct PolicyLds {
  static constexpr int PITCH = 2 * H;
  static constexpr int X = 0;                                   // bf16 [RP][32]
  static constexpr int A1 = X + RP * 64;                        // bf16 [RP][H]
  static constexpr int A2 = A1 + RP * PITCH;                    // bf16 [RP][H]
  static constexpr int WH = A2 + RP * PITCH;                    // bf16 head image [16][H + 8]
  static constexpr int BIAS = WH + HeadImg<H>::BYTES;           // f32 b0[H], b1[H]
  static constexpr int HS = BIAS + 2 * H * 4;                   // f32 head bias[8], logstd[8]
  static constexpr int XD = HS + 16 * 4;                        // f64 [RP][33] raw observations
  static constexpr int EPS = XD + RP * kPolicyXsPitch * 8;      // f32 [RP][8] sampling noise
  static constexpr int TOTAL = EPS + RP * 8 * 4;
  static_assert(TOTAL <= 163840, "LDS budget");
};

// Barriers are LDS-only (lds_sync): the waves hand each other data through LDS only, and the
// window / state stores issued before a barrier are not waited for there
template <int H, int ACT, int NH, bool ACTOR, bool STAMP = false>
__device__ __forceinline__ void policy_body(const PolicyFusedArgs &q, const FusedNet &N,
                                            char *lds) {
  // STAMP (diagnostic build): wave 0 records s_memtime at each phase boundary
  uint64_t tst[9];
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
  double *const xd = reinterpret_cast<double *>(lds + L::XD);
  float *const eps_s = reinterpret_cast<float *>(lds + L::EPS);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int row0 = blockIdx.x * RP;
  const int A = q.act_dim;
  const int O = q.obs_dim;
  const int nrow = min(RP, q.n - row0);
  // the window / state writer: the actor's workgroups, or the critic's on a value-only call
  const bool writer = ACTOR || !q.do_actor;

  // ---- prologue: every global load of the step issued before any use (one memory latency for
  //      the whole prologue).  Observations: element e = (row e/32, feature e%32) of the block's
  //      rows, from clamped valid addresses (no load behind a branch).  Parameters: the bf16 head
  //      image's f32 sources, b0 / b1, head bias / log-std.  Sampling noise: host eps or Philox,
  //      computed here by every thread for (row tid/8, action tid%8) ----
  // Nullable inputs are read from a valid stand-in address (the head weights) and masked only
  // where the values are stored to LDS: a load behind a branch, or a select the compiler turns
  // into one, makes it wait for every load issued before it.  Pointer choices are wave-uniform
  // (scalar selects) and the loads go through address-space-1 pointers (global, not flat).
  const float *const fb = N.wh;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  // the Philox counter base first: the noise below waits only for this load
  const uint64_t obraw =
      *gptr(q.offset_base ? q.offset_base : reinterpret_cast<const uint64_t *>(fb));
  const int erow = tid >> 3, ea = tid & 7;
  const int64_t eidx = static_cast<int64_t>(row0 + erow) * A + ea;
  float eraw = 0.f;
  if constexpr (ACTOR) {
    const int64_t eidx_c = static_cast<int64_t>(row0 + min(erow, nrow - 1)) * A + min(ea, A - 1);
    eraw = gptr(q.eps ? q.eps : fb)[q.eps ? eidx_c : 0];
  }
  const double *const xsrc = q.obs_d ? q.obs_d : q.window_d;  // W = 1: the window is the obs
  constexpr int XE = RP * kFusedKX / NT;                         // 2 elements per thread
  double xv[XE];
#pragma unroll
  for (int k = 0; k < XE; ++k) {
    const int e = tid + NT * k, row = e >> 5, f = e & 31;
    const int64_t gi = static_cast<int64_t>(row0 + min(row, nrow - 1)) * O + min(f, O - 1);
    xv[k] = gptr(xsrc)[gi];
  }
  constexpr int WHE = 16 * (H / 2) / NT;  // head-image f32 pairs per thread
  float2 whv[WHE];
  const int nh_real = ACTOR ? A : 1;
#pragma unroll
  for (int k = 0; k < WHE; ++k) {
    const int i = tid + NT * k, a = i / (H / 2), f = 2 * (i % (H / 2));
    const uint64_t u = *gptr(reinterpret_cast<const uint64_t *>(N.wh + min(a, nh_real - 1) * H + f));
    whv[k] = make_float2(__uint_as_float(static_cast<uint32_t>(u)), __uint_as_float(static_cast<uint32_t>(u >> 32)));
  }
  static_assert(2 * H == NT, "one bias value per thread: waves 0..NW/2-1 b0, the rest b1");
  const float braw = gptr(wu < NW / 2 ? (N.b0 ? N.b0 : fb) : (N.b1 ? N.b1 : fb))[tid % H];
  // hs[0..7] head bias, hs[8..15] the actor's log-std (wave 0)
  const float hraw = gptr(wu == 0 && (lane & 8) ? (q.logstd ? q.logstd : fb)
                                                : (N.bh ? N.bh : fb))[tid & 7];
  // the L0 weight fragments and the first W1 ring fragments: in flight under the observation
  // loads and the f64 statistics instead of at the start of their passes
  bf16x8 w0f[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
    w0f[s] = *reinterpret_cast<const bf16x8 *>(N.w0b + (32 * w + r) * kFusedKX + 16 * s + 8 * h);
  bf16x8 ring[PD + 1];
  wring_prime<H>(w_frag_base<H>(N.w1b, w, lane), ring);
  float epsv = 0.f;
  if (ACTOR && !q.eps && ea < A && erow < nrow)
    epsv = philox_normal_at(q.seed, q.offset + (q.offset_base ? obraw : 0) + eidx);
  PSTAMP(1);
  // ---- LDS images of the loaded values (masking happens here); the raw window row out
  //      (writer, obs given) ----
#pragma unroll
  for (int k = 0; k < WHE; ++k) {
    const int i = tid + NT * k, a = i / (H / 2), f = 2 * (i % (H / 2));
    const bool ok = a < nh_real;
    *reinterpret_cast<uint32_t *>(whb + a * HeadImg<H>::PITCH + 2 * f) =
        pack2(ok ? whv[k].x : 0.f, ok ? whv[k].y : 0.f);
  }
  bias[tid] = (wu < NW / 2 ? N.b0 != nullptr : N.b1 != nullptr) ? braw : 0.f;
  if (tid < 16)
    hs[tid] = (tid < 8 ? (tid < nh_real && N.bh != nullptr) : (ACTOR && tid - 8 < A)) ? hraw : 0.f;
  if (ACTOR && tid < RP * 8) eps_s[tid] = q.eps ? ((ea < A && erow < nrow) ? eraw : 0.f) : epsv;
#pragma unroll
  for (int k = 0; k < XE; ++k) {
    const int e = tid + NT * k, row = e >> 5, f = e & 31;
    const bool ok = row < nrow && f < O;
    xd[row * kPolicyXsPitch + f] = ok ? xv[k] : 0.0;
    if (ok && writer && q.obs_d)
      q.window_d[static_cast<int64_t>(row0 + row) * O + f] = xv[k];
  }
  lds_sync();
  PSTAMP(2);
  // ---- per-(row, slice) mean and std on every wave, and the standardised states in the same
  //      phase: lane = feature (lanes 0-31 and 32-63 are two rows), each wave 4 rows as two
  //      interleaved chains.  row_stats.h's pairwise tree over the 32 slots is a DPP / permlane
  //      butterfly across the 32 lanes (slice_stats_lanes), so mean / std are bitwise the layered
  //      A1 kernel's; every lane ends with its rows' statistics and standardises its own feature
  //      right there ((x - mean) / std in f64, then f32): no statistics round trip through LDS and
  //      no separate phase / barrier.  The bf16 X image (16-bit stores, RNE like pack2) and the
  //      f32 state (writer workgroups) ----
  static_assert(4 * NW == RP, "four rows per wave");
  {
    const int f = lane & 31;
    const int ra = 4 * w + 2 * (lane >> 5), rb = ra + 1;  // the two rows of this lane
    const double xa = xd[ra * kPolicyXsPitch + f], xb = xd[rb * kPolicyXsPitch + f];
    float ya = f < O ? static_cast<float>(xa) : 0.f, yb = f < O ? static_cast<float>(xb) : 0.f;
    if (q.normalize) {
      ya = 0.f;
      yb = 0.f;
      for (int sl = 0; sl < q.tab.count; ++sl) {
        const int lo = q.tab.edge[sl], hi = q.tab.edge[sl + 1];
        if (hi - lo <= 0) continue;  // uniform
        const bool in = f >= lo && f < hi;
        const SliceStats2 s2 = slice_stats_lanes(xa, xb, in, hi - lo);
        if (in) {
          ya = static_cast<float>((xa - s2.mean[0]) / s2.sd[0]);
          yb = static_cast<float>((xb - s2.mean[1]) / s2.sd[1]);
        }
      }
    }
    if (ra >= nrow) ya = 0.f;
    if (rb >= nrow) yb = 0.f;
    *reinterpret_cast<uint16_t *>(ximg + x_off(ra, f >> 3) + 2 * (f & 7)) =
        static_cast<uint16_t>(pack2(ya, 0.f) & 0xffffu);
    *reinterpret_cast<uint16_t *>(ximg + x_off(rb, f >> 3) + 2 * (f & 7)) =
        static_cast<uint16_t>(pack2(yb, 0.f) & 0xffffu);
    if (writer && f < O) {
      if (ra < nrow) q.state_d[static_cast<int64_t>(row0 + ra) * O + f] = ya;
      if (rb < nrow) q.state_d[static_cast<int64_t>(row0 + rb) * O + f] = yb;
    }
  }
  lds_sync();
  PSTAMP(3);
  PSTAMP(4);

  // ---- L0: a1 = act(W0 x + b0) -> A1 image ----
  {
    f32x16 acc[NTP];
#pragma unroll
    for (int t = 0; t < NTP; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int t = 0; t < NTP; ++t)
        acc[t] = mfma(w0f[s], lds_b128(ximg + x_off(32 * t + r, 2 * s + h)), acc[t]);
    }
    mfma_drain(acc);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * w + 8 * g + 4 * h;
      const float4 bv = *reinterpret_cast<const float4 *>(bias + f0);
#pragma unroll
      for (int t = 0; t < NTP; ++t) {
        const float y0 = act_forward(acc[t][4 * g] + bv.x, ACT);
        const float y1 = act_forward(acc[t][4 * g + 1] + bv.y, ACT);
        const float y2 = act_forward(acc[t][4 * g + 2] + bv.z, ACT);
        const float y3 = act_forward(acc[t][4 * g + 3] + bv.w, ACT);
        *reinterpret_cast<uint2 *>(a1img + img_off(32 * t + r, 4 * w + g, L::PITCH) + 8 * h) =
            make_uint2(pack2(y0, y1), pack2(y2, y3));
      }
    }
  }
  lds_sync();
  PSTAMP(5);

  // ---- L1: a2 = act(W1 a1 + b1) -> A2 image (bf16: the head's operand) ----
  {
    f32x16 a2[NTP];
#pragma unroll
    for (int t = 0; t < NTP; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) a2[t][e] = 0.f;
    mlp_pass<H>(w_frag_base<H>(N.w1b, w, lane), a1img, r, h, ring, a2);
    PSTAMP(6);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int f0 = 32 * w + 8 * g + 4 * h;
      const float4 bv = *reinterpret_cast<const float4 *>(bias + H + f0);
#pragma unroll
      for (int t = 0; t < NTP; ++t)
        *reinterpret_cast<uint2 *>(a2img + img_off(32 * t + r, 4 * w + g, L::PITCH) + 8 * h) =
            make_uint2(pack2(act_forward(a2[t][4 * g] + bv.x, ACT), act_forward(a2[t][4 * g + 1] + bv.y, ACT)),
                       pack2(act_forward(a2[t][4 * g + 2] + bv.z, ACT), act_forward(a2[t][4 * g + 3] + bv.w, ACT)));
    }
  }
  lds_sync();
  PSTAMP(7);

  // ---- heads: z = a2 . W_h^T on the 16x16x32 MFMA (the update kernel's bf16 products); waves w
  //      and w + 4 form the same 16-row tile and split its rows: lane -> head n = lane & 15, rows
  //      16 (w & 3) + 4 (lane >> 4) + 2 (w >> 2) + {0, 1}; RP / 16 tiles, so waves with
  //      (w & 3) >= RP / 16 only take part in the exchange barrier ----
  {
    const int n = lane & 15, qg = lane >> 4, tile = w & 3, half = w >> 2;
    const bool head_wave = tile < RP / 16;
    // K split between the wave pair (the update kernel's head order): half 0 sums k-steps
    // 0..H/64-1, half 1 the rest; partners swap their kept rows through the free A1 region
    f32x4 zacc = {0.f, 0.f, 0.f, 0.f};
    if (head_wave) {
#pragma unroll
      for (int s = half * (H / 64); s < (half + 1) * (H / 64); ++s)
        zacc = mfma16(lds_b128(a2img + img_off(16 * tile + n, 4 * s + qg, L::PITCH)),
                      lds_b128(whb + n * HeadImg<H>::PITCH + 2 * (32 * s + 8 * qg)), zacc);
    }
    asm volatile("s_nop 15" : "+v"(zacc));
    float *const xch = reinterpret_cast<float *>(a1img);  // [8 waves][64 lanes][2]
    *reinterpret_cast<float2 *>(xch + 2 * (w * 64 + lane)) =
        half ? make_float2(zacc[0], zacc[1]) : make_float2(zacc[2], zacc[3]);
    lds_sync();
    const float2 px = *reinterpret_cast<const float2 *>(xch + 2 * ((w ^ (NW / 2)) * 64 + lane));
    const float zr[2] = {(half ? zacc[2] : zacc[0]) + px.x, (half ? zacc[3] : zacc[1]) + px.y};
    if (!head_wave) {
    } else if constexpr (ACTOR) {
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
          const float e = eps_s[(env - row0) * 8 + n];  // staged in the prologue
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
  PSTAMP(8);
  if constexpr (STAMP) {
    if (tid == 0 && blockIdx.x < 128) {
      uint64_t *dst = q.stamps + (static_cast<int64_t>(blockIdx.y) * 128 + blockIdx.x) * 11;
#pragma unroll
      for (int k = 0; k < 8; ++k) dst[k] = tst[k + 1] - tst[k];
      dst[9] = tst[8] - tst[0];
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
  const dim3 grid(ceil_div(q.n, RP), (q.do_actor && q.do_critic) ? 2 : 1);
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
