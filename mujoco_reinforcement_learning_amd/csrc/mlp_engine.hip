// Actor-critic MLP forward/backward on gfx950 MFMA + the PPO loss heads + split-K gradient
// reduction, behind the ppo_ctx C-ABI (ppo_policy_step, ppo_minibatch_grad).
//
// Every dense fc-layer product is one MFMA GEMM template (v_mfma_f32_32x32x2_f32: exact f32
// inputs, f32 accumulate -- the reference computes in f32, so parity keeps f32 operands):
//   forward   Y  = act(X W^T + b)          A = X  [rows][in]  (optionally gathered by row index)
//   input grad dX = (dY W) * act'(X)        A = dY [rows][out], B = W [out][in]
//   weight grad dW = dY^T X  (split-K over the minibatch rows, per-split slabs, + bias colsums)
// Operands are staged global -> registers -> LDS ([k][m] / [k][n], row stride +2 words: the
// transposing store is conflict-free for 32-lane write groups, the MFMA fragment reads are
// consecutive), double-buffered with one barrier per k-tile.  Actor and critic layers of equal
// shape run in one launch (blockIdx.z = net).
//
// Heads (output widths A and 1) are wave-per-row VALU kernels: tanh/mean, sampling, log-prob,
// clipped surrogate, Huber, and the head backward, with torch's formulas (SURVEY.md s8(a) A3-A4,
// A11-A13).  Reductions are in a fixed order (split slabs summed 0..S-1), so results are
// bit-reproducible run to run.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include "common.h"
#include "ctx.h"
#include "fused_policy.h"
#include "fused_update.h"
#include "gemm.h"
#include "gemm_ops.h"
#include "reduce_slabs.h"
#include "timing.h"
#include "wide_path.h"

namespace ppo {

// ============================================================================================
// Heads
// ============================================================================================
constexpr int kMaxAct = 32;

struct PolicyHeadArgs {
  const float *ha;   // actor last hidden (n, da) or null
  const float *hc;   // critic last hidden (n, dc) or null
  int da, dc, n, act_dim;
  const float *wa, *ba, *logstd;  // actor head (A, da), (A) or null, (A)
  const float *wc, *bc;           // critic head (1, dc), (1)
  float omv;
  const float *eps;               // (n, A) or null -> Philox(seed, offset + row*A + a)
  uint64_t seed, offset;
  const uint64_t *offset_base;    // device counter added to offset (ppo_ctx_set_rng_counter)
  float *action, *logp, *value, *mean;
  int bf16;                       // precision bf16: head operands rounded to bf16 (f32 accumulate)
};

// One wave per env row.  logp follows Normal.log_prob term by term:
//   (-(x-mu)^2) / (2*var) - log(std) - log(sqrt(2*pi)),  var = std*std,  summed a = 0..A-1.
template <int HPL>
__global__ __launch_bounds__(256) void policy_head_kernel(PolicyHeadArgs q) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= q.n) return;
  if (q.ha) {
    float h[HPL];
    const float *hr = q.ha + static_cast<int64_t>(row) * q.da;
#pragma unroll
    for (int j = 0; j < HPL; ++j) {
      const int k = lane + 64 * j;
      h[j] = (k < q.da) ? (q.bf16 ? bf16_round(hr[k]) : hr[k]) : 0.f;
    }
    float my_z = 0.f;
    for (int a = 0; a < q.act_dim; ++a) {
      const float *w = q.wa + static_cast<int64_t>(a) * q.da;
      float part = 0.f;
#pragma unroll
      for (int j = 0; j < HPL; ++j) {
        const int k = lane + 64 * j;
        if (k < q.da) part = fmaf(h[j], q.bf16 ? bf16_round(w[k]) : w[k], part);
      }
      const float z = wave_sum(part);
      if (lane == a) my_z = z;
    }
    float lp = 0.f;
    if (lane < q.act_dim) {
      const int a = lane;
      const float z = q.ba ? my_z + q.ba[a] : my_z;
      const float mu = q.omv * tanhf(z);
      const float sd = expf(q.logstd[a]);
      const int64_t idx = static_cast<int64_t>(row) * q.act_dim + a;
      const float e =
          q.eps ? q.eps[idx]
                : philox_normal_at(q.seed, q.offset + (q.offset_base ? *q.offset_base : 0) + idx);
      const float x = e * sd + mu;  // torch.normal: randn*std then + mean (two roundings)
      if (q.action) q.action[idx] = x;
      if (q.mean) q.mean[idx] = mu;
      const float d = x - mu;
      const float var = sd * sd;
      lp = ((-(d * d)) / (2.f * var) - logf(sd)) - kLogSqrt2Pi;
    }
    if (q.logp) {
      float s = 0.f;
      for (int a = 0; a < q.act_dim; ++a) s += __shfl(lp, a, 64);
      if (lane == 0) q.logp[row] = s;
    }
  }
  if (q.hc && q.value) {
    const float *hr = q.hc + static_cast<int64_t>(row) * q.dc;
    float part = 0.f;
#pragma unroll
    for (int j = 0; j < HPL; ++j) {
      const int k = lane + 64 * j;
      if (k < q.dc)
        part = q.bf16 ? fmaf(bf16_round(hr[k]), bf16_round(q.wc[k]), part) : fmaf(hr[k], q.wc[k], part);
    }
    const float v = wave_sum(part);
    if (lane == 0) q.value[row] = q.bc ? v + q.bc[0] : v;
  }
}

struct UpdateHeadArgs {
  const float *ha, *hc;          // last hidden (rows, da) / (rows, dc), minibatch order
  float *ga, *gc;                // OUT: dH_L (rows, da) / (rows, dc)
  float *dza, *dzc;              // OUT: d(head pre-activation) (rows, A) / (rows, 1)
  int da, dc, act_dim, act;
  const float *wa, *ba, *logstd, *wc, *bc;
  float omv;
  const int32_t *rows;           // storage row of minibatch row j
  int rows_max;
  const int32_t *rows_n;         // device count (nullable)
  const float *actions, *old_logp, *adv, *vtarget;  // storage arrays
  float clip_lo, clip_hi, ent_coef, inv_b, inv_ba;
  float *logstd_part;            // (splits, A)
  float *loss_part;              // (splits, 2): sum over rows of actor / critic loss terms
  int splits;
  // fused head weight gradient (update_head_q4_kernel<NJ, true>): per split, at hw_part +
  // split * hw_stride: actor W (A, da) | actor b (A) at off_ba | critic W (dc) at off_wc |
  // critic b at off_bc
  float *hw_part;
  int hw_stride, off_ba, off_wc, off_bc;
  int bf16;                      // precision bf16: every head product on bf16-rounded operands
};

// operand rounding of precision mode bf16 (identity in f32 mode)
__device__ __forceinline__ float rb(float x, int bf16) { return bf16 ? bf16_round(x) : x; }
__device__ __forceinline__ float4 rb4(float4 v, int bf16) {
  return bf16 ? make_float4(bf16_round(v.x), bf16_round(v.y), bf16_round(v.z), bf16_round(v.w)) : v;
}

// Fast head: 4 lanes per row, 16 rows per wave pass, D = 16*NJ columns (actor and critic last
// hidden widths equal).  Lane (row r = lane>>2, quarter qd = lane&3) holds float4 chunks
// 16t + 4qd of its row; a head dot product is NJ float4 FMAs against LDS-staged head weights
// (same address for the 16 rows -> LDS broadcast) plus a 2-step shuffle over the row's 4 lanes.
// Per-action work (tanh, log-prob, dz) is spread over the 4 lanes: lane qd owns actions
// a = 4k + qd.  Same torch formulas as update_head_kernel below.
// FW (A <= kFusedHeadAct): also accumulate the head layer's weight gradient, dW = dz^T H_L and
// db = sum dz per net, over the block's rows while H_L is hot in L1/L2 -- lane owns float4
// column chunk c = lane + 64u of both nets -- so the split-K head GEMM (a second full read of
// H_L) is not launched.  Waves combine in a fixed order; one partial per block.
constexpr int kFusedHeadAct = 8;
template <int NJ, bool FW>
// two workgroups per CU where the registers allow it (NJ <= 16: 512 blocks then run in one round)
__global__ __launch_bounds__(256, NJ <= 16 ? 2 : 1) void update_head_q4_kernel(UpdateHeadArgs q) {
  constexpr int D = 16 * NJ;
  // action groups of 4 per lane: the fused-wgrad instantiation runs only for A <= kFusedHeadAct,
  // so it sizes its per-action registers for that (kMaxAct / 4 groups cost it 30 VGPRs)
  constexpr int KA = FW ? kFusedHeadAct / 4 : kMaxAct / 4;
  constexpr int CH = (4 * NJ + 63) / 64;  // float4 column chunks per lane (fused wgrad)
  constexpr int AF = FW ? kFusedHeadAct : 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ float red[4][kMaxAct + 2];
  __shared__ float dvs[4][16];
  const int A = q.act_dim;
  float *wsh = smem;                   // (A + 1) x D: actor head rows, then the critic row
  float *lps = smem + (A + 1) * D;     // [4 waves][16 rows][kMaxAct] log-probs
  float *dzs = lps + 4 * 16 * kMaxAct;  // [4 waves][16 rows][kMaxAct] d(pre-tanh)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane >> 2, qd = lane & 3;
  for (int i = tid; i < A * D; i += 256) wsh[i] = rb(q.wa[i], q.bf16);
  for (int i = tid; i < D; i += 256) wsh[A * D + i] = rb(q.wc[i], q.bf16);
  __syncthreads();
  const int count = q.rows_n ? *q.rows_n : q.rows_max;
  const int r0 = static_cast<int>((static_cast<int64_t>(blockIdx.x) * count) / q.splits);
  const int r1 = static_cast<int>((static_cast<int64_t>(blockIdx.x + 1) * count) / q.splits);
  float *lp_row = lps + (wid * 16 + r) * kMaxAct;
  float *dz_row = dzs + (wid * 16 + r) * kMaxAct;
  float ls_acc[KA];
#pragma unroll
  for (int k = 0; k < KA; ++k) ls_acc[k] = 0.f;
  float la_acc = 0.f, lc_acc = 0.f;
  float4 wa_acc[CH][AF], wc_acc[CH];
  float b_acc = 0.f;  // lane a < A: actor bias a; lane A: critic bias
#pragma unroll
  for (int u = 0; u < CH; ++u) {
    wc_acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int a = 0; a < AF; ++a) wa_acc[u][a] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int base = r0 + 16 * wid; base < r1; base += 64) {  // wave-uniform trip count
    const int j = base + r;
    const bool valid = j < r1;
    const int64_t sr = valid ? q.rows[j] : 0;
    float4 h[NJ];
    const float4 *hrow = reinterpret_cast<const float4 *>(q.ha + static_cast<int64_t>(j) * D);
#pragma unroll
    for (int t = 0; t < NJ; ++t) h[t] = valid ? hrow[4 * t + qd] : make_float4(0, 0, 0, 0);
    // ---- actor head: z_a for the lane's own actions a = 4k + qd
    float zk[KA];
#pragma unroll
    for (int k = 0; k < KA; ++k) {
      zk[k] = 0.f;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int a = 4 * k + qq;
        if (a < A) {
          const float4 *w = reinterpret_cast<const float4 *>(wsh + a * D);
          float p = 0.f;
#pragma unroll
          for (int t = 0; t < NJ; ++t) {
            const float4 wv = w[4 * t + qd];
            const float4 hb = rb4(h[t], q.bf16);
            p = fmaf(hb.x, wv.x, p);
            p = fmaf(hb.y, wv.y, p);
            p = fmaf(hb.z, wv.z, p);
            p = fmaf(hb.w, wv.w, p);
          }
          p += __shfl_xor(p, 1, 64);
          p += __shfl_xor(p, 2, 64);
          if (qq == qd) zk[k] = p;
        }
      }
    }
    float yk[KA], dk[KA], vk[KA];
#pragma unroll
    for (int k = 0; k < KA; ++k) {
      const int a = 4 * k + qd;
      yk[k] = 0.f, dk[k] = 0.f, vk[k] = 1.f;
      if (a < A) {
        const float z = q.ba ? zk[k] + q.ba[a] : zk[k];
        const float y = tanhf(z);
        const float mu = q.omv * y;
        const float sd = expf(q.logstd[a]);
        const float x = valid ? q.actions[sr * A + a] : mu;
        const float d = x - mu;
        const float var = sd * sd;
        lp_row[a] = ((-(d * d)) / (2.f * var) - logf(sd)) - kLogSqrt2Pi;
        yk[k] = y, dk[k] = d, vk[k] = var;
      }
    }
    __threadfence_block();
    float logp = 0.f;
    for (int a = 0; a < A; ++a) logp += lp_row[a];
    const float old_lp = valid ? q.old_logp[sr] : logp;
    const float adv = valid ? q.adv[sr] : 0.f;
    const float ratio = expf(logp - old_lp);
    const float s1 = ratio * adv;
    const float cl = ratio < q.clip_lo ? q.clip_lo : (ratio > q.clip_hi ? q.clip_hi : ratio);
    const float s2 = cl * adv;
    const float mn = (s1 != s1 || s2 != s2) ? (s1 + s2) : (s2 < s1 ? s2 : s1);
    const float g = -q.inv_b;
    const float g1 = (s1 < s2) ? g : (s1 == s2 ? g * 0.5f : 0.f);
    const float g2 = (s2 < s1) ? g : (s1 == s2 ? g * 0.5f : 0.f);
    const bool inside = (ratio >= q.clip_lo) && (ratio <= q.clip_hi);
    const float dratio = g1 * adv + (inside ? g2 * adv : 0.f);
    const float dlogp = valid ? dratio * ratio : 0.f;
    if (valid && qd == 0) la_acc += mn;
#pragma unroll
    for (int k = 0; k < KA; ++k) {
      const int a = 4 * k + qd;
      if (a < A) {
        const float dmu = dlogp * (dk[k] / vk[k]);
        const float dz = (dmu * q.omv) * (1.f - yk[k] * yk[k]);
        dz_row[a] = dz;
        if (valid) {
          ls_acc[k] += dlogp * ((dk[k] * dk[k]) / vk[k] - 1.f) - q.ent_coef * q.inv_ba;
          q.dza[static_cast<int64_t>(j) * A + a] = dz;
        }
      }
    }
    __threadfence_block();
    // ---- dH_L(actor) = (dz . W_head) * act'(h)
    float4 *grow = reinterpret_cast<float4 *>(q.ga + static_cast<int64_t>(j) * D);
#pragma unroll
    for (int t = 0; t < NJ; ++t) {
      float4 s = make_float4(0, 0, 0, 0);
      for (int a = 0; a < A; ++a) {
        const float dz = rb(dz_row[a], q.bf16);
        const float4 wv = reinterpret_cast<const float4 *>(wsh + a * D)[4 * t + qd];
        s.x = fmaf(dz, wv.x, s.x);
        s.y = fmaf(dz, wv.y, s.y);
        s.z = fmaf(dz, wv.z, s.z);
        s.w = fmaf(dz, wv.w, s.w);
      }
      if (valid)
        grow[4 * t + qd] = make_float4(act_backward(s.x, h[t].x, q.act), act_backward(s.y, h[t].y, q.act),
                                       act_backward(s.z, h[t].z, q.act), act_backward(s.w, h[t].w, q.act));
    }
    // ---- critic
    const float4 *crow = reinterpret_cast<const float4 *>(q.hc + static_cast<int64_t>(j) * D);
#pragma unroll
    for (int t = 0; t < NJ; ++t) h[t] = valid ? crow[4 * t + qd] : make_float4(0, 0, 0, 0);
    const float4 *wc = reinterpret_cast<const float4 *>(wsh + A * D);
    float p = 0.f;
#pragma unroll
    for (int t = 0; t < NJ; ++t) {
      const float4 wv = wc[4 * t + qd];
      const float4 hb = rb4(h[t], q.bf16);
      p = fmaf(hb.x, wv.x, p);
      p = fmaf(hb.y, wv.y, p);
      p = fmaf(hb.z, wv.z, p);
      p = fmaf(hb.w, wv.w, p);
    }
    p += __shfl_xor(p, 1, 64);
    p += __shfl_xor(p, 2, 64);
    const float v = q.bc ? p + q.bc[0] : p;
    const float vt = valid ? q.vtarget[sr] : v;
    const float diff = v - vt;
    const float ad = fabsf(diff);
    if (valid && qd == 0) lc_acc += (ad < 1.f) ? 0.5f * ad * ad : (ad - 0.5f);
    const float dv = q.inv_b * (diff < -1.f ? -1.f : (diff > 1.f ? 1.f : diff));
    if (valid && qd == 0) q.dzc[j] = dv;
    float4 *gcrow = reinterpret_cast<float4 *>(q.gc + static_cast<int64_t>(j) * D);
    const float dvb = rb(dv, q.bf16);
#pragma unroll
    for (int t = 0; t < NJ; ++t) {
      const float4 wv = wc[4 * t + qd];
      if (valid)
        gcrow[4 * t + qd] =
            make_float4(act_backward(dvb * wv.x, h[t].x, q.act), act_backward(dvb * wv.y, h[t].y, q.act),
                        act_backward(dvb * wv.z, h[t].z, q.act), act_backward(dvb * wv.w, h[t].w, q.act));
    }
    if constexpr (FW) {
      // head dW += dz^T H over this pass's 16 rows (dz rows of invalid j are exactly 0 and are
      // skipped anyway); H re-read by columns from L1/L2
      if (qd == 0) dvs[wid][r] = valid ? dv : 0.f;
      __threadfence_block();
      const int nrow = min(16, r1 - base);
      for (int rr = 0; rr < nrow; ++rr) {
        const int64_t jj = base + rr;
        const float *dzr = dzs + (wid * 16 + rr) * kMaxAct;
        const float dvr = dvs[wid][rr];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int c = lane + 64 * u;
          if (c < 4 * NJ) {
            const float4 ha4 = rb4(reinterpret_cast<const float4 *>(q.ha + jj * D)[c], q.bf16);
            const float4 hc4 = rb4(reinterpret_cast<const float4 *>(q.hc + jj * D)[c], q.bf16);
#pragma unroll
            for (int a = 0; a < AF; ++a) {
              if (a < A) {
                const float dz = rb(dzr[a], q.bf16);
                wa_acc[u][a].x = fmaf(dz, ha4.x, wa_acc[u][a].x);
                wa_acc[u][a].y = fmaf(dz, ha4.y, wa_acc[u][a].y);
                wa_acc[u][a].z = fmaf(dz, ha4.z, wa_acc[u][a].z);
                wa_acc[u][a].w = fmaf(dz, ha4.w, wa_acc[u][a].w);
              }
            }
            const float dvrb = rb(dvr, q.bf16);
            wc_acc[u].x = fmaf(dvrb, hc4.x, wc_acc[u].x);
            wc_acc[u].y = fmaf(dvrb, hc4.y, wc_acc[u].y);
            wc_acc[u].z = fmaf(dvrb, hc4.z, wc_acc[u].z);
            wc_acc[u].w = fmaf(dvrb, hc4.w, wc_acc[u].w);
          }
        }
        if (lane < A) b_acc += dzr[lane];
        else if (lane == A) b_acc += dvr;
      }
    }
  }
  if constexpr (FW) {
    // combine the 4 waves' partials in wave order through LDS (the staged head weights and the
    // log-prob scratch are dead now), then one coalesced partial per block
    __syncthreads();
    float *acc_sh = wsh;   // (A + 1) x D
    float *bias_sh = lps;  // A + 1
    for (int w = 0; w < 4; ++w) {
      if (wid == w) {
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int c = lane + 64 * u;
          if (c < 4 * NJ) {
#pragma unroll
            for (int a = 0; a <= AF; ++a) {
              if (a <= A) {
                const float4 v = (a == A || a == AF) ? wc_acc[u] : wa_acc[u][a < AF ? a : 0];
                float4 *dst = reinterpret_cast<float4 *>(acc_sh + a * D) + c;
                if (w == 0) {
                  *dst = v;
                } else {
                  const float4 o = *dst;
                  *dst = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
                }
              }
            }
          }
        }
        if (lane <= A) bias_sh[lane] = (w == 0) ? b_acc : bias_sh[lane] + b_acc;
      }
      __syncthreads();
    }
    float *dst = q.hw_part + static_cast<int64_t>(blockIdx.x) * q.hw_stride;
    for (int i = tid; i < A * D / 4; i += 256)
      reinterpret_cast<float4 *>(dst)[i] = reinterpret_cast<const float4 *>(acc_sh)[i];
    for (int i = tid; i < D / 4; i += 256)
      reinterpret_cast<float4 *>(dst + q.off_wc)[i] =
          reinterpret_cast<const float4 *>(acc_sh + A * D)[i];
    if (tid < A && q.ba) dst[q.off_ba + tid] = bias_sh[tid];
    if (tid == 0) dst[q.off_bc] = bias_sh[A];
  }
  // ---- fixed-order reductions: over the 16 rows of the wave (lane bits 2..5), then waves 0..3
#pragma unroll
  for (int k = 0; k < KA; ++k)
#pragma unroll
    for (int off = 4; off < 64; off <<= 1) ls_acc[k] += __shfl_xor(ls_acc[k], off, 64);
#pragma unroll
  for (int off = 4; off < 64; off <<= 1) {
    la_acc += __shfl_xor(la_acc, off, 64);
    lc_acc += __shfl_xor(lc_acc, off, 64);
  }
  if (r == 0) {
#pragma unroll
    for (int k = 0; k < KA; ++k)
      if (4 * k + qd < A) red[wid][4 * k + qd] = ls_acc[k];
    if (qd == 0) {
      red[wid][kMaxAct] = la_acc;
      red[wid][kMaxAct + 1] = lc_acc;
    }
  }
  __syncthreads();
  if (tid < A)
    q.logstd_part[static_cast<int64_t>(blockIdx.x) * A + tid] =
        ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
  if (tid == 0) {
    q.loss_part[2 * blockIdx.x] = ((red[0][kMaxAct] + red[1][kMaxAct]) + red[2][kMaxAct]) +
                                  red[3][kMaxAct];
    q.loss_part[2 * blockIdx.x + 1] =
        ((red[0][kMaxAct + 1] + red[1][kMaxAct + 1]) + red[2][kMaxAct + 1]) + red[3][kMaxAct + 1];
  }
}

// Generic head (any widths): one wave per row.  Gradients follow torch's autograd formulas:
// minimum() splits a tie's gradient in halves, clamp passes it on the closed interval,
// huber_loss_backward clips at +-delta, tanh backward is grad*(1-y*y).
template <int HPL>
__global__ __launch_bounds__(256) void update_head_kernel(UpdateHeadArgs q) {
  __shared__ float red[4][kMaxAct + 2];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int count = q.rows_n ? *q.rows_n : q.rows_max;
  const int r0 = static_cast<int>((static_cast<int64_t>(blockIdx.x) * count) / q.splits);
  const int r1 = static_cast<int>((static_cast<int64_t>(blockIdx.x + 1) * count) / q.splits);
  const int A = q.act_dim;
  float lsacc = 0.f;                 // lane a: d loss / d logstd_a over this wave's rows
  float la_acc = 0.f, lc_acc = 0.f;  // lane 0: loss sums
  for (int j = r0 + wid; j < r1; j += 4) {
    const int64_t sr = q.rows[j];
    // ---------------- actor ----------------
    float h[HPL];
    const float *hr = q.ha + static_cast<int64_t>(j) * q.da;
#pragma unroll
    for (int t = 0; t < HPL; ++t) {
      const int k = lane + 64 * t;
      h[t] = (k < q.da) ? hr[k] : 0.f;
    }
    float my_z = 0.f;
    for (int a = 0; a < A; ++a) {
      const float *w = q.wa + static_cast<int64_t>(a) * q.da;
      float part = 0.f;
#pragma unroll
      for (int t = 0; t < HPL; ++t) {
        const int k = lane + 64 * t;
        if (k < q.da) part = fmaf(rb(h[t], q.bf16), rb(w[k], q.bf16), part);
      }
      const float z = wave_sum(part);
      if (lane == a) my_z = z;
    }
    float lp = 0.f, y = 0.f, d = 0.f, var = 1.f;
    if (lane < A) {
      const float z = q.ba ? my_z + q.ba[lane] : my_z;
      y = tanhf(z);
      const float mu = q.omv * y;
      const float sd = expf(q.logstd[lane]);
      const float x = q.actions[sr * A + lane];
      d = x - mu;
      var = sd * sd;
      lp = ((-(d * d)) / (2.f * var) - logf(sd)) - kLogSqrt2Pi;
    }
    float logp = 0.f;
    for (int a = 0; a < A; ++a) logp += __shfl(lp, a, 64);
    const float ratio = expf(logp - q.old_logp[sr]);
    const float adv = q.adv[sr];
    const float s1 = ratio * adv;
    const float cl = ratio < q.clip_lo ? q.clip_lo : (ratio > q.clip_hi ? q.clip_hi : ratio);
    const float s2 = cl * adv;
    const float mn = (s1 != s1 || s2 != s2) ? (s1 + s2) : (s2 < s1 ? s2 : s1);
    const float g = -q.inv_b;
    const float g1 = (s1 < s2) ? g : (s1 == s2 ? g * 0.5f : 0.f);
    const float g2 = (s2 < s1) ? g : (s1 == s2 ? g * 0.5f : 0.f);
    const bool inside = (ratio >= q.clip_lo) && (ratio <= q.clip_hi);
    const float dratio = g1 * adv + (inside ? g2 * adv : 0.f);
    const float dlogp = dratio * ratio;
    float dz = 0.f;
    if (lane < A) {
      const float dmu = dlogp * (d / var);
      dz = (dmu * q.omv) * (1.f - y * y);
      lsacc += dlogp * ((d * d) / var - 1.f) - q.ent_coef * q.inv_ba;
      q.dza[static_cast<int64_t>(j) * A + lane] = dz;
    }
    if (lane == 0) la_acc += mn;
    // dH_L(actor) = (dz . W_head) * act'(h)
    float *gr = q.ga + static_cast<int64_t>(j) * q.da;
#pragma unroll
    for (int t = 0; t < HPL; ++t) {
      const int k = lane + 64 * t;
      if (k < q.da) {
        float s = 0.f;
        for (int a = 0; a < A; ++a)
          s = fmaf(rb(__shfl(dz, a, 64), q.bf16), rb(q.wa[static_cast<int64_t>(a) * q.da + k], q.bf16), s);
        gr[k] = act_backward(s, h[t], q.act);
      }
    }
    // ---------------- critic ----------------
    const float *cr = q.hc + static_cast<int64_t>(j) * q.dc;
#pragma unroll
    for (int t = 0; t < HPL; ++t) {
      const int k = lane + 64 * t;
      h[t] = (k < q.dc) ? cr[k] : 0.f;
    }
    float part = 0.f;
#pragma unroll
    for (int t = 0; t < HPL; ++t) {
      const int k = lane + 64 * t;
      if (k < q.dc) part = fmaf(rb(h[t], q.bf16), rb(q.wc[k], q.bf16), part);
    }
    float v = wave_sum(part);
    if (q.bc) v = v + q.bc[0];
    const float diff = v - q.vtarget[sr];
    const float ad = fabsf(diff);
    if (lane == 0) lc_acc += (ad < 1.f) ? 0.5f * ad * ad : (ad - 0.5f);
    const float dv = q.inv_b * (diff < -1.f ? -1.f : (diff > 1.f ? 1.f : diff));
    if (lane == 0) q.dzc[j] = dv;
    float *gc = q.gc + static_cast<int64_t>(j) * q.dc;
#pragma unroll
    for (int t = 0; t < HPL; ++t) {
      const int k = lane + 64 * t;
      if (k < q.dc) gc[k] = act_backward(rb(dv, q.bf16) * rb(q.wc[k], q.bf16), h[t], q.act);
    }
  }
  // fixed-order block reduction: waves 0..3
  if (lane < A) red[wid][lane] = lsacc;
  if (lane == 0) {
    red[wid][kMaxAct] = la_acc;
    red[wid][kMaxAct + 1] = lc_acc;
  }
  __syncthreads();
  if (threadIdx.x < A) {
    const float s = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) +
                    red[3][threadIdx.x];
    q.logstd_part[static_cast<int64_t>(blockIdx.x) * A + threadIdx.x] = s;
  }
  if (threadIdx.x == 0) {
    q.loss_part[2 * blockIdx.x] = ((red[0][kMaxAct] + red[1][kMaxAct]) + red[2][kMaxAct]) +
                                  red[3][kMaxAct];
    q.loss_part[2 * blockIdx.x + 1] =
        ((red[0][kMaxAct + 1] + red[1][kMaxAct + 1]) + red[2][kMaxAct + 1]) + red[3][kMaxAct + 1];
  }
}

// ============================================================================================
// Minibatch state gather: xg[j][0:din] = states[rows[j]][:], zero padded to ldx (16-B rows), so
// both layer-1 GEMMs (forward and weight-gradient) stream one contiguous, vector-loadable buffer
// instead of re-gathering 68-B rows element by element.
// ============================================================================================
__global__ void gather_states_kernel(const float *__restrict__ states, const int32_t *__restrict__ rows,
                                     const int32_t *__restrict__ rows_n, int b, int din, int ldx,
                                     float *__restrict__ xg) {
  const int count = rows_n ? *rows_n : b;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= static_cast<int64_t>(count) * ldx) return;
  const int j = static_cast<int>(i / ldx), c = static_cast<int>(i % ldx);
  xg[i] = (c < din) ? states[static_cast<int64_t>(rows[j]) * din + c] : 0.f;
}

// ============================================================================================
// Split-K reduction of the slabs into the flat gradient + loss scalars
// ============================================================================================
__global__ __launch_bounds__(kRedThreads) void reduce_slabs_kernel(ReduceArgs q) {
  (void)reduce_slab_block(q, blockIdx.x);
}

// ============================================================================================
// Context
// ============================================================================================
// ============================================================================================
// Per-launch timing (timing.h): event pairs on each dispatch packet while enabled (bench.py's
// live roofline), read back after the timed region.
// ============================================================================================
static const char *const kClassNames[KC_COUNT] = {
    "gemm_fwd",     "gemm_dgrad", "gemm_wgrad", "update_head", "policy_head", "reduce_slabs",
    "gather_states", "gae",       "adam",       "normalize_rows", "obs", "minibatch_rows",
    "env_harness", "fused_update", "lstm", "conv"};

thread_local Timing *g_tim = nullptr;
Timing *g_free_tim = nullptr;

const char *intern_name(const char *fmt, ...) {
  static std::mutex mu;
  static std::deque<std::string> names;
  char buf[160];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  std::lock_guard<std::mutex> lock(mu);
  for (const std::string &s : names)
    if (s == buf) return s.c_str();
  names.emplace_back(buf);
  return names.back().c_str();
}

}  // namespace ppo


namespace ppo {

struct TimingScope {  // routes this thread's launches to ctx->tim while timing is enabled
  explicit TimingScope(ppo_ctx *ctx) { g_tim = ctx->tim.on ? &ctx->tim : nullptr; }
  ~TimingScope() { g_tim = nullptr; }
};

constexpr int kSlabSplits = 64;
constexpr int64_t kParamAlign = 16;  // floats: every flat tensor starts 64-B aligned
constexpr int64_t kWsAlign = 64;     // floats: workspace buffers start 256-B aligned

static inline int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }
constexpr int kHeadSplits = 512;

static int hpl_for(int width) {
  if (width <= 256) return 4;
  if (width <= 512) return 8;
  return 16;
}

// Forward through the hidden layers of the requested nets.  x: (rows, in) f32 with optional
// row gather.  Nets whose layer-l shapes agree share one launch.
static int forward_hidden(ppo_ctx *ctx, const bool use[2], const float *x, const int32_t *x_rows,
                          int rows, const int32_t *rows_n, hipStream_t st, int ldx) {
  const int max_l = std::max(use[0] ? ctx->net[0].n_hidden : 0, use[1] ? ctx->net[1].n_hidden : 0);
  for (int l = 0; l < max_l; ++l) {
    GemmBatch gb{};
    gb.prec = ctx->prec;
    gb.k = 0;
    gb.rows_n = rows_n;
    gb.act = ctx->cfg.activation;
    int np = 0, max_n = 0;
    int kdim = -1;
    for (int z = 0; z < 2; ++z) {
      const NetDesc &nd = ctx->net[z];
      if (!use[z] || l >= nd.n_hidden) continue;
      const LayerDesc &L = nd.layer[l];
      if (kdim >= 0 && kdim != L.in) {  // shapes differ: flush what we have
        int rc = gemm_rows_fwd_nk(gb, np, rows, max_n, st);
        if (rc) return rc;
        np = 0;
        max_n = 0;
      }
      kdim = L.in;
      GemmProblem &P = gb.p[np++];
      P.a = (l == 0) ? x : nd.h[l - 1];
      P.lda = (l == 0) ? ldx : nd.layer[l - 1].out;
      P.b = ctx->params + L.w_off;
      P.ldb = L.in;
      P.c = nd.h[l];
      P.ldc = L.out;
      P.bias = L.b_off >= 0 ? ctx->params + L.b_off : nullptr;
      P.m = rows;
      P.n = L.out;
      gb.k = L.in;
      max_n = std::max(max_n, L.out);
    }
    if (np) {
      int rc = gemm_rows_fwd_nk(gb, np, rows, max_n, st);
      if (rc) return rc;
    }
  }
  return 0;
}

static const int g_fused_enabled = env_knob("PPO_FUSED", 1);
// PPO_FUSED_DIRECT=0: the 8-wave fused update reads the gathered xb / srow copies (written by the
// prep kernel or the previous step tail) instead of the staged records through the row indices
// (the ctx default; ppo_ctx_fused_direct switches it)
static const int g_fused_direct = env_knob("PPO_FUSED_DIRECT", 1);

// Pointers of both nets for the fused kernels (bf16 images from ctx->fw, f32 masters in params).
static void fused_nets(const ppo_ctx *ctx, FusedNet (&out)[2]) {
  for (int z = 0; z < 2; ++z) {
    const NetDesc &nd = ctx->net[z];
    FusedNet &fn = out[z];
    fn.w0b = ctx->fw[z][0];
    fn.w1b = ctx->fw[z][1];
    fn.w1bt = ctx->fw[z][2];
    fn.w0 = ctx->params + nd.layer[0].w_off;
    fn.w1 = ctx->params + nd.layer[1].w_off;
    fn.b0 = nd.layer[0].b_off >= 0 ? ctx->params + nd.layer[0].b_off : nullptr;
    fn.b1 = nd.layer[1].b_off >= 0 ? ctx->params + nd.layer[1].b_off : nullptr;
    fn.wh = ctx->params + nd.layer[2].w_off;
    fn.bh = nd.layer[2].b_off >= 0 ? ctx->params + nd.layer[2].b_off : nullptr;
    fn.off_w0 = nd.layer[0].w_off;
    fn.off_b0 = nd.layer[0].b_off;
    fn.off_w1 = nd.layer[1].w_off;
    fn.off_b1 = nd.layer[1].b_off;
    fn.off_wh = nd.layer[2].w_off;
    fn.off_bh = nd.layer[2].b_off;
  }
}

static bool fused_active(const ppo_ctx *ctx) {
  return ctx->prec == PPO_PREC_BF16 && ctx->fused_ok && g_fused_enabled;
}

// Precision bf16 with supported shapes: gather + bf16 weight refresh, the persistent fused
// forward/loss/backward kernel (one partial-gradient slab per workgroup), then the fixed-order
// slab reduction.  Same contract as the layered path below.
static FusedArgs fused_args(ppo_ctx *ctx, const float *states_d, const float *actions_d,
                            const float *old_logp_d, const float *adv_d, const float *vtarget_d,
                            const int32_t *rows_d, int b, const int32_t *count_d, float clip_lo,
                            float clip_hi, float entropy_coef, float inv_b, float inv_ba,
                            bool staged, bool pack_w) {
  FusedArgs q{};
  fused_nets(ctx, q.net);
  q.logstd = ctx->params + ctx->net[0].logstd_off;
  q.off_logstd = ctx->net[0].logstd_off;
  q.xb = ctx->fxb;
  q.srow = ctx->fsrow;
  q.states = states_d;
  q.actions = actions_d;
  q.old_logp = old_logp_d;
  q.adv = adv_d;
  q.vtarget = vtarget_d;
  q.rows = rows_d;
  q.rows_n = count_d;
  q.rec = staged ? ctx->frec : nullptr;
  q.n_rec = staged ? ctx->frec_rows : 0;
  q.pack_w = pack_w;
  q.b = b;
  q.din = ctx->cfg.obs_dim * ctx->cfg.window;
  q.act_dim = ctx->cfg.act_dim;
  q.act = ctx->cfg.activation;
  q.hidden = ctx->fused_hidden;
  q.omv = ctx->cfg.output_max_value;
  q.clip_lo = clip_lo;
  q.clip_hi = clip_hi;
  q.ent_coef = entropy_coef;
  q.inv_b = inv_b;
  q.inv_ba = inv_ba;
  q.slabs = ctx->fslabs;
  q.slab_stride = ctx->total_params;
  q.loss_part = ctx->floss;
  q.stamps = ctx->fstamp_on ? ctx->fstamps : nullptr;
  q.G = std::min(kFusedMaxWG, ceil_div(b, kFusedRows));
  q.direct = staged && ctx->fdirect;
  return q;
}

// gather (q.b rows; 0 = none) and, with q.pack_w, the weight-image refresh
static int fused_prep(const ppo_ctx *ctx, const FusedArgs &q, hipStream_t st) {
  const double H = ctx->fused_hidden;
  const int din = q.din, A = q.act_dim;
  // algorithmic traffic: gather (row index, din + A + 3 floats -- or one 128 B record -- in;
  // 64 + 64 B out per row) and weight images (f32 in, 3 bf16 images out per net)
  const double wbytes =
      q.pack_w ? 2.0 * (4.0 * H * (din + H) + 2.0 * H * (kFusedKX + 2.0 * H)) : 0.0;
  const double in_row = q.rec ? 4.0 + kRecordBytes : 4.0 * (1 + din + A + 3);
  const TimRec rec{KC_GATHER, "fused_prep_kernel", 0.0,
                   static_cast<double>(q.b) * (in_row + 2.0 * kFusedKX + 4.0 * kFusedSP) + wbytes};
  return fused_prep_launch(q, rec, st);
}

// The gathered-copy record (ctx.h fg_rows): a caller's PPO_STAGED_ROWS_GATHERED is a promise
// about stream order that nothing on the device checks, so the host keeps which rows the last
// staged gather wrote and gathers again when the promise names other rows.  The check is POINTER
// identity (the index buffer's address and count), not content: a caller that rewrites the same
// index buffer in place (e.g. a fresh permutation into one buffer) must not pass
// PPO_STAGED_ROWS_GATHERED for it.  A gather is recorded only once its launch was issued
// successfully; a failed entry point clears the record.
static bool gathered_holds(const ppo_ctx *ctx, const int32_t *rows_d, int b) {
  return rows_d != nullptr && ctx->fg_rows == rows_d && ctx->fg_b == b;
}
static void note_gathered(ppo_ctx *ctx, const int32_t *rows_d, int b) {
  ctx->fg_rows = rows_d;
  ctx->fg_b = rows_d ? b : 0;
}

static int fused_forward_backward(ppo_ctx *ctx, const FusedArgs &q, hipStream_t st) {
  const int H = ctx->fused_hidden, din = q.din, A = q.act_dim, b = q.b;
  const int64_t P = ctx->total_params;
  ctx->fstamp_g = q.G;
  // FLOPs per row per net: forward (din*H + H*H + a*H), dgrad (H*H + a*H), wgrad (din*H +
  // H*H + a*H), a = A (actor) / 1 (critic); bytes: staged rows + one slab per workgroup
  double fl = 0.0;
  for (int z = 0; z < 2; ++z) {
    const double a = z == 0 ? A : 1;
    fl += 2.0 * b * ((din * H + H * H + a * H) + (H * H + a * H) + (din * H + H * H + a * H));
  }
  // HBM bytes: the staged rows once, the bf16 weight images once (every workgroup re-reads
  // them from L2, which is not HBM traffic) and one partial-gradient slab per workgroup
  const double by = static_cast<double>(b) * (2.0 * kFusedKX + 4.0 * kFusedSP) +
                    4.0 * q.G * static_cast<double>(P) + 2.0 * 2.0 * H * (kFusedKX + 2.0 * H);
  const int na = A <= 2 ? 2 : A <= 4 ? 4 : A <= 6 ? 6 : 8;
  const TimRec rec{KC_FUSED,
                   tim_active() ? intern_name("fused_update_kernel<%d, %d, %d, false, %d>", H, q.act, na,
                                              fused_sched(q.act))
                                : nullptr,
                   fl, by};
  return fused_update_launch(q, rec, st);
}

static ReduceArgs fused_reduce_args(const ppo_ctx *ctx, const FusedArgs &q, float *grad_d,
                                    float *loss_d) {
  const int A = q.act_dim;
  const int64_t P = ctx->total_params;
  ReduceArgs r{};
  int ns = 0;
  for (int z = 0; z < 2; ++z) {
    const NetDesc &nd = ctx->net[z];
    auto seg = [&](int64_t off, int64_t len) {
      ReduceSeg &g = r.seg[ns++];
      g.dst = off;
      g.len = len;
      g.src = ctx->fslabs + off;
      g.stride = P;
      g.nsplit = q.G;
    };
    if (z == 0) seg(nd.logstd_off, A);
    for (int l = 0; l <= nd.n_hidden; ++l) {
      const LayerDesc &L = nd.layer[l];
      seg(L.w_off, static_cast<int64_t>(L.out) * L.in);
      if (L.b_off >= 0) seg(L.b_off, L.out);
    }
  }
  r.nseg = ns;
  r.total = P;
  r.grad = grad_d;
  r.loss_part = ctx->floss;
  r.loss_splits = q.G;
  r.inv_b = q.inv_b;
  r.logstd = ctx->params + ctx->net[0].logstd_off;
  r.act_dim = A;
  r.ent_coef = q.ent_coef * ctx->ent_log_share;
  r.loss_out = loss_d;
  return r;
}

static int fused_minibatch_grad(ppo_ctx *ctx, const float *states_d, const float *actions_d,
                                const float *old_logp_d, const float *adv_d,
                                const float *vtarget_d, const int32_t *rows_d, int b,
                                const int32_t *count_d, float clip_lo, float clip_hi,
                                float entropy_coef, float inv_b, float inv_ba, float *grad_d,
                                float *loss_d, hipStream_t st, bool staged = false,
                                bool pack_w = true, bool gathered = false) {
  const FusedArgs q = fused_args(ctx, states_d, actions_d, old_logp_d, adv_d, vtarget_d, rows_d,
                                 b, count_d, clip_lo, clip_hi, entropy_coef, inv_b, inv_ba,
                                 staged, pack_w);
  gathered = gathered && staged && gathered_holds(ctx, rows_d, b);
  if ((!gathered && !q.direct) || pack_w) {
    FusedArgs p = q;
    p.b = (gathered || q.direct) ? 0 : b;
    if (int rc = fused_prep(ctx, p, st)) return rc;
    if (p.b > 0) note_gathered(ctx, staged && count_d == nullptr ? rows_d : nullptr, b);
  }
  const ReduceArgs r = fused_reduce_args(ctx, q, grad_d, loss_d);
  if (int rc = fused_forward_backward(ctx, q, st)) return rc;
  const int64_t P = ctx->total_params;
  launch_k(TimRec{KC_REDUCE, "reduce_slabs_kernel", static_cast<double>(q.G) * P,
                  4.0 * (static_cast<double>(q.G) + 1) * P},
           reduce_slabs_kernel, dim3(ceil_div(P, kRedParams)), dim3(kRedThreads), 0, st, r);
  PPO_LAUNCHED();
  return 0;
}

// AdamPackArgs for the ctx's bound parameters (both nets) and the fused weight images
static AdamPackArgs adam_pack_args(const ppo_ctx *ctx, const float *g_d, float *m_d, float *v_d,
                                   const float *sched_d, float neg_a, float neg_c, float bc2,
                                   float omb1, float b2, float omb2, float eps) {
  AdamPackArgs a{};
  a.p = ctx->params;
  a.g = g_d;
  a.m = m_d;
  a.v = v_d;
  a.n = ctx->total_params;
  a.n_actor = ctx->net[0].count;
  a.sched = sched_d;
  a.neg_a = neg_a;
  a.neg_c = neg_c;
  a.bc2 = bc2;
  a.w1 = omb1;
  a.b2 = b2;
  a.omb2 = omb2;
  a.eps = eps;
  FusedNet nets[2];
  fused_nets(ctx, nets);
  for (int z = 0; z < 2; ++z) {
    a.w0b[z] = const_cast<__bf16 *>(nets[z].w0b);
    a.w1b[z] = const_cast<__bf16 *>(nets[z].w1b);
    a.w1bt[z] = const_cast<__bf16 *>(nets[z].w1bt);
    a.off_w0[z] = nets[z].off_w0;
    a.off_w1[z] = nets[z].off_w1;
  }
  a.din = ctx->cfg.obs_dim * ctx->cfg.window;
  a.H = ctx->fused_hidden;
  return a;
}

static int check_ctx(const ppo_ctx *ctx) {
  PPO_REQUIRE(ctx != nullptr, "null ppo_ctx");
  PPO_REQUIRE(ctx->params != nullptr, "ppo_ctx: parameters not bound (ppo_bind_params)");
  return 0;
}

}  // namespace ppo

using namespace ppo;

extern "C" int ppo_ctx_create(const ppo_net_cfg *cfg, int device, ppo_ctx **out) {
  PPO_REQUIRE(cfg && out, "ppo_ctx_create: null argument");
  PPO_REQUIRE(cfg->obs_dim > 0 && cfg->window > 0, "ppo_ctx_create: bad obs/window");
  PPO_REQUIRE(cfg->act_dim > 0 && cfg->act_dim <= kMaxAct, "ppo_ctx_create: act_dim must be in [1, %d]",
              kMaxAct);
  PPO_REQUIRE(cfg->n_actor_hidden >= 1 && cfg->n_actor_hidden <= PPO_MAX_LAYERS &&
                  cfg->n_critic_hidden >= 1 && cfg->n_critic_hidden <= PPO_MAX_LAYERS,
              "ppo_ctx_create: hidden layer count must be in [1, %d]", PPO_MAX_LAYERS);
  PPO_REQUIRE(cfg->activation >= PPO_ACT_RELU && cfg->activation <= PPO_ACT_ELU,
              "ppo_ctx_create: unknown activation %d", cfg->activation);
  PPO_REQUIRE(cfg->max_rows > 0, "ppo_ctx_create: max_rows must be positive");
  PPO_HIP_TRY(hipSetDevice(device));
  ppo_ctx *ctx = new (std::nothrow) ppo_ctx();
  PPO_REQUIRE(ctx != nullptr, "ppo_ctx_create: out of host memory");
  ctx->cfg = *cfg;
  ctx->device = device;
  ctx->ent_log_share = 1.f;
  const int din = cfg->obs_dim * cfg->window;
  int64_t off = 0;
  int64_t ws_floats = 0;
  const int64_t R = cfg->max_rows;
  for (int z = 0; z < 2; ++z) {
    NetDesc &nd = ctx->net[z];
    nd.begin = off;
    const int nh = z == 0 ? cfg->n_actor_hidden : cfg->n_critic_hidden;
    const int32_t *hid = z == 0 ? cfg->actor_hidden : cfg->critic_hidden;
    const bool bias = z == 0 ? cfg->actor_use_bias != 0 : true;
    nd.n_hidden = nh;
    if (z == 0) {
      nd.logstd_off = off;
      off = align_up(off + cfg->act_dim, kParamAlign);
    } else {
      nd.logstd_off = -1;
    }
    int width = din;
    for (int l = 0; l <= nh; ++l) {
      const int o = (l < nh) ? hid[l] : (z == 0 ? cfg->act_dim : 1);
      if (l < nh && (o <= 0 || o > 1024)) {
        delete ctx;
        set_error("ppo_ctx_create: hidden width %d out of range [1, 1024]", o);
        return PPO_EINVAL;
      }
      LayerDesc &L = nd.layer[l];
      L.in = width;
      L.out = o;
      L.w_off = off;
      off = align_up(off + static_cast<int64_t>(o) * width, kParamAlign);
      L.b_off = bias ? off : -1;
      if (bias) off = align_up(off + o, kParamAlign);
      if (l < nh) ws_floats += align_up(R * o, kWsAlign);
      width = o;
    }
    ws_floats += align_up(R * nd.layer[nh].in, kWsAlign);   // g = dH_L (last hidden width)
    ws_floats += align_up(R * nd.layer[nh].out, kWsAlign);  // dz
    nd.count = off - nd.begin;
  }
  ctx->total_params = off;
  ws_floats += align_up(static_cast<int64_t>(kSlabSplits) * off, kWsAlign);
  ws_floats += align_up(static_cast<int64_t>(kHeadSplits) * (cfg->act_dim + 2), kWsAlign);
  {
    const int A = cfg->act_dim;
    const int da = ctx->net[0].layer[ctx->net[0].n_hidden].in;
    const int dc = ctx->net[1].layer[ctx->net[1].n_hidden].in;
    ctx->hw_off_ba = static_cast<int>(align_up(static_cast<int64_t>(A) * da, 4));
    ctx->hw_off_wc = ctx->hw_off_ba + static_cast<int>(align_up(A, 4));
    ctx->hw_off_bc = ctx->hw_off_wc + static_cast<int>(align_up(dc, 4));
    ctx->hw_stride = ctx->hw_off_bc + 4;
  }
  ws_floats += align_up(static_cast<int64_t>(kHeadSplits) * ctx->hw_stride, kWsAlign);
  const int ldx = static_cast<int>(align_up(din, 4));
  ws_floats += align_up(R * ldx, kWsAlign);
  void *arena = nullptr;
  hipError_t e = hipMalloc(&arena, ws_floats * sizeof(float) + 256);
  if (e != hipSuccess) {
    delete ctx;
    set_error("ppo_ctx_create: hipMalloc(%zu bytes) failed: %s", ws_floats * sizeof(float),
              hipGetErrorString(e));
    return PPO_EHIP;
  }
  ctx->arena = arena;
  float *p = static_cast<float *>(arena);
  for (int z = 0; z < 2; ++z) {
    NetDesc &nd = ctx->net[z];
    for (int l = 0; l < nd.n_hidden; ++l) {
      nd.h[l] = p;
      p += align_up(R * nd.layer[l].out, kWsAlign);
    }
    nd.g = p;
    p += align_up(R * nd.layer[nd.n_hidden].in, kWsAlign);
    nd.dz = p;
    p += align_up(R * nd.layer[nd.n_hidden].out, kWsAlign);
  }
  ctx->slabs = p;
  p += align_up(static_cast<int64_t>(kSlabSplits) * off, kWsAlign);
  ctx->head_part = p;
  p += align_up(static_cast<int64_t>(kHeadSplits) * (cfg->act_dim + 2), kWsAlign);
  ctx->head_w_part = p;
  p += align_up(static_cast<int64_t>(kHeadSplits) * ctx->hw_stride, kWsAlign);
  ctx->xg = p;
  ctx->ldx = ldx;
  p += align_up(R * ldx, kWsAlign);
  if (static_cast<int64_t>(p - static_cast<float *>(arena)) != ws_floats) {
    (void)hipFree(arena);
    delete ctx;
    set_error("ppo_ctx_create: internal workspace carve-out mismatch");
    return PPO_EHIP;
  }
  ctx->params = nullptr;
  // fused bf16 update: both nets 2 hidden layers of one compiled width, W*O <= 32, A <= 8
  {
    const NetDesc &na = ctx->net[0], &nc = ctx->net[1];
    const int H = na.layer[0].out;
    ctx->fused_ok = na.n_hidden == 2 && nc.n_hidden == 2 && fused_width_ok(H) &&
                    na.layer[1].out == H && nc.layer[0].out == H && nc.layer[1].out == H &&
                    din <= kFusedKX && cfg->act_dim <= kFusedMaxAct;
    ctx->fused_hidden = H;
    if (ctx->fused_ok) {
      const int64_t wimg = align_up(static_cast<int64_t>(H) * (kFusedKX + 2 * H), 128);
      const int64_t bytes = 2 * wimg * 2 + align_up(R * kFusedKX * 2, 256) +
                            align_up(R * kFusedSP * 4, 256) +
                            static_cast<int64_t>(kFusedMaxWG) * off * 4 + kFusedMaxWG * 2 * 4 + 1024;
      void *fa = nullptr;
      e = hipMalloc(&fa, bytes);
      if (e != hipSuccess) {
        (void)hipFree(arena);
        delete ctx;
        set_error("ppo_ctx_create: hipMalloc(%lld bytes) for the fused workspace failed: %s",
                  static_cast<long long>(bytes), hipGetErrorString(e));
        return PPO_EHIP;
      }
      ctx->farena = fa;
      char *c = static_cast<char *>(fa);
      for (int z = 0; z < 2; ++z) {
        __bf16 *wb = reinterpret_cast<__bf16 *>(c);
        ctx->fw[z][0] = wb;
        ctx->fw[z][1] = wb + static_cast<int64_t>(H) * kFusedKX;
        ctx->fw[z][2] = wb + static_cast<int64_t>(H) * (kFusedKX + H);
        c += wimg * 2;
      }
      ctx->fxb = reinterpret_cast<__bf16 *>(c);
      c += align_up(R * kFusedKX * 2, 256);
      ctx->fsrow = reinterpret_cast<float *>(c);
      c += align_up(R * kFusedSP * 4, 256);
      ctx->fslabs = reinterpret_cast<float *>(c);
      c += static_cast<int64_t>(kFusedMaxWG) * off * 4;
      ctx->floss = reinterpret_cast<float *>(c);
      c += kFusedMaxWG * 2 * 4;
      ctx->fdirect = g_fused_direct != 0;
    }
  }
  *out = ctx;
  return 0;
}

extern "C" int ppo_ctx_destroy(ppo_ctx *ctx) {
  if (!ctx) return 0;
  (void)hipSetDevice(ctx->device);
  if (g_free_tim == &ctx->tim) g_free_tim = nullptr;
  for (int i = 0; i < 2 * ctx->tim.capacity; ++i) (void)hipEventDestroy(ctx->tim.ev[i]);
  delete[] ctx->tim.ev;
  delete[] ctx->tim.cls;
  delete[] ctx->tim.kname;
  delete[] ctx->tim.flops;
  delete[] ctx->tim.bytes;
  if (ctx->arena) (void)hipFree(ctx->arena);
  if (ctx->farena) (void)hipFree(ctx->farena);
  if (ctx->fstamps) (void)hipFree(ctx->fstamps);
  if (ctx->frec) (void)hipFree(ctx->frec);
  wide_free(ctx);
  delete ctx;
  return 0;
}

extern "C" int64_t ppo_param_count(const ppo_ctx *ctx, int net) {
  if (!ctx) return -1;
  if (net == 0 || net == 1) return ctx->net[net].count;
  return ctx->total_params;
}

extern "C" int ppo_param_offsets(const ppo_ctx *ctx, int64_t *offsets, int max_tensors) {
  PPO_REQUIRE(ctx != nullptr, "ppo_param_offsets: null ctx");
  int n = 0;
  auto put = [&](int64_t off) {
    if (offsets && n < max_tensors) offsets[n] = off;
    ++n;
  };
  for (int z = 0; z < 2; ++z) {
    const NetDesc &nd = ctx->net[z];
    if (z == 0) put(nd.logstd_off);
    for (int l = 0; l <= nd.n_hidden; ++l) {
      put(nd.layer[l].w_off);
      if (nd.layer[l].b_off >= 0) put(nd.layer[l].b_off);
    }
  }
  return n;
}

extern "C" int ppo_bind_params(ppo_ctx *ctx, float *params_d) {
  PPO_REQUIRE(ctx && params_d, "ppo_bind_params: null argument");
  ctx->params = params_d;
  return 0;
}

extern "C" int ppo_policy_step(ppo_ctx *ctx, const float *state_d, int n, const float *eps_d,
                               uint64_t seed, uint64_t offset, float *action_d, float *logp_d,
                               float *value_d, float *mean_d, void *stream) {
  if (int rc = check_ctx(ctx)) return rc;
  PPO_REQUIRE(state_d && n > 0, "ppo_policy_step: bad state / n");
  PPO_REQUIRE(n <= ctx->cfg.max_rows, "ppo_policy_step: n=%d exceeds max_rows=%d", n,
              ctx->cfg.max_rows);
  hipStream_t st = as_stream(stream);
  TimingScope timing_scope(ctx);
  if (wide_active(ctx))
    return wide_policy_step(ctx, state_d, n, eps_d, seed, offset, action_d, logp_d, value_d,
                            mean_d, true, st);
  const bool use[2] = {action_d || logp_d || mean_d, value_d != nullptr};
  if (!use[0] && !use[1]) return 0;
  if (int rc = forward_hidden(ctx, use, state_d, nullptr, n, nullptr, st,
                              ctx->cfg.obs_dim * ctx->cfg.window))
    return rc;
  const NetDesc &A = ctx->net[0], &C = ctx->net[1];
  PolicyHeadArgs q{};
  q.n = n;
  q.act_dim = ctx->cfg.act_dim;
  q.omv = ctx->cfg.output_max_value;
  if (use[0]) {
    const LayerDesc &hl = A.layer[A.n_hidden];
    q.ha = A.h[A.n_hidden - 1];
    q.da = hl.in;
    q.wa = ctx->params + hl.w_off;
    q.ba = hl.b_off >= 0 ? ctx->params + hl.b_off : nullptr;
    q.logstd = ctx->params + A.logstd_off;
  }
  if (use[1]) {
    const LayerDesc &hl = C.layer[C.n_hidden];
    q.hc = C.h[C.n_hidden - 1];
    q.dc = hl.in;
    q.wc = ctx->params + hl.w_off;
    q.bc = ctx->params + hl.b_off;
  }
  q.eps = eps_d;
  q.seed = seed;
  q.offset = offset;
  q.offset_base = ctx->rng_counter;
  q.action = action_d;
  q.logp = logp_d;
  q.value = value_d;
  q.mean = mean_d;
  q.bf16 = ctx->prec == PPO_PREC_BF16;
  const int hpl = hpl_for(std::max(q.da, q.dc));
  const int grid = ceil_div(n, 4);
  const int na = q.act_dim;
  const TimRec rec{KC_POLICY_HEAD,
                   tim_active() ? intern_name("policy_head_kernel<%d>", hpl) : nullptr,
                   2.0 * n * (static_cast<double>(q.da) * na + q.dc),
                   4.0 * n * (q.da + q.dc + (eps_d ? na : 0) + (action_d ? na : 0) +
                              (mean_d ? na : 0) + (logp_d ? 1 : 0) + (value_d ? 1 : 0))};
  if (hpl == 4) launch_k(rec, policy_head_kernel<4>, dim3(grid), dim3(256), 0, st, q);
  else if (hpl == 8) launch_k(rec, policy_head_kernel<8>, dim3(grid), dim3(256), 0, st, q);
  else launch_k(rec, policy_head_kernel<16>, dim3(grid), dim3(256), 0, st, q);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_pack_weights(ppo_ctx *ctx, void *stream) {
  if (int rc = check_ctx(ctx)) return rc;
  if (wide_active(ctx)) {
    TimingScope timing_scope(ctx);
    return wide_pack(ctx, as_stream(stream));
  }
  if (!fused_active(ctx)) return 0;  // the layered path reads the f32 masters directly
  TimingScope timing_scope(ctx);
  FusedArgs q{};
  fused_nets(ctx, q.net);
  q.b = 0;
  q.pack_w = true;
  q.din = ctx->cfg.obs_dim * ctx->cfg.window;
  q.hidden = ctx->fused_hidden;
  const double H = ctx->fused_hidden;
  const TimRec rec{KC_GATHER, "fused_prep_kernel", 0.0,
                   2.0 * (4.0 * H * (q.din + H) + 2.0 * H * (kFusedKX + 2.0 * H))};
  return fused_prep_launch(q, rec, as_stream(stream));
}

extern "C" int ppo_ctx_fused_active(const ppo_ctx *ctx) {
  return (ctx && fused_active(ctx)) ? 1 : 0;
}

// The ctx's record buffer grown to n_rows (outside a graph capture: the first call per size).
static int ensure_records(ppo_ctx *ctx, int64_t n_rows, hipStream_t st, const char *who) {
  if (n_rows > ctx->frec_cap) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    PPO_REQUIRE(hipStreamIsCapturing(st, &cap) == hipSuccess &&
                    cap == hipStreamCaptureStatusNone,
                "%s: first call for %lld rows inside a graph capture", who,
                static_cast<long long>(n_rows));
    (void)hipStreamSynchronize(st);
    if (ctx->frec) (void)hipFree(ctx->frec);
    ctx->frec = nullptr;
    ctx->frec_cap = 0;
    void *p = nullptr;
    const hipError_t e = hipMalloc(&p, static_cast<size_t>(n_rows) * kRecordBytes);
    PPO_REQUIRE(e == hipSuccess, "%s: hipMalloc(%lld records): %s", who,
                static_cast<long long>(n_rows), hipGetErrorString(e));
    ctx->frec = static_cast<uint4 *>(p);
    ctx->frec_cap = n_rows;
  }
  ctx->frec_rows = n_rows;
  return 0;
}

extern "C" int ppo_stage_records(ppo_ctx *ctx, const float *states_d, const float *actions_d,
                                 const float *old_logp_d, const float *adv_d,
                                 const float *vtarget_d, int64_t n_rows, void *stream) {
  if (int rc = check_ctx(ctx)) return rc;
  PPO_REQUIRE(fused_active(ctx), "ppo_stage_records: needs the fused bf16 path "
                                 "(ppo_ctx_fused_active)");
  note_gathered(ctx, nullptr, 0);  // new records: any gathered copy is stale
  PPO_REQUIRE(states_d && actions_d && old_logp_d && adv_d && vtarget_d && n_rows > 0,
              "ppo_stage_records: null buffer or n_rows <= 0");
  hipStream_t st = as_stream(stream);
  if (int rc = ensure_records(ctx, n_rows, st, "ppo_stage_records")) return rc;
  TimingScope timing_scope(ctx);
  const int din = ctx->cfg.obs_dim * ctx->cfg.window, A = ctx->cfg.act_dim;
  const TimRec rec{KC_GATHER, "fused_records_kernel", 0.0,
                   static_cast<double>(n_rows) * (4.0 * (din + A + 3) + kRecordBytes)};
  return fused_records_launch(ctx->frec, states_d, actions_d, old_logp_d, adv_d, vtarget_d,
                              n_rows, din, A, rec, st);
}

extern "C" int ppo_gae_stage_records(ppo_ctx *ctx, const float *value_d,
                                     const float *next_value_d, const void *reward_d,
                                     int reward_is_f64, const uint8_t *done_d,
                                     const uint8_t *terminated_d, int force_last_done, int n,
                                     int t, double gamma, double lmbda, float *adv_d,
                                     float *vtarget_d, const float *states_d,
                                     const float *actions_d, const float *old_logp_d,
                                     void *stream) {
  if (int rc = check_ctx(ctx)) return rc;
  PPO_REQUIRE(fused_active(ctx), "ppo_gae_stage_records: needs the fused bf16 path "
                                 "(ppo_ctx_fused_active)");
  note_gathered(ctx, nullptr, 0);  // new records: any gathered copy is stale
  PPO_REQUIRE(value_d && next_value_d && reward_d && terminated_d && adv_d && vtarget_d &&
                  states_d && actions_d && old_logp_d,
              "ppo_gae_stage_records: null buffer");
  PPO_REQUIRE(n > 0 && t > 0, "ppo_gae_stage_records: bad shape n=%d t=%d", n, t);
  const int64_t n_rows = static_cast<int64_t>(n) * t;
  if (t > 16 * 16) {  // beyond the pipelined scan: the two passes
    if (int rc = ppo_gae(value_d, next_value_d, reward_d, reward_is_f64, done_d, terminated_d,
                         force_last_done, n, t, gamma, lmbda, adv_d, vtarget_d, stream))
      return rc;
    return ppo_stage_records(ctx, states_d, actions_d, old_logp_d, adv_d, vtarget_d, n_rows,
                             stream);
  }
  hipStream_t st = as_stream(stream);
  if (int rc = ensure_records(ctx, n_rows, st, "ppo_gae_stage_records")) return rc;
  TimingScope timing_scope(ctx);
  const int din = ctx->cfg.obs_dim * ctx->cfg.window, A = ctx->cfg.act_dim;
  GaeRecordArgs g{};
  g.value = value_d;
  g.next_value = next_value_d;
  g.reward = reward_d;
  g.done = done_d;
  g.term = terminated_d;
  g.force_last = force_last_done;
  g.n = n;
  g.t_len = t;
  g.gamma_f = static_cast<float>(gamma);
  g.lg_f = static_cast<float>(lmbda * gamma);
  g.adv = adv_d;
  g.vtarget = vtarget_d;
  g.states = states_d;
  g.actions = actions_d;
  g.old_logp = old_logp_d;
  g.rec = ctx->frec;
  g.din = din;
  g.act_dim = A;
  // algorithmic bytes: the GAE's (V, V', reward, terminated [+ done] in; adv, vtarget out) plus
  // the record pass's (state, actions, old_logp in; the 128 B record out)
  const double per_row = 4 + 4 + (reward_is_f64 ? 8 : 4) + 1 + (done_d ? 1 : 0) + 4 + 4 +
                         4.0 * (din + A + 1) + kRecordBytes;
  const TimRec rec{KC_GAE, "gae_records_kernel", 0.0, static_cast<double>(n_rows) * per_row};
  return gae_records_launch(g, reward_is_f64 != 0, rec, st);
}

extern "C" int ppo_minibatch_grad_staged(ppo_ctx *ctx, const int32_t *rows_d, int b,
                                         const int32_t *count_d, float clip_lo, float clip_hi,
                                         float entropy_coef, float inv_b, float inv_ba,
                                         float *grad_d, float *loss_d, int flags, void *stream) {
  if (int rc = check_ctx(ctx)) return rc;
  PPO_REQUIRE(fused_active(ctx) && ctx->frec && ctx->frec_rows > 0,
              "ppo_minibatch_grad_staged: no staged records (ppo_stage_records first)");
  PPO_REQUIRE(rows_d && grad_d && loss_d, "ppo_minibatch_grad_staged: null buffer");
  PPO_REQUIRE(b > 0 && b <= ctx->cfg.max_rows,
              "ppo_minibatch_grad_staged: b=%d outside [1, max_rows=%d]", b, ctx->cfg.max_rows);
  PPO_REQUIRE((flags & ~(PPO_STAGED_WEIGHTS_CURRENT | PPO_STAGED_ROWS_GATHERED)) == 0,
              "ppo_minibatch_grad_staged: flags %d", flags);
  PPO_REQUIRE(!(flags & PPO_STAGED_ROWS_GATHERED) || count_d == nullptr,
              "ppo_minibatch_grad_staged: pre-gathered rows take no device count");
  TimingScope timing_scope(ctx);
  return fused_minibatch_grad(ctx, nullptr, nullptr, nullptr, nullptr, nullptr, rows_d, b,
                              count_d, clip_lo, clip_hi, entropy_coef, inv_b, inv_ba, grad_d,
                              loss_d, as_stream(stream), true,
                              (flags & PPO_STAGED_WEIGHTS_CURRENT) == 0,
                              (flags & PPO_STAGED_ROWS_GATHERED) != 0);
}

extern "C" int ppo_adam_pack_gather(ppo_ctx *ctx, const float *g_d, float *m_d, float *v_d,
                                    const float *sched_d, float neg_step_actor,
                                    float neg_step_critic, float bc2_sqrt, float one_minus_beta1,
                                    float beta2, float one_minus_beta2, float eps,
                                    const int32_t *next_rows_d, int next_b, void *stream) {
  if (int rc = check_ctx(ctx)) return rc;
  PPO_REQUIRE(fused_active(ctx) && ctx->frec && ctx->frec_rows > 0,
              "ppo_adam_pack_gather: no staged records (ppo_stage_records first)");
  PPO_REQUIRE(g_d && m_d && v_d, "ppo_adam_pack_gather: null buffer");
  PPO_REQUIRE(next_b >= 0 && next_b <= ctx->cfg.max_rows && (next_b == 0) == (next_rows_d == nullptr),
              "ppo_adam_pack_gather: next_b=%d", next_b);
  TimingScope timing_scope(ctx);
  TailArgs t{};
  t.a = adam_pack_args(ctx, g_d, m_d, v_d, sched_d, neg_step_actor, neg_step_critic, bc2_sqrt,
                       one_minus_beta1, beta2, one_minus_beta2, eps);
  t.rows = next_rows_d;
  t.rec = ctx->frec;
  t.n_rec = ctx->frec_rows;
  t.xb = ctx->fxb;
  t.srow = ctx->fsrow;
  // direct: the next fused launch reads its rows through the indices, nothing to gather
  const bool direct = next_b > 0 && fused_args(ctx, nullptr, nullptr, nullptr, nullptr, nullptr,
                                               next_rows_d, next_b, nullptr, 0.f, 0.f, 0.f, 0.f,
                                               0.f, true, false).direct;
  t.b = direct ? 0 : next_b;
  t.reduce = false;
  ReduceArgs r{};
  r.total = ctx->total_params;
  const double P = static_cast<double>(ctx->total_params), H = ctx->fused_hidden;
  const TimRec rec{KC_ADAM, "step_tail_kernel", 0.0,
                   28.0 * P + 2.0 * 2.0 * H * (t.a.din + 2.0 * H) +
                       static_cast<double>(t.b) * (4.0 + 2.0 * kRecordBytes)};
  if (int rc = step_tail_launch(r, t, rec, as_stream(stream))) {
    note_gathered(ctx, nullptr, 0);
    return rc;
  }
  if (t.b > 0) note_gathered(ctx, next_rows_d, t.b);
  return 0;
}

extern "C" int ppo_gather_staged_rows(ppo_ctx *ctx, const int32_t *rows_d, int b, void *stream) {
  if (int rc = check_ctx(ctx)) return rc;
  PPO_REQUIRE(fused_active(ctx) && ctx->frec && ctx->frec_rows > 0,
              "ppo_gather_staged_rows: no staged records (ppo_stage_records first)");
  PPO_REQUIRE(rows_d && b > 0 && b <= ctx->cfg.max_rows,
              "ppo_gather_staged_rows: b=%d outside [1, max_rows=%d]", b, ctx->cfg.max_rows);
  TimingScope timing_scope(ctx);
  const FusedArgs q = fused_args(ctx, nullptr, nullptr, nullptr, nullptr, nullptr, rows_d, b,
                                 nullptr, 0.f, 0.f, 0.f, 0.f, 0.f, true, false);
  if (int rc = fused_prep(ctx, q, as_stream(stream))) return rc;
  note_gathered(ctx, rows_d, b);
  return 0;
}

extern "C" int ppo_adam_pack(ppo_ctx *ctx, const float *g_d, float *m_d, float *v_d,
                             const float *sched_d, float neg_step_actor, float neg_step_critic,
                             float bc2_sqrt, float one_minus_beta1, float beta2,
                             float one_minus_beta2, float eps, void *stream) {
  if (int rc = check_ctx(ctx)) return rc;
  PPO_REQUIRE(fused_active(ctx), "ppo_adam_pack: needs the fused bf16 path");
  PPO_REQUIRE(g_d && m_d && v_d, "ppo_adam_pack: null buffer");
  TimingScope timing_scope(ctx);
  const AdamPackArgs a = adam_pack_args(ctx, g_d, m_d, v_d, sched_d, neg_step_actor,
                                        neg_step_critic, bc2_sqrt, one_minus_beta1, beta2,
                                        one_minus_beta2, eps);
  const double Hd = a.H;
  const TimRec rec{KC_ADAM, "adam_pack_kernel", 0.0,
                   28.0 * a.n + 2.0 * 2.0 * Hd * (a.din + 2.0 * Hd)};
  return adam_pack_launch(a, rec, as_stream(stream));
}

extern "C" int ppo_update_step_staged(ppo_ctx *ctx, const int32_t *rows_d, int b,
                                      const int32_t *next_rows_d, int next_b, float clip_lo,
                                      float clip_hi, float entropy_coef, float inv_b,
                                      float inv_ba, float *grad_d, float *loss_d, float *m_d,
                                      float *v_d, const float *sched_d, float neg_step_actor,
                                      float neg_step_critic, float bc2_sqrt,
                                      float one_minus_beta1, float beta2, float one_minus_beta2,
                                      float eps, int flags, void *stream) {
  if (int rc = check_ctx(ctx)) return rc;
  PPO_REQUIRE(fused_active(ctx) && ctx->frec && ctx->frec_rows > 0,
              "ppo_update_step_staged: no staged records (ppo_stage_records first)");
  PPO_REQUIRE(rows_d && grad_d && loss_d && m_d && v_d, "ppo_update_step_staged: null buffer");
  PPO_REQUIRE(b > 0 && b <= ctx->cfg.max_rows && next_b >= 0 && next_b <= ctx->cfg.max_rows &&
                  (next_b == 0) == (next_rows_d == nullptr),
              "ppo_update_step_staged: b=%d next_b=%d (max_rows %d)", b, next_b,
              ctx->cfg.max_rows);
  PPO_REQUIRE((flags & ~(PPO_STAGED_WEIGHTS_CURRENT | PPO_STAGED_ROWS_GATHERED)) == 0,
              "ppo_update_step_staged: flags %d", flags);
  hipStream_t st = as_stream(stream);
  TimingScope timing_scope(ctx);
  const bool gathered = (flags & PPO_STAGED_ROWS_GATHERED) && gathered_holds(ctx, rows_d, b);
  const bool current = flags & PPO_STAGED_WEIGHTS_CURRENT;
  FusedArgs q = fused_args(ctx, nullptr, nullptr, nullptr, nullptr, nullptr, rows_d, b, nullptr,
                           clip_lo, clip_hi, entropy_coef, inv_b, inv_ba, true, !current);
  if ((!gathered && !q.direct) || !current) {
    FusedArgs p = q;
    p.b = (gathered || q.direct) ? 0 : b;
    if (int rc = fused_prep(ctx, p, st)) return rc;
    if (p.b > 0) note_gathered(ctx, rows_d, b);
  }
  // tail: slab reduction + Adam + weight images, and the next minibatch's row gather
  const ReduceArgs r = fused_reduce_args(ctx, q, grad_d, loss_d);
  TailArgs t{};
  t.a = adam_pack_args(ctx, grad_d, m_d, v_d, sched_d, neg_step_actor, neg_step_critic, bc2_sqrt,
                       one_minus_beta1, beta2, one_minus_beta2, eps);
  t.rows = next_rows_d;
  t.rec = ctx->frec;
  t.n_rec = ctx->frec_rows;
  t.xb = ctx->fxb;
  t.srow = ctx->fsrow;
  t.b = q.direct ? 0 : next_b;  // direct: the next fused launch reads its rows itself
  t.reduce = true;
  if (int rc = fused_forward_backward(ctx, q, st)) {
    note_gathered(ctx, nullptr, 0);
    return rc;
  }
  const double P = static_cast<double>(ctx->total_params), H = ctx->fused_hidden;
  const TimRec rec{KC_REDUCE, "step_tail_kernel", static_cast<double>(q.G) * P,
                   4.0 * (q.G + 1.0) * P + 24.0 * P + 2.0 * 2.0 * H * (q.din + 2.0 * H) +
                       static_cast<double>(t.b) * (4.0 + 2.0 * kRecordBytes)};
  if (int rc = step_tail_launch(r, t, rec, st)) {
    note_gathered(ctx, nullptr, 0);
    return rc;
  }
  if (t.b > 0) note_gathered(ctx, next_rows_d, t.b);
  return 0;
}

extern "C" int ppo_observe_act(ppo_ctx *ctx, double *window_d, const double *obs_d,
                               const uint8_t *reset_d, int all_reset, const int32_t *bounds,
                               int n_bounds, int normalize, float *state_d, int n,
                               const float *eps_d, uint64_t seed, uint64_t offset,
                               float *action_d, float *logp_d, float *value_d, float *mean_d,
                               void *stream) {
  if (int rc = check_ctx(ctx)) return rc;
  const int o = ctx->cfg.obs_dim, w = ctx->cfg.window;
  PPO_REQUIRE(window_d && state_d && n > 0, "ppo_observe_act: null window/state or n <= 0");
  PPO_REQUIRE(n <= ctx->cfg.max_rows, "ppo_observe_act: n=%d exceeds max_rows=%d", n,
              ctx->cfg.max_rows);
  PPO_REQUIRE(n_bounds >= 0 && n_bounds < 16, "ppo_observe_act: too many slices (%d)", n_bounds);
  PolicySlices tab{};
  tab.count = normalize ? n_bounds : 0;
  for (int i = 0; i <= n_bounds && normalize; ++i) {
    PPO_REQUIRE(bounds != nullptr, "ppo_observe_act: null bounds");
    PPO_REQUIRE(bounds[i] >= 0 && bounds[i] <= o && (i == 0 || bounds[i] >= bounds[i - 1]),
                "ppo_observe_act: bounds must be ascending within [0, O]");
    tab.edge[i] = bounds[i];
  }
  if (!fused_active(ctx) && wide_active(ctx) && wide_observe_ok(ctx, tab.count)) {
    // wide path: window push + standardisation + bf16 operand rows in one launch, then the GEMMs
    TimingScope timing_scope(ctx);
    if (int rc = wide_observe(ctx, window_d, obs_d, reset_d, all_reset, tab, normalize, state_d, n,
                              as_stream(stream)))
      return rc;
    return wide_policy_step(ctx, state_d, n, eps_d, seed, offset, action_d, logp_d, value_d,
                            mean_d, false, as_stream(stream), true);
  }
  if (!fused_active(ctx) || w > kPolicyMaxWindow) {  // layered: A1 kernels, then GEMM policy step
    if (obs_d) {
      int rc = ppo_obs_window_push(window_d, obs_d, 1, reset_d, all_reset, n, o, w, stream);
      if (rc) return rc;
    }
    if (int rc = ppo_obs_normalize(window_d, state_d, n, o, w, bounds, n_bounds, normalize, stream))
      return rc;
    if (wide_active(ctx)) {  // the weight images are current (ppo_pack_weights before the rollout)
      TimingScope timing_scope(ctx);
      return wide_policy_step(ctx, state_d, n, eps_d, seed, offset, action_d, logp_d, value_d,
                              mean_d, false, as_stream(stream));
    }
    return ppo_policy_step(ctx, state_d, n, eps_d, seed, offset, action_d, logp_d, value_d,
                           mean_d, stream);
  }
  TimingScope timing_scope(ctx);
  PolicyFusedArgs q{};
  fused_nets(ctx, q.net);
  q.logstd = ctx->params + ctx->net[0].logstd_off;
  q.n = n;
  q.obs_dim = o;
  q.window = w;
  q.act_dim = ctx->cfg.act_dim;
  q.act = ctx->cfg.activation;
  q.hidden = ctx->fused_hidden;
  q.omv = ctx->cfg.output_max_value;
  q.window_d = window_d;
  q.obs_d = obs_d;
  q.reset_d = reset_d;
  q.all_reset = all_reset;
  q.tab = tab;
  q.normalize = normalize;
  q.state_d = state_d;
  q.do_actor = (action_d || logp_d || mean_d) ? 1 : 0;
  q.do_critic = value_d ? 1 : 0;
  q.eps = eps_d;
  q.seed = seed;
  q.offset = offset;
  q.offset_base = ctx->rng_counter;
  q.stamps = ctx->fstamp_on ? ctx->fstamps : nullptr;
  if (q.stamps) ctx->fstamp_g = 128;
  q.action = action_d;
  q.logp = logp_d;
  q.value = value_d;
  q.mean = mean_d;
  const double H = ctx->fused_hidden, A = ctx->cfg.act_dim, din = o * w;
  const double fl = 2.0 * n * ((q.do_actor ? din * H + H * H + A * H : 0.0) +
                               (q.do_critic ? din * H + H * H + H : 0.0));
  const double by = static_cast<double>(n) *
                    (8.0 * o * w * (obs_d ? 2.0 : 1.0) + (obs_d ? 8.0 * o : 0.0) + 4.0 * din +
                     (eps_d ? 4.0 * A : 0.0) + (action_d ? 4.0 * A : 0.0) + (mean_d ? 4.0 * A : 0.0) +
                     (logp_d ? 4.0 : 0.0) + (value_d ? 4.0 : 0.0));
  const TimRec rec{KC_POLICY_HEAD,
                   tim_active() ? intern_name("policy_fused_kernel<%d, %d, %d, false>", ctx->fused_hidden, q.act,
                                             q.act_dim <= 2 ? 2 : q.act_dim <= 4 ? 4 : q.act_dim <= 6 ? 6 : 8)
                                : nullptr,
                   fl, by};
  return policy_fused_launch(q, rec, as_stream(stream));
}

extern "C" int ppo_minibatch_grad(ppo_ctx *ctx, const float *states_d, const float *actions_d,
                                  const float *old_logp_d, const float *adv_d,
                                  const float *vtarget_d, const int32_t *rows_d, int b,
                                  const int32_t *count_d, float clip_lo, float clip_hi,
                                  float entropy_coef, float inv_b, float inv_ba, float *grad_d,
                                  float *loss_d, void *stream) {
  if (int rc = check_ctx(ctx)) return rc;
  PPO_REQUIRE(states_d && actions_d && old_logp_d && adv_d && vtarget_d && rows_d && grad_d,
              "ppo_minibatch_grad: null buffer");
  PPO_REQUIRE(b > 0 && b <= ctx->cfg.max_rows, "ppo_minibatch_grad: b=%d outside [1, max_rows=%d]",
              b, ctx->cfg.max_rows);
  hipStream_t st = as_stream(stream);
  TimingScope timing_scope(ctx);
  if (fused_active(ctx))
    return fused_minibatch_grad(ctx, states_d, actions_d, old_logp_d, adv_d, vtarget_d, rows_d, b,
                                count_d, clip_lo, clip_hi, entropy_coef, inv_b, inv_ba, grad_d,
                                loss_d, st);
  if (wide_active(ctx))
    return wide_minibatch_grad(ctx, states_d, actions_d, old_logp_d, adv_d, vtarget_d, rows_d, b,
                               count_d, clip_lo, clip_hi, entropy_coef, inv_b, inv_ba, grad_d,
                               loss_d, st);
  const bool both[2] = {true, true};
  const int din = ctx->cfg.obs_dim * ctx->cfg.window;
  const int A = ctx->cfg.act_dim;
  launch_k(TimRec{KC_GATHER, "gather_states_kernel", 0.0, 4.0 * b * (2.0 * din + 1)},
           gather_states_kernel, dim3(ceil_div(static_cast<int64_t>(b) * ctx->ldx, 256)),
           dim3(256), 0, st, states_d, rows_d, count_d, b, din, ctx->ldx, ctx->xg);
  PPO_LAUNCHED();
  if (int rc = forward_hidden(ctx, both, ctx->xg, nullptr, b, count_d, st, ctx->ldx)) return rc;

  // ---- heads: loss, dz, dH_L -------------------------------------------------------------
  NetDesc &NA = ctx->net[0], &NC = ctx->net[1];
  const LayerDesc &HA = NA.layer[NA.n_hidden], &HC = NC.layer[NC.n_hidden];
  int head_splits = std::min(kHeadSplits, std::max(1, b / 32));
  UpdateHeadArgs u{};
  u.ha = NA.h[NA.n_hidden - 1];
  u.hc = NC.h[NC.n_hidden - 1];
  u.ga = NA.g;
  u.gc = NC.g;
  u.dza = NA.dz;
  u.dzc = NC.dz;
  u.da = HA.in;
  u.dc = HC.in;
  u.act_dim = A;
  u.act = ctx->cfg.activation;
  u.wa = ctx->params + HA.w_off;
  u.ba = HA.b_off >= 0 ? ctx->params + HA.b_off : nullptr;
  u.logstd = ctx->params + NA.logstd_off;
  u.wc = ctx->params + HC.w_off;
  u.bc = ctx->params + HC.b_off;
  u.omv = ctx->cfg.output_max_value;
  u.rows = rows_d;
  u.rows_max = b;
  u.rows_n = count_d;
  u.actions = actions_d;
  u.old_logp = old_logp_d;
  u.adv = adv_d;
  u.vtarget = vtarget_d;
  u.clip_lo = clip_lo;
  u.clip_hi = clip_hi;
  u.ent_coef = entropy_coef;
  u.inv_b = inv_b;
  u.inv_ba = inv_ba;
  u.logstd_part = ctx->head_part;
  u.loss_part = ctx->head_part + static_cast<int64_t>(kHeadSplits) * A;
  u.splits = head_splits;
  const int hpl = hpl_for(std::max(u.da, u.dc));
  const int nj = (u.da == u.dc && u.da % 16 == 0) ? u.da / 16 : 0;
  const bool aligned = reinterpret_cast<uintptr_t>(u.ha) % 16 == 0 &&
                       reinterpret_cast<uintptr_t>(u.hc) % 16 == 0;
  const bool q4 = aligned && (nj == 2 || nj == 4 || nj == 8 || nj == 16 || nj == 32);
  const bool fused_head_w = q4 && A <= kFusedHeadAct;  // head dW/db inside the head kernel
  u.hw_part = ctx->head_w_part;
  u.hw_stride = ctx->hw_stride;
  u.off_ba = ctx->hw_off_ba;
  u.off_wc = ctx->hw_off_wc;
  u.off_bc = ctx->hw_off_bc;
  u.bf16 = ctx->prec == PPO_PREC_BF16;
  // algorithmic FLOPs: head forward + dH_L (+ head dW when fused); bytes per row: read H_L
  // (actor, critic), action, 4 scalars + row index; write dH_L (actor, critic) and dz (A + 1)
  const TimRec rec{KC_UPDATE_HEAD,
                   !tim_active() ? nullptr
                   : q4 ? intern_name("update_head_q4_kernel<%d, %s>", nj,
                                      fused_head_w ? "true" : "false")
                        : intern_name("update_head_kernel<%d>", hpl),
                   2.0 * b * ((fused_head_w ? 3.0 : 2.0) * (A * u.da + u.dc)),
                   4.0 * b * (2.0 * u.da + 2.0 * u.dc + 2.0 * A + 6.0)};
  if (q4) {
    const size_t shm = sizeof(float) * ((A + 1) * static_cast<size_t>(u.da) + 2 * 4 * 16 * kMaxAct);
    auto launch = [&](auto kernel) -> int {
      if (shm > 64 * 1024)
        PPO_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize,
                                        static_cast<int>(shm)));
      launch_k(rec, kernel, dim3(head_splits), dim3(256), static_cast<uint32_t>(shm), st, u);
      return 0;
    };
    int rc = 0;
    if (fused_head_w) {
      if (nj == 2) rc = launch(update_head_q4_kernel<2, true>);
      else if (nj == 4) rc = launch(update_head_q4_kernel<4, true>);
      else if (nj == 8) rc = launch(update_head_q4_kernel<8, true>);
      else if (nj == 16) rc = launch(update_head_q4_kernel<16, true>);
      else rc = launch(update_head_q4_kernel<32, true>);
    } else {
      if (nj == 2) rc = launch(update_head_q4_kernel<2, false>);
      else if (nj == 4) rc = launch(update_head_q4_kernel<4, false>);
      else if (nj == 8) rc = launch(update_head_q4_kernel<8, false>);
      else if (nj == 16) rc = launch(update_head_q4_kernel<16, false>);
      else rc = launch(update_head_q4_kernel<32, false>);
    }
    if (rc) return rc;
  } else if (hpl == 4) {
    launch_k(rec, update_head_kernel<4>, dim3(head_splits), dim3(256), 0, st, u);
  } else if (hpl == 8) {
    launch_k(rec, update_head_kernel<8>, dim3(head_splits), dim3(256), 0, st, u);
  } else {
    launch_k(rec, update_head_kernel<16>, dim3(head_splits), dim3(256), 0, st, u);
  }
  PPO_LAUNCHED();

  // ---- weight gradients, split-K over rows, deepest layer first ---------------------------
  const int splits = std::min(kSlabSplits, std::max(1, b / 64));
  const int64_t P = ctx->total_params;
  auto partial = [&](int layer_from_top) -> int {
    // layer index per net: head = n_hidden, then n_hidden-1 ... 0
    GemmBatch gb{};
    gb.prec = ctx->prec;
    gb.k = b;
    gb.rows_n = count_d;
    gb.splits = splits;
    gb.slab_stride = P;
    int np = 0, max_m = 0, max_n = 0;
    for (int z = 0; z < 2; ++z) {
      NetDesc &nd = ctx->net[z];
      const int l = nd.n_hidden - layer_from_top;
      if (l < 0) continue;
      const LayerDesc &L = nd.layer[l];
      GemmProblem &Q = gb.p[np++];
      // dY of layer l: head -> dz, top hidden -> g, lower hidden -> h[l] (overwritten in place)
      Q.a = (l == nd.n_hidden) ? nd.dz : (l == nd.n_hidden - 1 ? nd.g : nd.h[l]);
      Q.lda = L.out;
      Q.b = (l == 0) ? ctx->xg : nd.h[l - 1];
      Q.ldb = (l == 0) ? ctx->ldx : L.in;
      Q.c = ctx->slabs + L.w_off;
      Q.ldc = L.in;
      Q.colsum = L.b_off >= 0 ? ctx->slabs + L.b_off : nullptr;
      Q.m = L.out;
      Q.n = L.in;
      max_m = std::max(max_m, L.out);
      max_n = std::max(max_n, L.in);
    }
    if (!np) return 0;
    if (np == 2 && (gb.p[0].m != gb.p[1].m || gb.p[0].n != gb.p[1].n) &&
        ((gb.p[0].m <= 32) != (gb.p[1].m <= 32) || (gb.p[0].n <= 32) != (gb.p[1].n <= 32))) {
      GemmBatch g1 = gb;
      g1.p[0] = gb.p[1];
      if (int rc = gemm_wgrad_partial(gb, 1, gb.p[0].m, gb.p[0].n, st)) return rc;
      return gemm_wgrad_partial(g1, 1, g1.p[0].m, g1.p[0].n, st);
    }
    return gemm_wgrad_partial(gb, np, max_m, max_n, st);
  };
  auto input_grad = [&](int layer_from_top) -> int {
    // dH_{l-1} = (dY_l W_l) * act'(H_{l-1}), written over H_{l-1}; l = n_hidden - layer_from_top
    GemmBatch gb{};
    gb.prec = ctx->prec;
    gb.rows_n = count_d;
    gb.act = ctx->cfg.activation;
    int np = 0, max_n = 0, kdim = -1;
    for (int z = 0; z < 2; ++z) {
      NetDesc &nd = ctx->net[z];
      const int l = nd.n_hidden - layer_from_top;
      if (l < 1 || l >= nd.n_hidden) continue;  // head handled in the head kernel
      const LayerDesc &L = nd.layer[l];
      if (kdim >= 0 && kdim != L.out) {
        if (int rc = gemm_rows_dx(gb, np, b, max_n, st)) return rc;
        np = 0;
        max_n = 0;
      }
      kdim = L.out;
      GemmProblem &Q = gb.p[np++];
      Q.a = (l == nd.n_hidden - 1) ? nd.g : nd.h[l];
      Q.lda = L.out;
      Q.b = ctx->params + L.w_off;
      Q.ldb = L.in;
      Q.c = nd.h[l - 1];
      Q.aux = nd.h[l - 1];
      Q.ldc = L.in;
      Q.m = b;
      Q.n = L.in;
      gb.k = L.out;
      max_n = std::max(max_n, L.in);
    }
    if (!np) return 0;
    return gemm_rows_dx(gb, np, b, max_n, st);
  };
  const int depth = std::max(NA.n_hidden, NC.n_hidden);
  for (int s = 0; s <= depth; ++s) {
    // dW of layer n_hidden - s (needs its input); the head's is already in head_w_part
    if (!(s == 0 && fused_head_w))
      if (int rc = partial(s)) return rc;
    if (int rc = input_grad(s)) return rc;    // then overwrite that input with its gradient
  }

  // ---- reduce slabs -> grad, loss scalars ---------------------------------------------------
  ReduceArgs r{};
  int ns = 0;
  for (int z = 0; z < 2; ++z) {
    NetDesc &nd = ctx->net[z];
    if (z == 0) {
      ReduceSeg &g = r.seg[ns++];
      g.dst = nd.logstd_off;
      g.len = A;
      g.src = ctx->head_part;
      g.stride = A;
      g.nsplit = head_splits;
    }
    for (int l = 0; l <= nd.n_hidden; ++l) {
      const LayerDesc &L = nd.layer[l];
      const bool head_fused = fused_head_w && l == nd.n_hidden;
      ReduceSeg &g = r.seg[ns++];
      g.dst = L.w_off;
      g.len = static_cast<int64_t>(L.out) * L.in;
      g.src = head_fused ? ctx->head_w_part + (z == 0 ? 0 : ctx->hw_off_wc) : ctx->slabs + L.w_off;
      g.stride = head_fused ? ctx->hw_stride : P;
      g.nsplit = head_fused ? head_splits : splits;
      if (L.b_off >= 0) {
        ReduceSeg &gbs = r.seg[ns++];
        gbs.dst = L.b_off;
        gbs.len = L.out;
        gbs.src = head_fused ? ctx->head_w_part + (z == 0 ? ctx->hw_off_ba : ctx->hw_off_bc)
                             : ctx->slabs + L.b_off;
        gbs.stride = head_fused ? ctx->hw_stride : P;
        gbs.nsplit = head_fused ? head_splits : splits;
      }
    }
  }
  r.nseg = ns;
  r.total = P;
  r.grad = grad_d;
  r.loss_part = u.loss_part;
  r.loss_splits = head_splits;
  r.inv_b = inv_b;
  r.logstd = ctx->params + NA.logstd_off;
  r.act_dim = A;
  r.ent_coef = entropy_coef * ctx->ent_log_share;
  r.loss_out = loss_d;
  launch_k(TimRec{KC_REDUCE, "reduce_slabs_kernel", static_cast<double>(splits) * P,
                  4.0 * (static_cast<double>(splits) + 1) * P},
           reduce_slabs_kernel, dim3(ceil_div(P, kRedParams)), dim3(kRedThreads), 0, st, r);  // P % 16 == 0
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_ctx_phase_stamps(ppo_ctx *ctx, int enable, uint64_t *host_out, int max_values) {
  PPO_REQUIRE(ctx != nullptr, "ppo_ctx_phase_stamps: null ctx");
  PPO_REQUIRE(ctx->fused_ok, "ppo_ctx_phase_stamps: network shape has no fused kernel");
  PPO_HIP_TRY(hipSetDevice(ctx->device));
  const int n = 2 * kFusedMaxWG * kStampSlots;
  if (enable) {
    if (!ctx->fstamps) PPO_HIP_TRY(hipMalloc(&ctx->fstamps, sizeof(uint64_t) * n));
    PPO_HIP_TRY(hipMemset(ctx->fstamps, 0, sizeof(uint64_t) * n));
    ctx->fstamp_on = 1;
    return 0;
  }
  ctx->fstamp_on = 0;
  if (!ctx->fstamps) return 0;
  PPO_HIP_TRY(hipDeviceSynchronize());
  const int got = 2 * ctx->fstamp_g * kStampSlots;
  if (host_out && max_values > 0)
    PPO_HIP_TRY(hipMemcpy(host_out, ctx->fstamps, sizeof(uint64_t) * std::min(got, max_values),
                          hipMemcpyDeviceToHost));
  return got;
}

extern "C" int ppo_ctx_set_precision(ppo_ctx *ctx, int prec) {
  PPO_REQUIRE(ctx != nullptr, "ppo_ctx_set_precision: null ctx");
  PPO_REQUIRE(prec == PPO_PREC_F32 || prec == PPO_PREC_BF16,
              "ppo_ctx_set_precision: unknown precision %d", prec);
  ctx->prec = prec;
  if (prec == PPO_PREC_BF16)  // the wide path's workspace, for the shapes it covers
    if (int rc = wide_alloc(ctx)) return rc;
  return 0;
}

extern "C" int ppo_ctx_loss_entropy_share(ppo_ctx *ctx, float share) {
  PPO_REQUIRE(ctx != nullptr, "ppo_ctx_loss_entropy_share: null ctx");
  ctx->ent_log_share = share;
  return 0;
}

extern "C" int ppo_ctx_fused_direct(ppo_ctx *ctx, int enable) {
  PPO_REQUIRE(ctx != nullptr, "ppo_ctx_fused_direct: null ctx");
  if (enable < 0) return ctx->fdirect ? 1 : 0;
  ctx->fdirect = enable != 0;
  note_gathered(ctx, nullptr, 0);
  return 0;
}

extern "C" int ppo_ctx_set_rng_counter(ppo_ctx *ctx, const uint64_t *counter_d) {
  PPO_REQUIRE(ctx != nullptr, "ppo_ctx_set_rng_counter: null ctx");
  ctx->rng_counter = counter_d;
  return 0;
}

namespace ppo {
int timing_enable(Timing &t, int enable, int capacity) {
  if (enable && capacity > t.capacity) {
    for (int i = 0; i < 2 * t.capacity; ++i) (void)hipEventDestroy(t.ev[i]);
    delete[] t.ev;
    delete[] t.cls;
    delete[] t.kname;
    delete[] t.flops;
    delete[] t.bytes;
    t.ev = new hipEvent_t[2 * capacity];
    t.cls = new int[capacity];
    t.kname = new const char *[capacity];
    t.flops = new double[capacity];
    t.bytes = new double[capacity];
    for (int i = 0; i < 2 * capacity; ++i) PPO_HIP_TRY(hipEventCreate(&t.ev[i]));
    t.capacity = capacity;
  }
  if (enable) {
    t.used = 0;
    for (int c = 0; c < KC_COUNT; ++c) t.ms[c] = t.fl[c] = t.by[c] = 0, t.n[c] = 0;
    t.per_kernel.clear();
  }
  t.on = enable != 0 && t.capacity > 0;
  if (t.on) g_free_tim = &t;
  else if (g_free_tim == &t) g_free_tim = nullptr;
  return 0;
}

// Folds pending records into the per-class and per-kernel totals (host sync on their events).
static int timing_fold(Timing &t) {
  for (int i = 0; i < t.used; ++i) {
    PPO_HIP_TRY(hipEventSynchronize(t.ev[2 * i + 1]));
    float ms = 0.f;
    PPO_HIP_TRY(hipEventElapsedTime(&ms, t.ev[2 * i], t.ev[2 * i + 1]));
    const int c = t.cls[i];
    t.ms[c] += ms;
    t.fl[c] += t.flops[i];
    t.by[c] += t.bytes[i];
    t.n[c] += 1;
    const char *name = t.kname[i] ? t.kname[i] : kClassNames[c];
    KernelTotals *k = nullptr;
    for (KernelTotals &e : t.per_kernel)
      if (e.name == name) k = &e;
    if (!k) {
      t.per_kernel.push_back(KernelTotals{name, c, 0.0, 0.0, 0.0, 0});
      k = &t.per_kernel.back();
    }
    k->ms += ms;
    k->fl += t.flops[i];
    k->by += t.bytes[i];
    k->n += 1;
  }
  t.used = 0;
  return 0;
}

int timing_read_class(Timing &t, int kclass, double *total_ms, int64_t *launches, double *flops,
                      double *bytes) {
  if (kclass < 0) return KC_COUNT;
  PPO_REQUIRE(kclass < KC_COUNT, "timing read: class %d out of range", kclass);
  if (int rc = timing_fold(t)) return rc;
  if (total_ms) *total_ms = t.ms[kclass];
  if (launches) *launches = t.n[kclass];
  if (flops) *flops = t.fl[kclass];
  if (bytes) *bytes = t.by[kclass];
  return 0;
}

int timing_read_kernel(Timing &t, int index, const char **name, int *kclass, double *total_ms,
                       int64_t *launches, double *flops, double *bytes) {
  if (int rc = timing_fold(t)) return rc;
  const int count = static_cast<int>(t.per_kernel.size());
  if (index < 0) return count;
  PPO_REQUIRE(index < count, "timing read: kernel index %d out of range [0, %d)", index, count);
  const KernelTotals &k = t.per_kernel[index];
  if (name) *name = k.name;
  if (kclass) *kclass = k.cls;
  if (total_ms) *total_ms = k.ms;
  if (launches) *launches = k.n;
  if (flops) *flops = k.fl;
  if (bytes) *bytes = k.by;
  return 0;
}
}  // namespace ppo

extern "C" int ppo_ctx_timing(ppo_ctx *ctx, int enable, int capacity) {
  PPO_REQUIRE(ctx != nullptr, "ppo_ctx_timing: null ctx");
  return timing_enable(ctx->tim, enable, capacity);
}

extern "C" int ppo_ctx_timing_read(ppo_ctx *ctx, int kclass, double *total_ms, int64_t *launches,
                                   double *flops, double *bytes) {
  PPO_REQUIRE(ctx != nullptr, "ppo_ctx_timing_read: null ctx");
  return timing_read_class(ctx->tim, kclass, total_ms, launches, flops, bytes);
}

extern "C" int ppo_ctx_timing_kernel(ppo_ctx *ctx, int index, const char **name, int *kclass,
                                     double *total_ms, int64_t *launches, double *flops,
                                     double *bytes) {
  PPO_REQUIRE(ctx != nullptr, "ppo_ctx_timing_kernel: null ctx");
  return timing_read_kernel(ctx->tim, index, name, kclass, total_ms, launches, flops, bytes);
}

extern "C" const char *ppo_kernel_class_name(int kclass) {
  return (kclass >= 0 && kclass < KC_COUNT) ? kClassNames[kclass] : "";
}
