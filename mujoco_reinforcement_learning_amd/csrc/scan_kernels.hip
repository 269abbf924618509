// HBM-bound kernels of the PPO hot path (gfx950): GAE scan (A7/A8), per-env standardisation
// over T (A6/A9), observation window + per-sample standardisation (A1), minibatch row maps
// (A10), fused Adam (A15), and the synthetic-env / Philox harness kernels.
//
// Layout: every (N, T) rollout quantity is time-major, element (n, t) at t*N + n, so a wave of
// 64 envs reads one 256-B row segment per timestep (coalesced), and the per-env recurrences run
// one env per lane with no cross-lane traffic.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "adam_elem.h"
#include "common.h"
#include "gae_pipe.h"
#include "row_stats.h"
#include "timing.h"

namespace ppo {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// ============================================================================================
// GAE + value target (torchrl 0.6.0 generalized_advantage_estimate, ppo.py:70-80)
// ============================================================================================
// Per env (lane) a backward recurrence over T carried in the REWARD's dtype (torch promotion:
// f64 numpy rewards make delta and prev_advantage f64; f32 rewards keep everything f32):
//   g_nt  = gamma_f * (!term)                (f32, torch: python float * int tensor)
//   delta = ((RT)r + (RT)(g_nt*v')) - (RT)v
//   disc  = lg_f * (!done)                   (f32, lg_f = f32(lambda*gamma in double))
//   prev  = delta + prev * (RT)disc          (two roundings, no FMA)
//   adv = (float)prev ; vtarget = adv + v    (f32)
// Loads are issued a chunk of CH timesteps ahead of the dependent chain so the scan is bound by
// HBM latency/bandwidth rather than by one load per dependent step.
template <typename RT, int CH>
__global__ __launch_bounds__(64) void gae_kernel(const float *__restrict__ value,
                                                 const float *__restrict__ next_value,
                                                 const RT *__restrict__ reward,
                                                 const uint8_t *__restrict__ done,
                                                 const uint8_t *__restrict__ term, int force_last,
                                                 int n, int t_len, float gamma_f, float lg_f,
                                                 float *__restrict__ adv,
                                                 float *__restrict__ vtarget) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n) return;
  RT prev = 0;
  int t_hi = t_len;  // process chunks [t_hi-CH, t_hi) from the end
  while (t_hi > 0) {
    const int t_lo = t_hi - CH > 0 ? t_hi - CH : 0;
    const int cnt = t_hi - t_lo;
    float v[CH], vn[CH];
    RT r[CH];
    uint8_t dn[CH], tm[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (i < cnt) {
        const int64_t idx = static_cast<int64_t>(t_lo + i) * n + env;
        v[i] = value[idx];
        vn[i] = next_value[idx];
        r[i] = reward[idx];
        tm[i] = term[idx];
        dn[i] = done ? done[idx] : tm[i];
      }
    }
#pragma unroll
    for (int i = CH - 1; i >= 0; --i) {
      if (i < cnt) {
        const int t = t_lo + i;
        const bool is_done = dn[i] != 0 || (force_last && t == t_len - 1);
        const float g_nt = gamma_f * (tm[i] ? 0.f : 1.f);
        const float gv = g_nt * vn[i];
        const RT delta = (r[i] + static_cast<RT>(gv)) - static_cast<RT>(v[i]);
        const float disc = lg_f * (is_done ? 0.f : 1.f);
        prev = delta + prev * static_cast<RT>(disc);
        const float a = static_cast<float>(prev);
        const int64_t idx = static_cast<int64_t>(t) * n + env;
        adv[idx] = a;
        vtarget[idx] = a + v[i];
      }
    }
    t_hi = t_lo;
  }
}

// LDS-staged variant: a 256-thread block owns EB envs.  Phase 1: every thread issues its share
// of the [T][EB] tile loads (V, V', r, terminated) at once -> LDS (latency paid once, all CUs
// loading).  Phase 2: EB lanes run the same recurrence as gae_kernel out of LDS.  Phase 3: all
// threads store adv / vtarget coalesced.  Bit-identical to gae_kernel.  T*EB must fit LDS.
template <typename RT, int EB, int IT>  // IT = ceil(T*EB / 256) load slots per thread
__global__ __launch_bounds__(256) void gae_lds_kernel(const float *__restrict__ value,
                                                      const float *__restrict__ next_value,
                                                      const RT *__restrict__ reward,
                                                      const uint8_t *__restrict__ done,
                                                      const uint8_t *__restrict__ term,
                                                      int force_last, int n, int t_len,
                                                      float gamma_f, float lg_f,
                                                      float *__restrict__ adv,
                                                      float *__restrict__ vtarget) {
  extern __shared__ __attribute__((aligned(16))) unsigned char gae_smem[];
  const int total = t_len * EB;
  RT *s_r = reinterpret_cast<RT *>(gae_smem);
  float *s_v = reinterpret_cast<float *>(s_r + total);
  float *s_vn = s_v + total;
  uint8_t *s_fl = reinterpret_cast<uint8_t *>(s_vn + total);  // bit0 term, bit1 done
  const int env0 = blockIdx.x * EB;
  const int tid = threadIdx.x;
  // issue every load of this thread before the first LDS store: one HBM latency per block
  // delta and the discount do not depend on the carry: every thread computes them for its slots
  // (same operations as gae_kernel), so the serial chain below is one mul + one add per step.
  float lv[IT];
  RT ld[IT];
  uint8_t lfl[IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int e = tid + 256 * k;
    const int t = e / EB, c = e - (e / EB) * EB;
    const int env = env0 + c;
    if (e < total && env < n) {
      const int64_t idx = static_cast<int64_t>(t) * n + env;
      const float v = value[idx];
      const float vn = next_value[idx];
      const RT r = reward[idx];
      const uint8_t tm = term[idx];
      const uint8_t dn = done ? done[idx] : tm;
      const float g_nt = gamma_f * (tm ? 0.f : 1.f);
      const float gv = g_nt * vn;
      lv[k] = v;
      ld[k] = (r + static_cast<RT>(gv)) - static_cast<RT>(v);
      lfl[k] = static_cast<uint8_t>((dn || (force_last && t == t_len - 1)) ? 1 : 0);
    }
  }
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int e = tid + 256 * k;
    if (e < total && env0 + (e - (e / EB) * EB) < n) {
      s_v[e] = lv[k];
      s_r[e] = ld[k];  // delta
      s_fl[e] = lfl[k];
    }
  }
  __syncthreads();
  if (tid < EB && env0 + tid < n) {
    RT prev = 0;
    constexpr int U = 8;  // LDS reads of 8 steps issued ahead of their dependent chain
    int t = t_len - 1;
    for (; t >= U - 1; t -= U) {
      RT delta[U];
      float disc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = (t - u) * EB + tid;
        delta[u] = s_r[e];
        disc[u] = lg_f * (s_fl[e] ? 0.f : 1.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        prev = delta[u] + prev * static_cast<RT>(disc[u]);
        s_vn[(t - u) * EB + tid] = static_cast<float>(prev);
      }
    }
    for (; t >= 0; --t) {
      const int e = t * EB + tid;
      prev = s_r[e] + prev * static_cast<RT>(lg_f * (s_fl[e] ? 0.f : 1.f));
      s_vn[e] = static_cast<float>(prev);
    }
  }
  __syncthreads();
  for (int e = tid; e < total; e += 256) {
    const int t = e / EB, c = e - (e / EB) * EB;
    const int env = env0 + c;
    if (env < n) {
      const int64_t idx = static_cast<int64_t>(t) * n + env;
      const float a = s_vn[e];
      adv[idx] = a;
      vtarget[idx] = a + s_v[e];  // value_target = advantage + state_value (f32)
    }
  }
}

// Pipelined variant (the default for T <= 16*KMAX): gae_pipe.h's body with no extra outputs.
template <typename RT, int EB, int KMAX>
__global__ __launch_bounds__(EB * 16) void gae_pipe_kernel(const float *__restrict__ value,
                                                           const float *__restrict__ next_value,
                                                           const RT *__restrict__ reward,
                                                           const uint8_t *__restrict__ done,
                                                           const uint8_t *__restrict__ term,
                                                           int force_last, int n, int t_len,
                                                           float gamma_f, float lg_f,
                                                           float *__restrict__ adv,
                                                           float *__restrict__ vtarget) {
  GaeNoEmit em;
  gae_pipe_body<RT, EB, KMAX>(value, next_value, reward, done, term, force_last, n, t_len, gamma_f,
                              lg_f, adv, vtarget, em);
}

// Producer / consumer variant (gae_pipe.h gae_chain_body): EB*16 producer threads + one chain wave.
template <typename RT, int EB, int KMAX>
__global__ __launch_bounds__(EB * 16 + 64) void gae_chain_kernel(const float *__restrict__ value,
                                                                 const float *__restrict__ next_value,
                                                                 const RT *__restrict__ reward,
                                                                 const uint8_t *__restrict__ done,
                                                                 const uint8_t *__restrict__ term,
                                                                 int force_last, int n, int t_len,
                                                                 float gamma_f, float lg_f,
                                                                 float *__restrict__ adv,
                                                                 float *__restrict__ vtarget) {
  gae_chain_body<RT, EB, KMAX>(value, next_value, reward, done, term, force_last, n, t_len, gamma_f,
                               lg_f, adv, vtarget);
}

// ============================================================================================
// Per-env standardisation over T (ppo.py:66-69 rewards f64, :81-88 advantage / value target f32)
// x <- ((x - mean_T) / std_T) * scale, unbiased std.  torch computes mean in the tensor dtype and
// std with a double Welford accumulator; we accumulate both in f64 and round where torch rounds.
// ============================================================================================
template <typename T>
__global__ __launch_bounds__(64) void normalize_rows_kernel(T *__restrict__ x, int n, int t_len,
                                                            double scale) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n) return;
  double s = 0.0;
  for (int t = 0; t < t_len; ++t) s += static_cast<double>(x[static_cast<int64_t>(t) * n + env]);
  const T mean = static_cast<T>(s / t_len);
  double cs = 0.0;
  for (int t = 0; t < t_len; ++t) {
    const T c = x[static_cast<int64_t>(t) * n + env] - mean;
    cs += static_cast<double>(c);
  }
  const double cmean = cs / t_len;
  double ss = 0.0;
  for (int t = 0; t < t_len; ++t) {
    const double d = static_cast<double>(x[static_cast<int64_t>(t) * n + env] - mean) - cmean;
    ss += d * d;
  }
  const T stdv = static_cast<T>(sqrt(ss / (t_len - 1)));
  const T sc = static_cast<T>(scale);
  for (int t = 0; t < t_len; ++t) {
    const int64_t idx = static_cast<int64_t>(t) * n + env;
    const T c = x[idx] - mean;
    x[idx] = (c / stdv) * sc;
  }
}

// ============================================================================================
// Observation window (helper.py:51-64, running_gym_sequential_vectorized.py:53-58)
// ============================================================================================
template <typename OT>
__global__ void obs_window_push_kernel(double *__restrict__ window, const OT *__restrict__ obs,
                                       const uint8_t *__restrict__ reset, int all_reset, int n,
                                       int o, int w) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;  // (env, feat)
  if (i >= static_cast<int64_t>(n) * o) return;
  const int env = static_cast<int>(i / o);
  const double x = static_cast<double>(obs[i]);
  double *row = window + i * w;
  const bool full = all_reset || (reset && reset[env]);
  if (full) {
    for (int k = 0; k < w; ++k) row[k] = x;
  } else {
    for (int k = 0; k + 1 < w; ++k) row[k] = row[k + 1];
    row[w - 1] = x;
  }
}

struct SliceTable {
  int32_t edge[16];
  int32_t count;  // number of slices
};

// One thread per (env, window slot): standardise each feature slice in f64 (mean, unbiased std,
// std==0 -> 1; row_stats.h, the fused rollout step's exact arithmetic), cast to f32, write
// permuted (N, W, O).  running_gym_sequential_vectorized.py:61-92.  O <= 32 (wider rows take
// obs_normalize_wide_kernel).
__global__ __launch_bounds__(128) void obs_normalize_kernel(const double *__restrict__ window, float *__restrict__ state,
                                     int n, int o, int w, SliceTable tab, int normalize) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;  // (env, slot)
  if (i >= static_cast<int64_t>(n) * w) return;
  const int env = static_cast<int>(i / w);
  const int slot = static_cast<int>(i % w);
  const double *src = window + static_cast<int64_t>(env) * o * w + slot;  // feature f at f*w
  float *dst = state + (static_cast<int64_t>(env) * w + slot) * o;
  if (!normalize) {
    for (int f = 0; f < o; ++f) dst[f] = static_cast<float>(src[static_cast<int64_t>(f) * w]);
    return;
  }
  double x[32];
#pragma unroll
  for (int f = 0; f < 32; ++f) x[f] = f < o ? src[static_cast<int64_t>(f < o ? f : 0) * w] : 0.0;
  for (int s = 0; s < tab.count; ++s) {
    const int lo = tab.edge[s], hi = tab.edge[s + 1];
    if (hi - lo <= 0) continue;
    const SliceStats st = slice_stats32(x, lo, hi);
#pragma unroll
    for (int f = 0; f < 32; ++f)
      if (f >= lo && f < hi) dst[f] = static_cast<float>((x[f] - st.mean) / st.sd);
  }
}

// Wide observations (O > 32, e.g. Humanoid-v4 O=376 with its six slices): one wave per (env, slot)
// instead of one thread.  Each slice statistic is a lane-strided partial sum followed by a
// fixed xor-tree across the wave (deterministic run to run); the f64 result differs from the
// sequential loop only in summation order, i.e. it rounds to the same f32 state up to rare
// ties (the 1-ulp bar of test_obs_window_and_normalize).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

__global__ __launch_bounds__(256) void obs_normalize_wide_kernel(
    const double *__restrict__ window, float *__restrict__ state, int n, int o, int w,
    SliceTable tab, int normalize) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  if (i >= static_cast<int64_t>(n) * w) return;  // wave-uniform
  const int env = static_cast<int>(i / w);
  const int slot = static_cast<int>(i % w);
  const double *src = window + static_cast<int64_t>(env) * o * w + slot;  // feature f at f*w
  float *dst = state + (static_cast<int64_t>(env) * w + slot) * o;
  if (!normalize) {
    for (int f = lane; f < o; f += 64) dst[f] = static_cast<float>(src[static_cast<int64_t>(f) * w]);
    return;
  }
  for (int s = 0; s < tab.count; ++s) {
    const int lo = tab.edge[s], hi = tab.edge[s + 1];
    const int cnt = hi - lo;
    if (cnt <= 0) continue;
    double sum = 0.0;
    for (int f = lo + lane; f < hi; f += 64) sum += src[static_cast<int64_t>(f) * w];
    const double mean = wave_sum(sum) / cnt;
    double csum = 0.0;
    for (int f = lo + lane; f < hi; f += 64) csum += src[static_cast<int64_t>(f) * w] - mean;
    const double cmean = wave_sum(csum) / cnt;
    double ss = 0.0;
    for (int f = lo + lane; f < hi; f += 64) {
      const double d = (src[static_cast<int64_t>(f) * w] - mean) - cmean;
      ss += d * d;
    }
    double sd = sqrt(wave_sum(ss) / (cnt - 1));  // cnt == 1 -> NaN, as torch.std
    if (sd == 0.0) sd = 1.0;
    for (int f = lo + lane; f < hi; f += 64)
      dst[f] = static_cast<float>((src[static_cast<int64_t>(f) * w] - mean) / sd);
  }
}

// ============================================================================================
// Synthetic VecEnv step (harness; oracle/ppo_ref.py RefSyntheticEnv)
// ============================================================================================
__global__ void synthetic_env_step_kernel(const float *__restrict__ base_obs,
                                          const float *__restrict__ base_reward,
                                          const uint8_t *__restrict__ base_term,
                                          const float *__restrict__ action, int n, int o, int a,
                                          double *__restrict__ obs_out,
                                          double *__restrict__ reward_out,
                                          uint8_t *__restrict__ term_out) {
  // 32-bit index arithmetic (the host checks n * o < 2^31): a 64-bit divide is a long
  // software sequence ahead of the first load
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= static_cast<uint32_t>(n) * static_cast<uint32_t>(o)) return;
  const uint32_t env = i / static_cast<uint32_t>(o);
  const uint32_t f = i - env * static_cast<uint32_t>(o);
  const double act = static_cast<double>(action[env * a + (f % static_cast<uint32_t>(a))]);
  obs_out[i] = static_cast<double>(base_obs[i]) + 0.1 * act;
  if (f == 0) {
    double ctrl = 0.0;
    for (int j = 0; j < a; ++j) {
      const double aj = static_cast<double>(action[env * a + j]);
      ctrl = ctrl + aj * aj;
    }
    reward_out[env] = static_cast<double>(base_reward[env]) - 0.01 * ctrl;
    term_out[env] = base_term[env];
  }
}

// One step of the single test environment inside Algorithm.test (base_algorithm.py:21-48), with
// the host branch of :33-37 taken on the device: the step counter k lives in device memory, so
// the 1000-step evaluation loop never synchronises the host.  One block; thread f handles
// feature f.  Dynamics = env 0 of the synthetic streams at k (RefSyntheticEnv.test_step):
//   obs' = base_obs[(k+1) % (T+1), 0] + 0.1 a[f % A],  r = base_reward[k % T, 0] - 0.01 sum a^2,
//   terminated = base_term[k % T, 0];  terminated -> reset_environment(test): every window slot
//   := base_obs[0, 0] and k := 0 (helper.py:59-64); else shift + append (helper.py:51-57) and
//   k := k + 1.  rewards.append(r) (:38) is a sequential f64 running sum.
__global__ __launch_bounds__(256) void synthetic_test_step_kernel(
    const float *__restrict__ base_obs, const float *__restrict__ base_reward,
    const uint8_t *__restrict__ base_term, int t_len, int n_envs, const float *__restrict__ action,
    int o, int a, int w, double *__restrict__ window, int32_t *__restrict__ step,
    double *__restrict__ reward_sum, uint8_t *__restrict__ term_out) {
  const int k = *step;
  const int kt = k % t_len;
  const bool term = base_term[static_cast<int64_t>(kt) * n_envs] != 0;
  const float *nxt = base_obs + static_cast<int64_t>((k + 1) % (t_len + 1)) * n_envs * o;
  for (int f = threadIdx.x; f < o; f += blockDim.x) {
    double *row = window + static_cast<int64_t>(f) * w;
    if (term) {
      const double x0 = static_cast<double>(base_obs[f]);
      for (int s = 0; s < w; ++s) row[s] = x0;
    } else {
      const double x = static_cast<double>(nxt[f]) + 0.1 * static_cast<double>(action[f % a]);
      for (int s = 0; s + 1 < w; ++s) row[s] = row[s + 1];
      row[w - 1] = x;
    }
  }
  __syncthreads();  // every thread has read *step
  if (threadIdx.x == 0) {
    double ctrl = 0.0;
    for (int j = 0; j < a; ++j) {
      const double aj = static_cast<double>(action[j]);
      ctrl = ctrl + aj * aj;
    }
    const double r = static_cast<double>(base_reward[static_cast<int64_t>(kt) * n_envs]) - 0.01 * ctrl;
    *reward_sum = *reward_sum + r;
    *term_out = term ? 1 : 0;
    *step = term ? 0 : k + 1;
  }
}

// ============================================================================================
// Philox4x32-10 normals (perf-mode eps; the parity mode takes host torch.randn instead)
// ============================================================================================
__global__ void philox_normal_kernel(uint64_t seed, uint64_t offset, const uint64_t *counter,
                                     float *__restrict__ out, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t base = offset + (counter ? *counter : 0);
  if (i < n) out[i] = philox_normal_at(seed, base + static_cast<uint64_t>(i));
}

// ============================================================================================
// Minibatch rows (ppo.py:99-106): reference flat index f = n*T + t -> storage row t*N + n
// ============================================================================================
__global__ void perm_to_rows_kernel(const int64_t *__restrict__ perm, int64_t start, int b,
                                    int n_envs, int t_len, int32_t *__restrict__ rows) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= b) return;
  const int64_t f = perm[start + j];
  const int env = static_cast<int>(f / t_len);
  const int t = static_cast<int>(f % t_len);
  rows[j] = t * n_envs + env;
}

// Exact data-parallel variant: keep envs of [lo, hi) in order (block-wide scan, one block).
__global__ __launch_bounds__(1024) void perm_to_rows_shard_kernel(
    const int64_t *__restrict__ perm, int64_t start, int b, int n_envs, int t_len, int lo, int hi,
    int32_t *__restrict__ rows, int32_t *__restrict__ count) {
  __shared__ int wave_tot[16];
  __shared__ int base_s;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) base_s = 0;
  __syncthreads();
  for (int c0 = 0; c0 < b; c0 += 1024) {
    const int j = c0 + tid;
    int keep = 0, row = 0;
    if (j < b) {
      const int64_t f = perm[start + j];
      const int env = static_cast<int>(f / t_len);
      const int t = static_cast<int>(f % t_len);
      keep = (env >= lo && env < hi);
      row = t * (hi - lo) + (env - lo);  // rank-local time-major storage
    }
    const uint64_t mask = __ballot(keep);
    const int before = __popcll(mask & ((1ull << lane) - 1ull));
    if (lane == 0) wave_tot[wid] = __popcll(mask);
    __syncthreads();
    int off = base_s;
    for (int k = 0; k < wid; ++k) off += wave_tot[k];
    if (keep) rows[off + before] = row;
    __syncthreads();
    if (tid == 0) {
      int tot = 0;
      for (int k = 0; k < 16; ++k) tot += wave_tot[k];
      base_s += tot;
    }
    __syncthreads();
  }
  if (tid == 0) *count = base_s;
}

// Perf-mode shuffle: 4-round Feistel bijection on [0, 4^h) with cycle walking into [0, NT).
__device__ __forceinline__ uint32_t mix32(uint32_t x, uint32_t k) {
  x ^= k;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__global__ void feistel_rows_kernel(uint64_t seed, uint64_t epoch, int64_t start, int b,
                                    int n_envs, int t_len, int half_bits,
                                    int32_t *__restrict__ rows) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= b) return;
  const uint32_t total = static_cast<uint32_t>(n_envs) * static_cast<uint32_t>(t_len);
  const uint32_t hmask = (1u << half_bits) - 1u;
  uint32_t k[4];
  for (int r = 0; r < 4; ++r)
    k[r] = mix32(static_cast<uint32_t>(seed) ^ (0x9E3779B9u * (r + 1)),
                 static_cast<uint32_t>(seed >> 32) + static_cast<uint32_t>(epoch) * 0x85EBCA6Bu);
  uint32_t x = static_cast<uint32_t>(start + j);
  do {
    uint32_t l = x >> half_bits, rr = x & hmask;
    for (int r = 0; r < 4; ++r) {
      const uint32_t nl = rr;
      rr = l ^ (mix32(rr, k[r]) & hmask);
      l = nl;
    }
    x = (l << half_bits) | rr;
  } while (x >= total);
  const int env = static_cast<int>(x / t_len);
  const int t = static_cast<int>(x % t_len);
  rows[j] = t * n_envs + env;
}

// ============================================================================================
// Fused Adam (torch.optim.Adam single-tensor CPU path, adam.py _single_tensor_adam)
//   m = lerp(m, g, 1-b1)          -> vectorised lerp: fma(w, g-m, m) for w < 0.5
//   v = fma((1-b2)*g, g, v*b2)    -> mul_ then addcmul_ (contracted to one FMA on CPU)
//   denom = sqrt(v)/bc2_sqrt + eps
//   p = p + (neg_step*m)/denom    -> addcdiv_ (value*t1/t2)
// ============================================================================================
__global__ void adam_kernel(float *__restrict__ p, const float *__restrict__ g,
                            float *__restrict__ m, float *__restrict__ v, int64_t n,
                            int64_t n_actor, float neg_step_a, float neg_step_c, float w1,
                            float b2, float omb2, float bc2_sqrt, float eps) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float mi = m[i], vi = v[i];
  p[i] = adam_elem(p[i], g[i], mi, vi, (i < n_actor) ? neg_step_a : neg_step_c, w1, b2, omb2,
                   bc2_sqrt, eps);
  m[i] = mi;
  v[i] = vi;
}

// Same update with the step-dependent scalars (neg_step_actor, neg_step_critic, bc2_sqrt) read
// from device memory when the kernel runs: a hipGraph-captured optimizer loop replays with the
// schedule the host uploads for each iteration.
__global__ void adam_sched_kernel(float *__restrict__ p, const float *__restrict__ g,
                                  float *__restrict__ m, float *__restrict__ v, int64_t n,
                                  int64_t n_actor, const float *__restrict__ sched, float w1,
                                  float b2, float omb2, float eps) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float mi = m[i], vi = v[i];
  p[i] = adam_elem(p[i], g[i], mi, vi, (i < n_actor) ? sched[0] : sched[1], w1, b2, omb2,
                   sched[2], eps);
  m[i] = mi;
  v[i] = vi;
}

}  // namespace ppo

// ==============================================================================================
// C-ABI entry points
// ==============================================================================================
using namespace ppo;

extern "C" int ppo_abi_version(void) { return PPO_ABI_VERSION; }

extern "C" const char *ppo_last_error(void) { return g_err; }

// algorithmic bytes: read V, V', reward, terminated (+ done when given), write adv, vtarget
static double gae_bytes(size_t reward_bytes, bool has_done, int n, int t) {
  return static_cast<double>(n) * t * (4 + 4 + reward_bytes + 1 + (has_done ? 1 : 0) + 4 + 4);
}

extern "C" int ppo_gae(const float *value_d, const float *next_value_d, const void *reward_d,
                       int reward_is_f64, const uint8_t *done_d, const uint8_t *terminated_d,
                       int force_last_done, int n, int t, double gamma, double lmbda,
                       float *adv_d, float *vtarget_d, void *stream) {
  PPO_REQUIRE(value_d && next_value_d && reward_d && terminated_d && adv_d && vtarget_d,
              "ppo_gae: null buffer");
  PPO_REQUIRE(n > 0 && t > 0, "ppo_gae: bad shape n=%d t=%d", n, t);
  const float gamma_f = static_cast<float>(gamma);
  const float lg_f = static_cast<float>(lmbda * gamma);
  // LDS-staged scan.  EB envs per block: 16 (>= 256 blocks at N = 4096), 32 once N gives >= 2048
  // blocks anyway (full 128-B lines per time row); halved until the [T][EB] tile fits 128 KiB and
  // the per-thread load slots fit 16.  Very long horizons fall back to the register-chunked kernel.
  const size_t per_elem = (reward_is_f64 ? 8 : 4) + 4 + 4 + 1;
  static const int eb_knob = [] {  // PPO_GAE_EB overrides envs per block (experiments)
    const char *v = getenv("PPO_GAE_EB");
    return v ? atoi(v) : 0;
  }();
  int eb = eb_knob > 0 ? eb_knob : ((n >= 65536) ? 32 : 16);
  while (eb > 1 && (static_cast<size_t>(t) * eb * per_elem > 131072 || t * eb > 16 * 256))
    eb >>= 1;
  const size_t shm = static_cast<size_t>(t) * eb * per_elem + 16;
  // PPO_GAE_KERNEL=reg / lds / pipe / chain forces the register-chunked, the whole-tile LDS, the
  // pipelined or the producer/consumer scan (experiments; read per call)
  const char *kv = getenv("PPO_GAE_KERNEL");
  const int kind = (kv && kv[0] == 'r') ? 1 : (kv && kv[0] == 'l') ? 2 : (kv && kv[0] == 'p') ? 3
                 : (kv && kv[0] == 'c') ? 4 : 0;
  // the producer / consumer scan is opt-in (PPO_GAE_KERNEL=chain): at N = 4096, T = 128 it ties the
  // pipelined scan by the engine's events (5.77 vs 5.80 us; rocprofv3 5.44 vs 5.72) and is slower
  // from 16384 envs (15.3 vs 12.8 us) -- tools/gae_sizes.py, profiles/r06
  if (kind == 4 && t <= 16 * 16) {
    // producer / consumer scan: 16 envs per block (32 from N = 16384 at T <= 128: every chunk's
    // delta / discount stays LDS-resident), + one chain wave
    const int peb = (n >= 16384 && t <= 16 * 8) ? 32 : 16;
    hipStream_t st = as_stream(stream);
    FreeTimingScope timing_scope;
    auto go = [&](auto rt_tag, auto eb_tag, auto k_tag) {
      using RT = decltype(rt_tag);
      constexpr int EB = decltype(eb_tag)::value, KM = decltype(k_tag)::value;
      const TimRec rec{KC_GAE,
                       tim_active() ? intern_name("gae_chain_kernel<%s, %d, %d>",
                                                  sizeof(RT) == 8 ? "double" : "float", EB, KM)
                                    : nullptr,
                       0.0, gae_bytes(sizeof(RT), done_d != nullptr, n, t)};
      launch_k(rec, gae_chain_kernel<RT, EB, KM>, dim3(ceil_div(n, EB)), dim3(EB * 16 + 64), 0, st,
               value_d, next_value_d, static_cast<const RT *>(reward_d), done_d, terminated_d,
               force_last_done, n, t, gamma_f, lg_f, adv_d, vtarget_d);
    };
    auto by_eb = [&](auto rt_tag) {
      if (t > 16 * 8) go(rt_tag, std::integral_constant<int, 16>{}, std::integral_constant<int, 16>{});
      else if (peb == 16) go(rt_tag, std::integral_constant<int, 16>{}, std::integral_constant<int, 8>{});
      else go(rt_tag, std::integral_constant<int, 32>{}, std::integral_constant<int, 8>{});
    };
    if (reward_is_f64) by_eb(double{});
    else by_eb(float{});
    PPO_LAUNCHED();
    return 0;
  }
  if ((kind == 0 || kind == 3) && t <= 16 * 16) {
    // pipelined scan: 16 envs per block (>= 256 blocks at N = 4096), 32 from N = 16384.
    // Measured (tools/gae_sweep.py, per-dispatch events, T = 128): N = 4096 6.2 us (LDS-staged
    // 9.2 us), 16384 12.7 us, 65536 37.7 us = 69 % of HBM (LDS-staged 42 %), 131072 60 %,
    // 1048576 58 % (register-chunked scan 38 % / 54 %); at T = 16 a launch still takes 4.8 us --
    // the load -> chain -> store latency floor that bounds N = 4096
    const int peb = (eb_knob == 8 || eb_knob == 16 || eb_knob == 32) ? eb_knob : (n >= 16384 ? 32 : 16);
    hipStream_t st = as_stream(stream);
    FreeTimingScope timing_scope;
    auto go = [&](auto rt_tag, auto eb_tag, auto k_tag) {
      using RT = decltype(rt_tag);
      constexpr int EB = decltype(eb_tag)::value, KM = decltype(k_tag)::value;
      const TimRec rec{KC_GAE,
                       tim_active() ? intern_name("gae_pipe_kernel<%s, %d, %d>",
                                                  sizeof(RT) == 8 ? "double" : "float", EB, KM)
                                    : nullptr,
                       0.0, gae_bytes(sizeof(RT), done_d != nullptr, n, t)};
      launch_k(rec, gae_pipe_kernel<RT, EB, KM>, dim3(ceil_div(n, EB)), dim3(EB * 16), 0, st,
               value_d, next_value_d, static_cast<const RT *>(reward_d), done_d, terminated_d,
               force_last_done, n, t, gamma_f, lg_f, adv_d, vtarget_d);
    };
    auto by_k = [&](auto rt_tag, auto eb_tag) {
      if (t <= 16 * 8) go(rt_tag, eb_tag, std::integral_constant<int, 8>{});
      else go(rt_tag, eb_tag, std::integral_constant<int, 16>{});
    };
    auto by_eb = [&](auto rt_tag) {
      if (peb == 8) by_k(rt_tag, std::integral_constant<int, 8>{});
      else if (peb == 16) by_k(rt_tag, std::integral_constant<int, 16>{});
      else by_k(rt_tag, std::integral_constant<int, 32>{});
    };
    if (reward_is_f64) by_eb(double{});
    else by_eb(float{});
    PPO_LAUNCHED();
    return 0;
  }
  // measured (tools/gae_sweep.py, T=128): LDS-staged wins up to N = 65,536, the register-
  // chunked scan from N = 262,144 (its ~16k waves stream near 4.2 TB/s)
  if (kind != 1 && n < 131072 && shm <= 131072 && t * eb <= 16 * 256) {
    const int blocks = ceil_div(n, eb);
    const int it = ceil_div(static_cast<int64_t>(t) * eb, 256);
    hipStream_t st = as_stream(stream);
    FreeTimingScope timing_scope;
    int rc = 0;
    auto pick_it = [&](auto rt_tag, auto eb_tag) {
      using RT = decltype(rt_tag);
      constexpr int EB = decltype(eb_tag)::value;
      const RT *r = static_cast<const RT *>(reward_d);
      auto go = [&](auto kernel, int it_max) {
        if (shm > 65536 &&
            hipFuncSetAttribute(reinterpret_cast<const void *>(kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                static_cast<int>(shm)) != hipSuccess) {
          rc = PPO_EHIP;
          set_error("ppo_gae: cannot raise dynamic LDS to %zu bytes", shm);
          return;
        }
        const TimRec rec{KC_GAE,
                         tim_active() ? intern_name("gae_lds_kernel<%s, %d, %d>",
                                                    sizeof(RT) == 8 ? "double" : "float", EB,
                                                    it_max)
                                      : nullptr,
                         0.0, gae_bytes(sizeof(RT), done_d != nullptr, n, t)};
        launch_k(rec, kernel, dim3(blocks), dim3(256), static_cast<uint32_t>(shm), st, value_d,
                 next_value_d, r, done_d, terminated_d, force_last_done, n, t, gamma_f, lg_f,
                 adv_d, vtarget_d);
      };
      if (it <= 4) go(gae_lds_kernel<RT, EB, 4>, 4);
      else if (it <= 8) go(gae_lds_kernel<RT, EB, 8>, 8);
      else go(gae_lds_kernel<RT, EB, 16>, 16);
    };
    auto pick_eb = [&](auto rt_tag) {
      switch (eb) {
        case 32: pick_it(rt_tag, std::integral_constant<int, 32>{}); break;
        case 16: pick_it(rt_tag, std::integral_constant<int, 16>{}); break;
        case 8: pick_it(rt_tag, std::integral_constant<int, 8>{}); break;
        case 4: pick_it(rt_tag, std::integral_constant<int, 4>{}); break;
        case 2: pick_it(rt_tag, std::integral_constant<int, 2>{}); break;
        default: pick_it(rt_tag, std::integral_constant<int, 1>{}); break;
      }
    };
    if (reward_is_f64) pick_eb(double{});
    else pick_eb(float{});
    if (rc) return rc;
    PPO_LAUNCHED();
    return 0;
  }
  const int grid = ceil_div(n, 64);
  FreeTimingScope timing_scope;
  const TimRec rec{KC_GAE,
                   reward_is_f64 ? "gae_kernel<double, 16>" : "gae_kernel<float, 16>", 0.0,
                   gae_bytes(reward_is_f64 ? 8 : 4, done_d != nullptr, n, t)};
  if (reward_is_f64)
    launch_k(rec, gae_kernel<double, 16>, dim3(grid), dim3(64), 0, as_stream(stream), value_d,
             next_value_d, static_cast<const double *>(reward_d), done_d, terminated_d,
             force_last_done, n, t, gamma_f, lg_f, adv_d, vtarget_d);
  else
    launch_k(rec, gae_kernel<float, 16>, dim3(grid), dim3(64), 0, as_stream(stream), value_d,
             next_value_d, static_cast<const float *>(reward_d), done_d, terminated_d,
             force_last_done, n, t, gamma_f, lg_f, adv_d, vtarget_d);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_normalize_rows(void *x_d, int is_f64, int n, int t, double scale,
                                  void *stream) {
  PPO_REQUIRE(x_d && n > 0 && t > 0, "ppo_normalize_rows: bad args");
  const int grid = ceil_div(n, 64);
  FreeTimingScope timing_scope;
  const double elems = static_cast<double>(n) * t;  // algorithmic: read once, write once
  if (is_f64)
    launch_k(TimRec{KC_ROWS, "normalize_rows_kernel<double>", 0.0, 16.0 * elems},
             normalize_rows_kernel<double>, dim3(grid), dim3(64), 0, as_stream(stream),
             static_cast<double *>(x_d), n, t, scale);
  else
    launch_k(TimRec{KC_ROWS, "normalize_rows_kernel<float>", 0.0, 8.0 * elems},
             normalize_rows_kernel<float>, dim3(grid), dim3(64), 0, as_stream(stream),
             static_cast<float *>(x_d), n, t, scale);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_obs_window_push(double *window_d, const void *obs_d, int obs_is_f64,
                                   const uint8_t *reset_d, int all_reset, int n, int o, int w,
                                   void *stream) {
  PPO_REQUIRE(window_d && obs_d && n > 0 && o > 0 && w > 0, "ppo_obs_window_push: bad args");
  const int64_t total = static_cast<int64_t>(n) * o;
  const int grid = ceil_div(total, 256);
  FreeTimingScope timing_scope;
  // algorithmic: read the new obs and the W-1 kept slots, write W slots (f64 window)
  const double by = static_cast<double>(total) * ((obs_is_f64 ? 8 : 4) + 8.0 * (2 * w - 1));
  if (obs_is_f64)
    launch_k(TimRec{KC_OBS, "obs_window_push_kernel<double>", 0.0, by},
             obs_window_push_kernel<double>, dim3(grid), dim3(256), 0, as_stream(stream),
             window_d, static_cast<const double *>(obs_d), reset_d, all_reset, n, o, w);
  else
    launch_k(TimRec{KC_OBS, "obs_window_push_kernel<float>", 0.0, by},
             obs_window_push_kernel<float>, dim3(grid), dim3(256), 0, as_stream(stream),
             window_d, static_cast<const float *>(obs_d), reset_d, all_reset, n, o, w);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_obs_normalize(const double *window_d, float *state_d, int n, int o, int w,
                                 const int32_t *bounds, int n_bounds, int normalize,
                                 void *stream) {
  PPO_REQUIRE(window_d && state_d && n > 0 && o > 0 && w > 0, "ppo_obs_normalize: bad args");
  PPO_REQUIRE(n_bounds >= 0 && n_bounds < 16, "ppo_obs_normalize: too many slices (%d)",
              n_bounds);
  SliceTable tab{};
  tab.count = n_bounds;
  for (int i = 0; i <= n_bounds && normalize; ++i) {
    PPO_REQUIRE(bounds != nullptr, "ppo_obs_normalize: null bounds");
    tab.edge[i] = bounds[i];
    PPO_REQUIRE(bounds[i] >= 0 && bounds[i] <= o && (i == 0 || bounds[i] >= bounds[i - 1]),
                "ppo_obs_normalize: bounds must be ascending within [0, O]");
  }
  const int64_t total = static_cast<int64_t>(n) * w;
  FreeTimingScope timing_scope;
  if (o > 32)  // obs_normalize_kernel holds a row in 32 registers
    launch_k(TimRec{KC_OBS, "obs_normalize_wide_kernel", 0.0, 12.0 * total * o},
             obs_normalize_wide_kernel, dim3(ceil_div(total * 64, 256)), dim3(256), 0,
             as_stream(stream), window_d, state_d, n, o, w, tab, normalize);
  else
    launch_k(TimRec{KC_OBS, "obs_normalize_kernel", 0.0, 12.0 * total * o}, obs_normalize_kernel,
             dim3(ceil_div(total, 128)), dim3(128), 0, as_stream(stream), window_d, state_d, n, o,
             w, tab, normalize);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_synthetic_env_step(const float *base_obs_d, const float *base_reward_d,
                                      const uint8_t *base_term_d, const float *action_d, int n,
                                      int o, int a, double *obs_out_d, double *reward_out_d,
                                      uint8_t *term_out_d, void *stream) {
  PPO_REQUIRE(base_obs_d && base_reward_d && base_term_d && action_d && obs_out_d &&
                  reward_out_d && term_out_d && n > 0 && o > 0 && a > 0 &&
                  static_cast<int64_t>(n) * std::max(o, a) < (int64_t{1} << 31),
              "ppo_synthetic_env_step: bad args");
  const int64_t total = static_cast<int64_t>(n) * o;
  FreeTimingScope timing_scope;
  launch_k(TimRec{KC_ENV, "synthetic_env_step_kernel", 0.0,
                  12.0 * total + 4.0 * n * a + 14.0 * n},
           synthetic_env_step_kernel, dim3(ceil_div(total, 256)), dim3(256), 0,
           as_stream(stream), base_obs_d, base_reward_d, base_term_d, action_d, n, o, a,
           obs_out_d, reward_out_d, term_out_d);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_synthetic_test_step(const float *base_obs_d, const float *base_reward_d,
                                       const uint8_t *base_term_d, int t_len, int n_envs,
                                       const float *action_d, int o, int a, int w,
                                       double *window_d, int32_t *step_d, double *reward_sum_d,
                                       uint8_t *term_out_d, void *stream) {
  PPO_REQUIRE(base_obs_d && base_reward_d && base_term_d && action_d && window_d && step_d &&
                  reward_sum_d && term_out_d && t_len > 0 && n_envs > 0 && o > 0 && a > 0 &&
                  w > 0,
              "ppo_synthetic_test_step: bad args");
  FreeTimingScope timing_scope;
  launch_k(TimRec{KC_ENV, "synthetic_test_step_kernel", 0.0, 4.0 * o + 8.0 * o * (2 * w - 1)},
           synthetic_test_step_kernel, dim3(1), dim3(256), 0, as_stream(stream), base_obs_d,
           base_reward_d, base_term_d, t_len, n_envs, action_d, o, a, w, window_d, step_d,
           reward_sum_d, term_out_d);
  PPO_LAUNCHED();
  return 0;
}

// ---- host physics pool transfers (north_star: pinned hipMemcpyAsync obs->GPU / action->CPU) ----
extern "C" int ppo_host_register(void *host, int64_t bytes) {
  PPO_REQUIRE(host && bytes > 0, "ppo_host_register: bad args");
  PPO_HIP_TRY(hipHostRegister(host, static_cast<size_t>(bytes), hipHostRegisterMapped));
  return 0;
}

extern "C" int ppo_host_device_ptr(void *host, void **dev) {
  PPO_REQUIRE(host && dev, "ppo_host_device_ptr: null");
  PPO_HIP_TRY(hipHostGetDevicePointer(dev, host, 0));
  return 0;
}

extern "C" int ppo_host_unregister(void *host) {
  PPO_REQUIRE(host, "ppo_host_unregister: null");
  PPO_HIP_TRY(hipHostUnregister(host));
  return 0;
}

// kind 1: host -> device, 2: device -> host; asynchronous on `stream` (host side pinned or
// registered for a true DMA)
extern "C" int ppo_memcpy_async(void *dst, const void *src, int64_t bytes, int kind, void *stream) {
  PPO_REQUIRE(dst && src && bytes >= 0 && (kind == 1 || kind == 2), "ppo_memcpy_async: bad args");
  if (bytes == 0) return 0;
  PPO_HIP_TRY(hipMemcpyAsync(dst, src, static_cast<size_t>(bytes),
                             kind == 1 ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost,
                             as_stream(stream)));
  return 0;
}

extern "C" int ppo_philox_normal(uint64_t seed, uint64_t offset, float *out_d, int64_t n,
                                 void *stream) {
  PPO_REQUIRE(out_d && n >= 0, "ppo_philox_normal: bad args");
  if (n == 0) return 0;
  FreeTimingScope timing_scope;
  const uint64_t *nul = nullptr;
  launch_k(TimRec{KC_ENV, "philox_normal_kernel", 0.0, 4.0 * n}, philox_normal_kernel,
           dim3(ceil_div(n, 256)), dim3(256), 0, as_stream(stream), seed, offset, nul, out_d, n);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_philox_normal_ctr(uint64_t seed, uint64_t offset, const uint64_t *counter_d,
                                     float *out_d, int64_t n, void *stream) {
  PPO_REQUIRE(out_d && n >= 0, "ppo_philox_normal_ctr: bad args");
  if (n == 0) return 0;
  FreeTimingScope timing_scope;  // the rollout's sampling noise: policy-head work
  launch_k(TimRec{KC_POLICY_HEAD, "philox_normal_kernel", 0.0, 4.0 * n}, philox_normal_kernel,
           dim3(ceil_div(n, 256)), dim3(256), 0, as_stream(stream), seed, offset, counter_d, out_d,
           n);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_perm_to_rows(const int64_t *perm_d, int64_t start, int b, int n_envs, int t,
                                int shard_lo, int shard_hi, int32_t *rows_d, int32_t *count_d,
                                void *stream) {
  PPO_REQUIRE(perm_d && rows_d && b > 0 && n_envs > 0 && t > 0, "ppo_perm_to_rows: bad args");
  PPO_REQUIRE(static_cast<int64_t>(n_envs) * t < (1ll << 31), "ppo_perm_to_rows: N*T overflows");
  if (shard_lo < shard_hi) {
    PPO_REQUIRE(count_d && shard_lo >= 0 && shard_hi <= n_envs,
                "ppo_perm_to_rows: bad shard [%d, %d)", shard_lo, shard_hi);
    FreeTimingScope timing_scope;
    launch_k(TimRec{KC_PERM, "perm_to_rows_shard_kernel", 0.0, 12.0 * b},
             perm_to_rows_shard_kernel, dim3(1), dim3(1024), 0, as_stream(stream), perm_d, start,
             b, n_envs, t, shard_lo, shard_hi, rows_d, count_d);
  } else {
    FreeTimingScope timing_scope;
    launch_k(TimRec{KC_PERM, "perm_to_rows_kernel", 0.0, 12.0 * b}, perm_to_rows_kernel,
             dim3(ceil_div(b, 256)), dim3(256), 0, as_stream(stream), perm_d, start, b, n_envs,
             t, rows_d);
  }
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_feistel_rows(uint64_t seed, uint64_t epoch, int64_t start, int b, int n_envs,
                                int t, int32_t *rows_d, void *stream) {
  PPO_REQUIRE(rows_d && b > 0 && n_envs > 0 && t > 0, "ppo_feistel_rows: bad args");
  const int64_t total = static_cast<int64_t>(n_envs) * t;
  PPO_REQUIRE(total < (1ll << 30), "ppo_feistel_rows: N*T too large");
  PPO_REQUIRE(start >= 0 && start + b <= total, "ppo_feistel_rows: slice out of range");
  int bits = 1;
  while ((1ll << bits) < total) ++bits;
  const int half = (bits + 1) / 2;
  FreeTimingScope timing_scope;
  launch_k(TimRec{KC_PERM, "feistel_rows_kernel", 0.0, 4.0 * b}, feistel_rows_kernel,
           dim3(ceil_div(b, 256)), dim3(256), 0, as_stream(stream), seed, epoch, start, b, n_envs,
           t, half, rows_d);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_adam(float *p_d, const float *g_d, float *m_d, float *v_d, int64_t n,
                        int64_t n_actor, float neg_step_actor, float neg_step_critic,
                        float one_minus_beta1, float beta2, float one_minus_beta2, float bc2_sqrt,
                        float eps, void *stream) {
  PPO_REQUIRE(p_d && g_d && m_d && v_d && n > 0 && n_actor >= 0 && n_actor <= n,
              "ppo_adam: bad args");
  FreeTimingScope timing_scope;
  // algorithmic: read p, g, m, v and write p, m, v (f32) = 28 B/param
  launch_k(TimRec{KC_ADAM, "adam_kernel", 0.0, 28.0 * n}, adam_kernel, dim3(ceil_div(n, 256)),
           dim3(256), 0, as_stream(stream), p_d, g_d, m_d, v_d, n, n_actor, neg_step_actor,
           neg_step_critic, one_minus_beta1, beta2, one_minus_beta2, bc2_sqrt, eps);
  PPO_LAUNCHED();
  return 0;
}

extern "C" int ppo_adam_sched(float *p_d, const float *g_d, float *m_d, float *v_d, int64_t n,
                              int64_t n_actor, const float *sched_d, float one_minus_beta1,
                              float beta2, float one_minus_beta2, float eps, void *stream) {
  PPO_REQUIRE(p_d && g_d && m_d && v_d && sched_d && n > 0 && n_actor >= 0 && n_actor <= n,
              "ppo_adam_sched: bad args");
  FreeTimingScope timing_scope;
  launch_k(TimRec{KC_ADAM, "adam_sched_kernel", 0.0, 28.0 * n}, adam_sched_kernel,
           dim3(ceil_div(n, 256)), dim3(256), 0, as_stream(stream), p_d, g_d, m_d, v_d, n, n_actor,
           sched_d, one_minus_beta1, beta2, one_minus_beta2, eps);
  PPO_LAUNCHED();
  return 0;
}
