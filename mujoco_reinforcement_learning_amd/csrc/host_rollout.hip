// Native driver of the pipelined host-physics rollout (BASELINE
// north_star: "MuJoCo physics itself stays on the host cores as a vectorized subprocess pool with
// pinned hipMemcpyAsync obs->GPU / action->CPU overlapped on a side stream").
//
// Reference loop: running_gym_sequential_vectorized.py:40-59 (step the VecEnv, shift + append
// each env's window) driven by ppo.py:13-60 (one PPOAgent.act + get_state_value per step).  The
// engine splits the N envs into worker groups (host_pool.HostPhysicsPool) and runs, per step and
// group g, all from this one host thread -- no Python between the hand-offs:
//
//   GPU   host_ingest_kernel   the group's last-step rewards / terminations, read zero-copy from
//                              the page-locked shared memory into the rollout buffer
//   GPU   ppo_observe_act      window push + standardise + act on its rows, the new
//                              observations read zero-copy from the shared memory
//   GPU   host_egress_kernel   its actions written zero-copy into the shared memory
//   host  (event completes)    release the group's workers (generation word), wait for their
//                              done words, enqueue the group's next step
//
// Every transfer is a PCIe load or store inside a kernel on the one compute stream: no DMA
// submissions, no cross-stream events -- per hand-off three launches and one event.  Group 1's
// GPU work runs while group 0's physics is on the host cores, and the other way round.  Same
// rows, noise offsets and values as the Python protocol (HostPhysicsVecEnvHelper.begin_half /
// release_half / finish_half), tested bit for bit against the device env.
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "timing.h"

namespace {

constexpr int kCtrlT = 0, kCtrlGen = 2;  // host_pool.py control word layout (step, stop, gen)

// rewards (f64) and terminations (u8) of `rows` envs: shared memory (device-mapped) -> buffer
__global__ void host_ingest_kernel(const double *__restrict__ reward_h,
                                   const uint8_t *__restrict__ term_h, double *__restrict__ reward_d,
                                   uint8_t *__restrict__ term_d, int rows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < rows) {
    reward_d[i] = reward_h[i];
    term_d[i] = term_h[i];
  }
}

// the group's actions: rollout buffer -> shared memory (device-mapped), 16-B stores
__global__ void host_egress_kernel(const float *__restrict__ act_d, float *__restrict__ act_h,
                                   int64_t count) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (4 * i + 3 < count) {
    reinterpret_cast<float4 *>(act_h)[i] = reinterpret_cast<const float4 *>(act_d)[i];
  } else {
    for (int64_t k = 4 * i; k < count; ++k) act_h[k] = act_d[k];
  }
}

struct Side {
  hipEvent_t done = nullptr;  // the group's actions are in host memory
};

}  // namespace

extern "C" int ppo_host_rollout(ppo_ctx *ctx, ppo_host_pool_desc *pool, double *window_d,
                                const int32_t *bounds, int n_bounds, int normalize,
                                float *states_d, float *actions_d, float *logp_d, float *values_d,
                                double *reward_d, uint8_t *term_d, double *obs_next_d, int n,
                                int obs_dim, int window, int act_dim, int horizon,
                                const float *eps_d, uint64_t seed, uint64_t base_offset,
                                void *stream) {
  PPO_REQUIRE(ctx && pool && window_d && states_d && actions_d && logp_d && values_d && reward_d &&
                  term_d && obs_next_d,
              "ppo_host_rollout: null argument");
  PPO_REQUIRE(pool->groups >= 1 && pool->groups <= PPO_MAX_GROUPS,
              "ppo_host_rollout: %d groups", pool->groups);
  PPO_REQUIRE(pool->ctrl && pool->done && pool->action_dev && pool->obs_dev &&
                  pool->reward_dev && pool->term_dev,
              "ppo_host_rollout: pool shared-memory pointers missing");
  PPO_REQUIRE(n > 0 && horizon > 0 && obs_dim > 0 && window > 0 && act_dim > 0,
              "ppo_host_rollout: bad shape");
  for (int g = 0; g < pool->groups; ++g)
    PPO_REQUIRE(pool->group_lo[g] >= 0 && pool->group_lo[g] < pool->group_hi[g] &&
                    pool->group_hi[g] <= n && pool->worker_lo[g] < pool->worker_hi[g],
                "ppo_host_rollout: group %d bounds", g);
  const int G = pool->groups, O = obs_dim, W = window, A = act_dim;
  const int64_t din = static_cast<int64_t>(W) * O;
  hipStream_t cs = ppo::as_stream(stream);
  Side side[PPO_MAX_GROUPS];
  int rc = 0;
  auto fail = [&](hipError_t e, const char *what) {
    ppo::set_error("ppo_host_rollout: %s failed: %s", what, hipGetErrorString(e));
    rc = PPO_EHIP;
  };
  for (int g = 0; g < G && !rc; ++g) {
    const hipError_t e = hipEventCreateWithFlags(&side[g].done, hipEventDisableTiming);
    if (e != hipSuccess) fail(e, "event creation");
  }

  // group g at step t: (pushed) ingest the last step's rewards / terminations, observe + act
  // with the observations read from the shared memory, actions back into the shared memory, the
  // group's completion event (t == horizon: the bootstrap value only)
  auto act = [&](int t, int g, bool pushed) -> int {
    const int lo = pool->group_lo[g], hi = pool->group_hi[g], rows = hi - lo;
    const int64_t r0 = static_cast<int64_t>(t) * n + lo;
    const bool last = t == horizon;
    const double *obs = nullptr;
    const uint8_t *reset = nullptr;
    if (pushed) {
      const int64_t rp = static_cast<int64_t>(t - 1) * n + lo;
      ppo::launch_k(ppo::TimRec{ppo::KC_OBS, "host_ingest_kernel", 0.0, 9.0 * 2 * rows}, host_ingest_kernel,
               dim3(ppo::ceil_div(rows, 256)), dim3(256), 0, cs, pool->reward_dev + lo,
               pool->term_dev + lo, reward_d + rp, term_d + rp, rows);
      PPO_LAUNCHED();
      obs = pool->obs_dev + static_cast<int64_t>(lo) * O;
      reset = term_d + rp;
    }
    if (int r = ppo_observe_act(ctx, window_d + static_cast<int64_t>(lo) * O * W, obs, reset, 0,
                                bounds, n_bounds, normalize, states_d + r0 * din, rows,
                                (last || !eps_d) ? nullptr : eps_d + r0 * A, seed,
                                base_offset + static_cast<uint64_t>(r0) * A,
                                last ? nullptr : actions_d + r0 * A, last ? nullptr : logp_d + r0,
                                values_d + r0, nullptr, stream))
      return r;
    if (last) return 0;
    const int64_t count = static_cast<int64_t>(rows) * A;
    ppo::launch_k(ppo::TimRec{ppo::KC_OBS, "host_egress_kernel", 0.0, 8.0 * count}, host_egress_kernel,
             dim3(ppo::ceil_div((count + 3) / 4, 256)), dim3(256), 0, cs, actions_d + r0 * A,
             pool->action_dev + static_cast<int64_t>(lo) * A, count);
    PPO_LAUNCHED();
    PPO_HIP_TRY(hipEventRecord(side[g].done, cs));
    return 0;
  };
  // host: the group's actions have landed (its event completed) -> release its workers
  auto release = [&](int t, int g) -> int {
    int64_t *ctrl = pool->ctrl + 3 * g;
    __atomic_store_n(&ctrl[kCtrlT], static_cast<int64_t>(t), __ATOMIC_RELAXED);
    __atomic_store_n(&ctrl[kCtrlGen], ++pool->gen[g], __ATOMIC_RELEASE);
    return 0;
  };

  // Event-driven: each group advances as soon as its own next hand-off is ready (its actions have
  // landed -> release its workers; its workers are done -> results up + its next observe + act),
  // so a slow group never holds the other's GPU work behind it.  Groups own disjoint rows, and
  // every row's noise offset is fixed, so the interleaving does not change any value.
  enum { kActed, kRunning, kDone };
  int state[PPO_MAX_GROUPS], step[PPO_MAX_GROUPS];
  for (int g = 0; g < G && !rc; ++g) {
    rc = act(0, g, false);
    state[g] = kActed;
    step[g] = 0;
  }
  const auto t0 = std::chrono::steady_clock::now();
  // Watchdog: the call fails only when NO group has advanced for the stall limit (default 120 s,
  // PPO_HOST_ROLLOUT_STALL_MS overrides it per call), however long the whole rollout takes.
  const char *stall_env = getenv("PPO_HOST_ROLLOUT_STALL_MS");
  const long stall_ms = stall_env ? std::max(1L, atol(stall_env)) : 120000L;
  auto last_progress = t0;
  // PPO_HOST_ROLLOUT_STATS=1: per-phase host wall time (diagnostics on stderr)
  static const bool stats = getenv("PPO_HOST_ROLLOUT_STATS") != nullptr;
  double w_d2h = 0, w_phys = 0, w_enq = 0;
  auto since = [&](std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
  };
  std::chrono::steady_clock::time_point mark[PPO_MAX_GROUPS];
  for (int g = 0; g < G; ++g) mark[g] = t0;
  int remaining = G;
  bool stalled = false;
  for (long spins = 0; remaining > 0 && !rc; ++spins) {
    bool progress = false;
    for (int g = 0; g < G && !rc; ++g) {
      if (state[g] == kActed) {
        const hipError_t q = hipEventQuery(side[g].done);
        if (q == hipErrorNotReady) continue;
        if (q != hipSuccess) {
          fail(q, "hipEventQuery");
          break;
        }
        if (stats) {
          w_d2h += since(mark[g]);
          mark[g] = std::chrono::steady_clock::now();
        }
        rc = release(step[g], g);
        state[g] = kRunning;
        progress = true;
      } else if (state[g] == kRunning) {
        bool all = true;
        for (int w = pool->worker_lo[g]; w < pool->worker_hi[g] && all; ++w)
          all = __atomic_load_n(&pool->done[w], __ATOMIC_ACQUIRE) == pool->gen[g];
        if (!all) continue;
        std::chrono::steady_clock::time_point e0;
        if (stats) {
          w_phys += since(mark[g]);
          e0 = std::chrono::steady_clock::now();
        }
        rc = act(step[g] + 1, g, true);
        if (stats) {
          w_enq += since(e0);
          mark[g] = std::chrono::steady_clock::now();
        }
        ++step[g];
        state[g] = step[g] == horizon ? kDone : kActed;
        if (state[g] == kDone) --remaining;
        progress = true;
      }
    }
    if (progress) {
      last_progress = std::chrono::steady_clock::now();
    } else if ((spins & 1023) == 1023) {
      sched_yield();
      if (std::chrono::steady_clock::now() - last_progress > std::chrono::milliseconds(stall_ms)) {
        ppo::set_error("ppo_host_rollout: no group advanced for %ld ms (a host physics worker "
                       "died or stalled)", stall_ms);
        rc = PPO_EHIP;
        stalled = true;
      }
    }
  }
  if (stalled) {
    // Released groups' workers may still be writing the shared memory: give them a grace period
    // (the stall limit again) to publish, so a caller that closes or reuses the pool after the
    // error does not race them; report the pool unusable when they do not.
    const auto g0 = std::chrono::steady_clock::now();
    bool settled = false;
    while (!settled && std::chrono::steady_clock::now() - g0 < std::chrono::milliseconds(stall_ms)) {
      settled = true;
      for (int g = 0; g < G; ++g) {
        if (state[g] != kRunning) continue;
        for (int w = pool->worker_lo[g]; w < pool->worker_hi[g]; ++w)
          settled = settled && __atomic_load_n(&pool->done[w], __ATOMIC_ACQUIRE) == pool->gen[g];
      }
      if (!settled) sched_yield();
    }
    if (!settled)
      ppo::set_error("ppo_host_rollout: no group advanced for %ld ms and released workers did not "
                     "finish; the pool is unusable (close it)", stall_ms);
  }
  if (stats)
    fprintf(stderr,
            "ppo_host_rollout: %d steps x %d groups, %.1f us total; per group-step: act enqueue -> "
            "actions on host %.1f us, release -> physics done %.1f us, results + act enqueue %.1f us\n",
            horizon, G, since(t0), w_d2h / (horizon * G), w_phys / (horizon * G),
            w_enq / (horizon * G));
  // the shared memory may be reused by the caller right away: drain the last reads of it
  if (hipStreamSynchronize(cs) != hipSuccess && !rc) fail(hipGetLastError(), "hipStreamSynchronize");
  for (int g = 0; g < G; ++g)
    if (side[g].done) (void)hipEventDestroy(side[g].done);
  return rc;
}
