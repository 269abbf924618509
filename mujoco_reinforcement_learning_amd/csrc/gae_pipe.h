// The pipelined GAE + value-target scan (torchrl 0.6.0 generalized_advantage_estimate, called at
// ppo.py:70-80), shared by gae_pipe_kernel (scan_kernels.hip) and gae_records_kernel
// (fused_update.hip, the scan fused with the staged-record pass).  Semantics: scan_kernels.hip's
// GAE header comment (f64 carry when the rewards are f64, two roundings, no FMA).
//
// A block of EB*16 threads owns EB envs and walks the horizon backwards in chunks of TC = 16 time
// rows, thread (tt, c) holding slot k = time row T-1-(16k+tt) of env c.  Every load of every slot
// is issued up front (chunk 0 first, so chunk 0 lands first chip-wide); then per chunk: delta and
// the discount go to LDS, ONE barrier, the EB chain lanes run the chunk's 16 dependent steps while
// every thread stores the previous chunk's adv / vtarget (the chain that produced them finished
// before the barrier).  The chain starts when the first chunk has landed instead of after the
// whole tile, and the stores drain under the chain.
//
// Emit hooks ride the same schedule: em.load(buf, row, ok) in chunk k's iteration, before the
// barrier (row = t*N + env of the slot, clamped valid when !ok), and em.store(buf, row, a, vt)
// next to that row's adv / vtarget store one iteration later; buf = k & 1 is a compile-time
// constant under the unrolled chunk loop, so an emitter can double-buffer per-row operands in
// registers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"

namespace ppo {

struct GaeNoEmit {
  __device__ __forceinline__ void load(int, int64_t, bool) {}
  __device__ __forceinline__ void store(int, int64_t, float, float) {}
};

template <typename RT, int EB, int KMAX, class Emit>
__device__ __forceinline__ void gae_pipe_body(const float *__restrict__ value,
                                              const float *__restrict__ next_value,
                                              const RT *__restrict__ reward,
                                              const uint8_t *__restrict__ done,
                                              const uint8_t *__restrict__ term, int force_last,
                                              int n, int t_len, float gamma_f, float lg_f,
                                              float *__restrict__ adv, float *__restrict__ vtarget,
                                              Emit &em) {
  constexpr int TC = 16;
  __shared__ RT s_d[2][TC][EB];     // delta
  __shared__ RT s_q[2][TC][EB];     // (RT) disc
  __shared__ float s_o[2][TC][EB];  // f32 advantage
  const int tid = threadIdx.x, c = tid % EB, tt = tid / EB;
  const int env = blockIdx.x * EB + c;
  float lv[KMAX], lvn[KMAX];
  RT lr[KMAX];
  uint8_t ltm[KMAX], ldn[KMAX];
  // unconditional loads from clamped (valid) addresses: no branches or register merges between
  // them, so every load of every slot is in flight before the first use
  const int envc = env < n ? env : n - 1;
  const uint8_t *const dsrc = done ? done : term;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    const int t = t_len - 1 - (TC * k + tt);
    const int64_t idx = static_cast<int64_t>(t >= 0 ? t : 0) * n + envc;
    lv[k] = value[idx];
    lvn[k] = next_value[idx];
    lr[k] = reward[idx];
    ltm[k] = term[idx];
    ldn[k] = dsrc[idx];
  }
  RT prev = 0;
  // a fixed KMAX chunks (no data-dependent control flow, so no load is sunk into a branch);
  // rows t < 0 (T < 16 KMAX) carry delta = disc = 0 and come after t = 0 in the chain
#pragma unroll
  for (int k = 0; k <= KMAX; ++k) {
    const int buf = k & 1;
    if (k < KMAX) {
      const int t = t_len - 1 - (TC * k + tt);
      const float g_nt = gamma_f * (ltm[k] ? 0.f : 1.f);
      const float gv = g_nt * lvn[k];
      const RT delta = (lr[k] + static_cast<RT>(gv)) - static_cast<RT>(lv[k]);
      const bool is_done = ldn[k] != 0 || (force_last && t == t_len - 1);
      const RT q = static_cast<RT>(lg_f * (is_done ? 0.f : 1.f));
      const bool ok = t >= 0 && env < n;
      s_d[buf][tt][c] = ok ? delta : static_cast<RT>(0);
      s_q[buf][tt][c] = ok ? q : static_cast<RT>(0);
      em.load(buf, static_cast<int64_t>(t >= 0 ? t : 0) * n + envc, ok);
    }
    lds_sync();  // LDS hand-off only: the record loads and the previous chunk's stores stay in flight
    if (k < KMAX && tid < EB) {  // the chain: rows of this chunk in descending time
      RT d[TC], qq[TC];
#pragma unroll
      for (int j = 0; j < TC; ++j) {
        d[j] = s_d[buf][j][tid];
        qq[j] = s_q[buf][j][tid];
      }
#pragma unroll
      for (int j = 0; j < TC; ++j) {
        prev = d[j] + prev * qq[j];
        s_o[buf][j][tid] = static_cast<float>(prev);
      }
    }
    if (k > 0) {  // chunk k-1: its chain ran before this iteration's barrier
      const int kp = k - 1;
      const int t = t_len - 1 - (TC * kp + tt);
      if (t >= 0 && env < n) {
        const int64_t idx = static_cast<int64_t>(t) * n + env;
        const float a = s_o[buf ^ 1][tt][c];
        const float vt = a + lv[kp];  // value_target = advantage + state_value (f32)
        adv[idx] = a;
        vtarget[idx] = vt;
        em.store(buf ^ 1, idx, a, vt);
      }
    }
  }
}

// Producer / consumer form of the same scan (gae_chain_kernel, round 6): the EB*16 producer threads
// lay out and load exactly as gae_pipe_body, compute delta / discount for EVERY chunk as its loads
// land and publish each chunk through an LDS counter (no barrier: a producer never waits for the
// chain before the stores); one extra chain wave (lanes 0..EB-1, one env each) consumes the
// chunks in order -- 16 dependent f64 steps per chunk, the same operations in the same order as
// gae_pipe_body's chain -- and publishes its results per chunk; the producers then store adv /
// vtarget.  Bit-exact with gae_pipe_body.  Every spin is bounded (a lost update ends the kernel
// with wrong values, which the bit-exact tests catch, instead of hanging the GPU).
template <typename RT>
struct GaeDQ {
  RT d, q;
};

__device__ __forceinline__ int lds_load_relaxed(const int *p) {
  return __atomic_load_n(p, __ATOMIC_RELAXED);
}

template <typename RT, int EB, int KMAX>
__device__ __forceinline__ void gae_chain_body(const float *__restrict__ value,
                                               const float *__restrict__ next_value,
                                               const RT *__restrict__ reward,
                                               const uint8_t *__restrict__ done,
                                               const uint8_t *__restrict__ term, int force_last,
                                               int n, int t_len, float gamma_f, float lg_f,
                                               float *__restrict__ adv, float *__restrict__ vtarget) {
  constexpr int TC = 16, NP = EB * TC, PW = NP / 64;
  static_assert(NP % 64 == 0, "whole producer waves");
  constexpr int kSpin = 1 << 20;  // bound on every wait (64-cycle sleeps: about 30 ms)
  __shared__ GaeDQ<RT> s_dq[KMAX][TC][EB];
  __shared__ float s_o[KMAX][TC][EB];
  __shared__ int s_in[KMAX];  // producer waves that published chunk k
  __shared__ int s_out;       // chunks the chain has finished
  const int tid = threadIdx.x;
  if (tid < KMAX) s_in[tid] = 0;
  if (tid == KMAX) s_out = 0;
  __syncthreads();
  if (tid >= NP) {  // the chain wave
    const int c = tid - NP;
    if (c < EB) {
      RT prev = 0;
      for (int k = 0; k < KMAX; ++k) {
        for (int it = 0; it < kSpin && lds_load_relaxed(&s_in[k]) < PW; ++it) __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
        RT d[TC], q[TC];
#pragma unroll
        for (int j = 0; j < TC; ++j) {
          const GaeDQ<RT> v = s_dq[k][j][c];
          d[j] = v.d;
          q[j] = v.q;
        }
#pragma unroll
        for (int j = 0; j < TC; ++j) {
          prev = d[j] + prev * q[j];
          s_o[k][j][c] = static_cast<float>(prev);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the results are in LDS
        asm volatile("" ::: "memory");
        if (c == 0) __atomic_store_n(&s_out, k + 1, __ATOMIC_RELAXED);
      }
    }
    return;
  }
  const int c = tid % EB, tt = tid / EB;
  const int env = blockIdx.x * EB + c;
  float lv[KMAX], lvn[KMAX];
  RT lr[KMAX];
  uint8_t ltm[KMAX], ldn[KMAX];
  const int envc = env < n ? env : n - 1;
  const uint8_t *const dsrc = done ? done : term;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    const int t = t_len - 1 - (TC * k + tt);
    const int64_t idx = static_cast<int64_t>(t >= 0 ? t : 0) * n + envc;
    lv[k] = value[idx];
    lvn[k] = next_value[idx];
    lr[k] = reward[idx];
    ltm[k] = term[idx];
    ldn[k] = dsrc[idx];
  }
  // chunk j's results stored LAG chunks after j is published (the chain runs about a chunk
  // behind), so the stores stream out while later chunks still load; the waits spin on LDS only
  // (no vector-memory op inside a branch, so the loads' vmcnt schedule stays static)
  constexpr int LAG = 2;
  auto store_chunk = [&](int k) {
    for (int it = 0; it < kSpin && lds_load_relaxed(&s_out) <= k; ++it) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
    const int t = t_len - 1 - (TC * k + tt);
    const int64_t idx = static_cast<int64_t>(t >= 0 ? t : 0) * n + envc;
    const float a = s_o[k][tt][c];
    if (t >= 0 && env < n) {
      adv[idx] = a;
      vtarget[idx] = a + lv[k];  // value_target = advantage + state_value (f32)
    }
  };
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {  // publish chunk k as soon as its loads have landed
    const int t = t_len - 1 - (TC * k + tt);
    const float g_nt = gamma_f * (ltm[k] ? 0.f : 1.f);
    const float gv = g_nt * lvn[k];
    const RT delta = (lr[k] + static_cast<RT>(gv)) - static_cast<RT>(lv[k]);
    const bool is_done = ldn[k] != 0 || (force_last && t == t_len - 1);
    const RT q = static_cast<RT>(lg_f * (is_done ? 0.f : 1.f));
    const bool ok = t >= 0 && env < n;
    s_dq[k][tt][c] = GaeDQ<RT>{ok ? delta : static_cast<RT>(0), ok ? q : static_cast<RT>(0)};
    __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's writes of chunk k are in LDS
    asm volatile("" ::: "memory");
    if ((tid & 63) == 0) __atomic_fetch_add(&s_in[k], 1, __ATOMIC_RELAXED);
    if (k >= LAG) store_chunk(k - LAG);
  }
#pragma unroll
  for (int k = KMAX - LAG; k < KMAX; ++k) {
    if (k >= 0) store_chunk(k);
  }
}

}  // namespace ppo
