// Shared helpers for the gfx950 PPO engine: error plumbing across the C-ABI, activation
// functions with torch's exact forward/backward forms, wave reductions.
//
// Compiled with -ffp-contract=off: every a*b+c below is two roundings unless fmaf() is written,
// which is what the reference's torch-CPU ops do (SURVEY.md s7 "Bit-exactness").
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ppo_engine.h"

namespace ppo {

void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

#define PPO_REQUIRE(cond, ...)          \
  do {                                  \
    if (!(cond)) {                      \
      ::ppo::set_error(__VA_ARGS__);    \
      return PPO_EINVAL;                \
    }                                   \
  } while (0)

#define PPO_HIP_TRY(call)                                                        \
  do {                                                                           \
    hipError_t e_ = (call);                                                      \
    if (e_ != hipSuccess) {                                                      \
      ::ppo::set_error("%s failed: %s", #call, hipGetErrorString(e_));           \
      return PPO_EHIP;                                                           \
    }                                                                            \
  } while (0)

#define PPO_LAUNCHED() PPO_HIP_TRY(hipGetLastError())

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

inline int ceil_div(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

// ---- activations (network_block_creator.py:54-55: config["activation"]()) -------------------
// Forward matches torch's CPU kernels; backward is expressed on the layer OUTPUT y, which is what
// the engine keeps in HBM (ReLU: threshold_backward(grad, y, 0); Tanh: grad*(1-y*y); ELU(alpha=1):
// y<=0 -> grad*(y+1), the is_result form of elu_backward).
__device__ __forceinline__ float act_forward(float x, int act) {
  // IEEE-2019 maximum (v_maximum3_f32): NaN propagates and -0 -> +0, as torch's x > 0 ? x : 0
  if (act == PPO_ACT_RELU) return __builtin_elementwise_maximum(x, 0.f);
  if (act == PPO_ACT_TANH) return tanhf(x);
  if (act == PPO_ACT_IDENTITY) return x;
  return x > 0.f ? x : expm1f(x);  // ELU alpha=1
}

__device__ __forceinline__ float act_backward(float grad, float y, int act) {
  if (act == PPO_ACT_RELU) return (y <= 0.f) ? 0.f : grad;
  if (act == PPO_ACT_TANH) return grad * (1.f - y * y);
  if (act == PPO_ACT_IDENTITY) return grad;
  return (y <= 0.f) ? grad * (y + 1.f) : grad;
}

// bf16 round trip (round-to-nearest-even, the hardware v_cvt_pk_bf16_f32): the operand rounding of
// precision mode PPO_PREC_BF16 in the kernels that multiply on the VALU (bf16 x bf16 is exact in
// f32, so an f32 FMA of rounded operands is the product an MFMA would form).
__device__ __forceinline__ float bf16_round(float x) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
  const f2_t f = {x, 0.f};
  const uint32_t u = __builtin_bit_cast(uint32_t, __builtin_convertvector(f, b2_t));
  return __uint_as_float(u << 16);
}

// ---- wave64 reductions (butterfly: every lane ends with the same, order-fixed sum) ------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// log(sqrt(2*pi)) as torch.distributions.Normal subtracts it (python double -> f32 scalar).
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;
// 0.5 + 0.5*log(2*pi): Normal.entropy's constant.
constexpr float kEntropyConst = 1.41893853320467274178f;

// ---- Philox4x32-10 + Box-Muller (perf-mode eps; parity mode takes host torch.randn) --------
__device__ __forceinline__ void philox_round(uint32_t &c0, uint32_t &c1, uint32_t &c2,
                                             uint32_t &c3, uint32_t k0, uint32_t k1) {
  const uint64_t p0 = static_cast<uint64_t>(0xD2511F53u) * c0;
  const uint64_t p1 = static_cast<uint64_t>(0xCD9E8D57u) * c2;
  const uint32_t hi0 = static_cast<uint32_t>(p0 >> 32), lo0 = static_cast<uint32_t>(p0);
  const uint32_t hi1 = static_cast<uint32_t>(p1 >> 32), lo1 = static_cast<uint32_t>(p1);
  c0 = hi1 ^ c1 ^ k0;
  c1 = lo1;
  c2 = hi0 ^ c3 ^ k1;
  c3 = lo0;
}

__device__ __forceinline__ void philox4x32_10(uint64_t ctr, uint64_t key, uint32_t out[4]) {
  uint32_t c0 = static_cast<uint32_t>(ctr), c1 = static_cast<uint32_t>(ctr >> 32), c2 = 0, c3 = 0;
  uint32_t k0 = static_cast<uint32_t>(key), k1 = static_cast<uint32_t>(key >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c0, c1, c2, c3, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

__device__ __forceinline__ float u32_to_open01(uint32_t x) {
  return (static_cast<float>(x >> 8) + 0.5f) * (1.0f / 16777216.0f);  // (0,1)
}

// Element i of the stream (seed, offset) is normal #((offset+i) % 4) of Philox block (offset+i)/4.
__device__ __forceinline__ float philox_normal_at(uint64_t seed, uint64_t idx) {
  uint32_t r[4];
  philox4x32_10(idx >> 2, seed, r);
  const int lane = static_cast<int>(idx & 3);
  const uint32_t ua = (lane < 2) ? r[0] : r[2];
  const uint32_t ub = (lane < 2) ? r[1] : r[3];
  const float rad = sqrtf(-2.f * logf(u32_to_open01(ua)));
  const float th = 6.28318530717958647692f * u32_to_open01(ub);
  return (lane & 1) ? rad * sinf(th) : rad * cosf(th);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// outstanding global loads and stores (__syncthreads drains vmcnt, so a prefetch meant to stay in
// flight across a phase, or a store nobody in the workgroup reads, stalls every barrier).  The
// wait and the barrier are ONE asm statement with a memory clobber (CK's block_sync_lds form): the
// compiler can neither put a memory operation between them nor move one across the pair in either
// direction; the scheduling barriers keep the machine scheduler from doing the same.
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

}  // namespace ppo
