// Fused bf16 rollout policy step (fused_policy.hip): host-side argument block and launcher.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "fused_update.h"
#include "timing.h"

namespace ppo {

constexpr int kPolicyMaxWindow = 1;  // one net per workgroup: both read the window, W=1 only

struct PolicySlices {  // feature-slice edges of the per-sample standardisation (A1)
  int32_t edge[16];
  int32_t count;
};

struct PolicyFusedArgs {
  FusedNet net[2];               // bf16 W0 / W1 images + f32 biases and heads (w1bt unused)
  const float *logstd;
  int n, obs_dim, window, act_dim, act, hidden;
  float omv;
  // A1: window (N, O, W) f64 updated in place when obs_d != null (push), reset_d / all_reset as
  // ppo_obs_window_push; the standardised state (N, W*O) f32 is written to state_d
  double *window_d;
  const double *obs_d;
  const uint8_t *reset_d;
  int all_reset;
  PolicySlices tab;
  int normalize;
  float *state_d;
  // A2-A4 (each output nullable)
  int do_actor, do_critic;
  const float *eps;
  uint64_t seed, offset;
  const uint64_t *offset_base;
  uint64_t *stamps;              // diagnostics (ReLU only): (2, 128, 11) per-phase cycles, or null
  float *action, *logp, *value, *mean;
};

int policy_fused_launch(const PolicyFusedArgs &q, const TimRec &rec, hipStream_t st);

}  // namespace ppo
