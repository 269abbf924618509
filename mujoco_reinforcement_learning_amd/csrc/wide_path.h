// The wide layered path: the MLP actor-critic's rollout forward and minibatch forward + loss +
// backward with bf16-resident activations (PPO_PREC_BF16, ReLU nets the fused kernels do not
// cover, e.g. Humanoid 3x512 with O=376 and A=17).  Kernels: wide_gemm.h (products),
// wide_engine.hip (gather, heads, loss, weight images).  Entry points route here from
// ppo_policy_step / ppo_minibatch_grad / ppo_pack_weights (mlp_engine.hip) when wide_active().
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ctx.h"
#include "fused_policy.h"

namespace ppo {

struct WideNetWork {
  __bf16 *h[PPO_MAX_LAYERS];       // [rpad][ldh] hidden outputs (kept through the backward)
  __bf16 *dh[PPO_MAX_LAYERS];      // [rpad][ldh] dZ of hidden layer l (DGRAD of layer l + 1)
  int ldh[PPO_MAX_LAYERS];         // round_up(width, 64), pad columns stay zero
  __bf16 *w[PPO_MAX_LAYERS + 1];   // W image [round_up(out, 128)][round_up(in, 64)] (head: l = L)
  __bf16 *wt[PPO_MAX_LAYERS + 1];  // W^T image [round_up(in, 128)][round_up(out, 64)]
  int ldw[PPO_MAX_LAYERS + 1], ldwt[PPO_MAX_LAYERS + 1];
  float *colsum[PPO_MAX_LAYERS];   // [rpad / 64][out] bias-gradient partials per DGRAD row tile
  __bf16 *dz;                      // [rpad][64] head pre-activation gradients (bf16 operand)
  float *z;                        // [rpad][32] head pre-activations (f32)
  // rollout (wide_policy_fused_kernel): fragment-major W images, one 1 KB block of the 64 lanes'
  // 32x32x16 A fragments per (k-step, 32-feature tile); null when the fused rollout is off
  __bf16 *wf[PPO_MAX_LAYERS + 1];
  int wf_tiles[PPO_MAX_LAYERS + 1];  // 32-feature tiles (round_up(out, 32) / 32)
  int wf_ks[PPO_MAX_LAYERS + 1];     // 16-deep k-steps (round_up(in, 128) / 16)
};

struct WideWork {
  int rpad;                        // rows allocated: round_up(max_rows, 128)
  __bf16 *x;                       // [rpad][ldx] bf16 states (gathered minibatch / rollout rows)
  int ldx;                         // round_up(W*O, 128)
  bool fused_rollout;              // wide_policy_fused_kernel covers the nets (wide_alloc)
  WideNetWork net[2];
  float *part;                     // loss-kernel partials [blocks][kWidePart]
  float *loss_part;                // [blocks][2]
  int64_t img_elems;               // bf16 elements of all weight images (pack kernel extent)
  void *arena;
};

constexpr int kWideLossRows = 8;    // rows per loss-kernel block (32 lanes per row)
constexpr int kWidePart = 96;       // per block: logstd grads [0,32), actor head bias [32,64),
                                    // critic head bias [64]

// shapes the wide path covers (precision is checked at use)
bool wide_shapes_ok(const ppo_ctx *ctx);
bool wide_active(const ppo_ctx *ctx);
// allocate / free the workspace (outside graph capture)
int wide_alloc(ppo_ctx *ctx);
void wide_free(ppo_ctx *ctx);
// refresh the bf16 weight images from the f32 master parameters
// frag: also the fragment-major images of the fused rollout (before a rollout / policy step)
struct GatherArgs;  // wide_engine.hip: a minibatch's row staging, run in the same launch
int wide_pack(ppo_ctx *ctx, hipStream_t st, bool frag = true, const GatherArgs *gather = nullptr);
int wide_policy_step(ppo_ctx *ctx, const float *state_d, int n, const float *eps_d, uint64_t seed,
                     uint64_t offset, float *action_d, float *logp_d, float *value_d,
                     float *mean_d, bool pack, hipStream_t st,
                     bool staged = false);  // pack: refresh the images first; staged: x holds the rows
// rollout observation step in one launch: window push + standardisation + the bf16 operand rows
bool wide_observe_ok(const ppo_ctx *ctx, int n_slices);
int wide_observe(ppo_ctx *ctx, double *window_d, const double *obs_d, const uint8_t *reset_d,
                 int all_reset, const PolicySlices &tab, int normalize, float *state_d, int n,
                 hipStream_t st);
int wide_minibatch_grad(ppo_ctx *ctx, const float *states_d, const float *actions_d,
                        const float *old_logp_d, const float *adv_d, const float *vtarget_d,
                        const int32_t *rows_d, int b, const int32_t *count_d, float clip_lo,
                        float clip_hi, float entropy_coef, float inv_b, float inv_ba,
                        float *grad_d, float *loss_d, hipStream_t st);

}  // namespace ppo
