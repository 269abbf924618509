// The MLP actor-critic context (ppo_ctx, include/ppo_engine.h) and its layer descriptors, shared by
// the layered / fused engine (mlp_engine.hip) and the wide bf16-resident path (wide_engine.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ppo_engine.h"
#include "timing.h"

namespace ppo {

struct LayerDesc {
  int in, out;
  int64_t w_off, b_off;  // flat offsets (b_off < 0: no bias)
};

struct NetDesc {
  int n_hidden;
  LayerDesc layer[PPO_MAX_LAYERS + 1];  // hidden layers then the head
  int64_t begin, count;
  int64_t logstd_off;                   // actor only
  float *h[PPO_MAX_LAYERS];             // workspace: hidden outputs (max_rows, width)
  float *g;                             // workspace: dH_L
  float *dz;                            // workspace: head pre-activation grads (max_rows, out)
};

struct WideWork;  // wide_path.h

}  // namespace ppo

struct ppo_ctx {
  ppo_net_cfg cfg;
  int device;
  ppo::NetDesc net[2];
  int64_t total_params;
  float *params;
  float *slabs;          // (kSlabSplits, total_params)
  float *head_part;      // logstd partials (kHeadSplits, A) + loss partials (kHeadSplits, 2)
  float *head_w_part;    // fused head dW/db partials (kHeadSplits, hw_stride), UpdateHeadArgs
  const uint64_t *rng_counter;  // device Philox offset base (nullable), read at kernel run time
  int prec;                     // GEMM precision (ppo_ctx_set_precision), PPO_PREC_F32 default
  int hw_stride, hw_off_ba, hw_off_wc, hw_off_bc;
  float *xg;             // gathered minibatch states (max_rows, ldx)
  int ldx;               // round_up(W*O, 4)
  void *arena;
  // persistent fused update (bf16, two equal hidden layers; fused_update.hip)
  bool fused_ok;                // network shapes the fused kernel supports
  int fused_hidden;
  __bf16 *fw[2][3];             // per net: bf16 W0 image (H, 32), W1 (H, H), W1^T (H, H)
  __bf16 *fxb;                  // (max_rows, 32) staged bf16 states
  float *fsrow;                 // (max_rows, 16) staged row scalars
  float *fslabs;                // (kFusedMaxWG, total_params) partial gradients
  float *floss;                 // (kFusedMaxWG, 2) loss-term partials
  void *farena;
  uint4 *frec;                  // (frec_cap, 128 B) staged records (ppo_stage_records)
  int64_t frec_cap, frec_rows;
  uint64_t *fstamps;            // diagnostics: per-phase cycle sums (ppo_ctx_phase_stamps)
  int fstamp_on, fstamp_g;
  int fdirect;                  // ppo_ctx_fused_direct: the 8-wave kernel reads staged records via rows
  // which minibatch the gathered copy (fxb / fsrow) holds: the rows_d pointer and count of the
  // last staged gather (prep or step tail), nullptr when unknown -- PPO_STAGED_ROWS_GATHERED is
  // honoured only when it names exactly these rows, otherwise the entry point gathers again
  const int32_t *fg_rows;
  int fg_b;
  ppo::WideWork *wide;          // wide bf16-resident layered path (wide_path.h), or null
  ppo_comm *comm;               // data-parallel communicator (ppo_ctx_set_comm; not owned)
  float ent_log_share;          // ppo_ctx_loss_entropy_share (logged actor loss only)
  ppo::Timing tim;
};
