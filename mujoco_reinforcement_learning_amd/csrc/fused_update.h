// Persistent fused minibatch update (precision mode bf16, two equal hidden layers): host-side
// argument block and launchers, shared by mlp_engine.hip (ppo_minibatch_grad) and
// fused_update.hip (the kernels).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "reduce_slabs.h"
#include "timing.h"

namespace ppo {

constexpr int kFusedRows = 64;      // minibatch rows per chunk (one LDS-resident tile)
constexpr int kFusedKX = 32;        // layer-0 input width padded for the 32x32x16 MFMA
constexpr int kFusedSP = 16;        // per-row scalar pitch: actions[A], old_logp, adv, vtarget
constexpr int kFusedMaxAct = 8;
constexpr int kFusedMaxWG = 128;    // workgroups (= partial-gradient slabs) per net
// phase-stamp slots per workgroup: 10 chunk-loop phases, prologue, epilogue (slab stores
// drained), and the body's s_memrealtime ticks (100 MHz) for the cycle -> time calibration
constexpr int kStampSlots = 13;

struct FusedNet {
  const __bf16 *w0b;   // (H, 32)  bf16(W0), input columns >= din zero
  const __bf16 *w1b;   // (H, H)   bf16(W1)
  const __bf16 *w1bt;  // (H, H)   bf16(W1)^T
  const float *w0, *w1;        // f32 masters (prep kernel source)
  const float *b0, *b1;        // hidden biases (nullable: NetworkConfig.use_bias = False)
  const float *wh, *bh;        // head (A_net, H) f32, bias (A_net) (nullable)
  int64_t off_w0, off_b0, off_w1, off_b1, off_wh, off_bh;  // flat offsets (b: -1 = none)
};

// One 128 B record per stored row: bf16 state[32] (columns >= din zero) | f32 actions[A],
// old_logp, adv, vtarget, zeros -- the per-row image the prep gather copies.
constexpr int kRecordBytes = 2 * kFusedKX + 4 * kFusedSP;
static_assert(kRecordBytes == 128, "one record per 128 B line");
int fused_records_launch(uint4 *rec, const float *states, const float *actions,
                         const float *old_logp, const float *adv, const float *vtarget,
                         int64_t n_rows, int din, int act_dim, const TimRec &trec, hipStream_t st);

// GAE + value target (gae_pipe.h) with the records staged in the same pass (gae_records_kernel):
// rows t*n + env of the (t_len, n) time-major arrays.
struct GaeRecordArgs {
  const float *value, *next_value;
  const void *reward;  // f32 or f64 (reward_f64)
  const uint8_t *done, *term;
  int force_last, n, t_len;
  float gamma_f, lg_f;
  float *adv, *vtarget;
  const float *states, *actions, *old_logp;
  uint4 *rec;
  int din, act_dim;
};
int gae_records_launch(const GaeRecordArgs &g, bool reward_f64, const TimRec &rec,
                       hipStream_t st);

// Adam over the flat parameters of both nets (adam_elem) that also writes the updated values
// into the fused kernels' bf16 weight images, so the next minibatch needs no weight refresh.
struct AdamPackArgs {
  float *p;
  const float *g;
  float *m, *v;
  int64_t n, n_actor;
  const float *sched;          // device (neg_step_actor, neg_step_critic, bc2_sqrt), or null
  float neg_a, neg_c, bc2;     // host scalars when sched is null
  float w1, b2, omb2, eps;
  __bf16 *w0b[2], *w1b[2], *w1bt[2];
  int64_t off_w0[2], off_w1[2];
  int din, H;
};
int adam_pack_launch(const AdamPackArgs &a, const TimRec &rec, hipStream_t st);

// The single-rank optimizer-step tail of a staged minibatch, in one launch: blocks
// [0, ceil(P/256)) fold the slabs (reduce_slab_block) and apply Adam + the weight-image refresh
// to the parameters they just reduced (a.g is the reduced gradient, also written); the remaining
// blocks gather the NEXT minibatch's rows from the staged records (b = 0: none).
struct TailArgs {
  AdamPackArgs a;
  const int32_t *rows;
  const uint4 *rec;
  int64_t n_rec;
  __bf16 *xb;
  float *srow;
  int b;
  bool reduce;  // false: no slab reduction, Adam on the gradient already in a.g (data parallel)
};
int step_tail_launch(const ReduceArgs &r, const TailArgs &t, const TimRec &rec, hipStream_t st);

struct FusedArgs {
  FusedNet net[2];             // 0 actor, 1 critic
  const float *logstd;
  int64_t off_logstd;
  // minibatch staged by fused_prep_kernel (rows >= count are zero)
  __bf16 *xb;                  // (b, 32) bf16 states
  float *srow;                 // (b, 16) f32 actions[A], old_logp, adv, vtarget
  // prep sources: time-major storage arrays gathered through rows
  const float *states, *actions, *old_logp, *adv, *vtarget;
  const int32_t *rows;
  const int32_t *rows_n;       // device row count (exact data parallel), nullable -> b
  // staged records (fused_records_launch): when set, the prep gather copies one 128 B record
  // per row instead of reading the five storage arrays
  const uint4 *rec;
  int64_t n_rec;
  // direct (rec set, 8-wave kernel): the fused kernel reads each row's record through rows[]
  // itself, one chunk ahead -- no gathered xb / srow copy is written or read
  bool direct;
  bool pack_w;                 // prep also refreshes the bf16 weight images from the masters
  int b, din, act_dim, act, hidden;
  float omv, clip_lo, clip_hi, ent_coef, inv_b, inv_ba;
  float *slabs;                // (G, slab_stride) partial gradients in the flat layout
  int64_t slab_stride;
  float *loss_part;            // (G, 2): actor / critic loss-term sums per workgroup
  int G;                       // workgroups per net
  uint64_t *stamps;            // diagnostics: (2, G, 11) per-phase cycle sums, or null
};
// Gather the minibatch (bf16 states + row scalars) and, with q.pack_w, refresh the bf16 weight
// images.
int fused_prep_launch(const FusedArgs &q, const TimRec &rec, hipStream_t st);
// The persistent fused forward + loss + backward kernel.  grid (G, 2), 512 threads.
int fused_update_launch(const FusedArgs &q, const TimRec &rec, hipStream_t st);
// Supported hidden widths (compiled instantiations).
bool fused_width_ok(int hidden);
// The phase schedule the fused kernel runs for activation `act` (its SCHED template argument:
// part of the launched instantiation's name, e.g. for the rocprof agreement check).
int fused_sched(int act);

}  // namespace ppo
