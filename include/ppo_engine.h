/*
 * ppo_engine.h -- C-ABI of the MI355X (gfx950) PPO rollout-and-update engine.
 *
 * One shared object (mujoco_reinforcement_learning_amd/libppo_engine.so), plain pointers and
 * sizes, no torch types.  Every pointer argument named *_d is a caller-owned DEVICE buffer
 * (a PyTorch-ROCm tensor's data_ptr()), contiguous, in the dtype and layout documented at the
 * function.  `stream` is a hipStream_t passed as void* (torch.cuda.current_stream().cuda_stream);
 * nothing in the library synchronises the host except ppo_ctx_create/destroy.
 *
 * Return codes: 0 = ok, PPO_EINVAL on a bad argument (shape, null, size), PPO_EHIP on a HIP
 * runtime error; the message is in ppo_last_error() (thread-local).  The Python host raises
 * RuntimeError with that message (mirroring the reference's RuntimeError/ValueError style).
 *
 * The reference has no FFI: its "plugin interface" is a set of duck-typed Python classes.  Each
 * entry point below replaces the reference function cited next to it; the Python host
 * (mujoco_reinforcement_learning_amd/) keeps the reference's class/method surface on top.
 *
 * Buffer layout.  The rollout buffer is TIME-major in HBM: element (n, t) of
 * the reference's (N, T) TensorDict lives at storage row s = t*N + n, so one rollout step writes
 * one contiguous row block and the GAE scan reads coalesced rows.  The reference's flat minibatch
 * index f = n*T + t (memory.view(-1), ppo.py:99) is translated by ppo_perm_to_rows.
 *
 * Flat parameter layout: actor then critic, each in torch `Module.parameters()` order, i.e.
 *   actor : actor_logstd[A], then per layer l: W_l[out][in] (row-major, torch Linear), b_l[out]
 *   critic: per layer l: W_l[out][in], b_l[out]
 * each tensor starting at a 16-float aligned offset (ppo_param_offsets) so weight rows load as
 * 16-B vectors.  Gradients, Adam moments and split-K partial slabs use the same layout.
 */
#ifndef PPO_ENGINE_H
#define PPO_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PPO_ABI_VERSION 1
#define PPO_EINVAL (-22)
#define PPO_EHIP (-5)
#define PPO_MAX_LAYERS 8
#define PPO_PREC_F32 0  /* GEMMs on v_mfma_f32_32x32x2_f32: the reference's f32 (parity mode) */
#define PPO_PREC_BF16 1 /* GEMM operands rounded to bf16, f32 accumulate (BASELINE configs[1]) */

/* NetworkConfig.activation_class (features.py:41-54; main.py uses ReLU). */
enum { PPO_ACT_RELU = 0, PPO_ACT_TANH = 1, PPO_ACT_ELU = 2 };
/* No activation: the LSTM gate projections and the critic's output layer. */
#define PPO_ACT_IDENTITY 3

/* Shapes of the actor-critic (models/linear/actor.py:9-23, models/critic.py:6-20,
 * network_block_creator.py:24-72).  The critic flattens the (N, W, O) state like the actor. */
typedef struct ppo_net_cfg {
  int32_t obs_dim;          /* NetworkConfig.input_shape (O) */
  int32_t window;           /* EnvironmentConfig.window_length (W) */
  int32_t act_dim;          /* NetworkConfig.output_shape (A), <= 32 */
  int32_t activation;       /* PPO_ACT_* for every hidden layer */
  int32_t actor_use_bias;   /* NetworkConfig.use_bias (critic always has biases, critic.py:20) */
  int32_t n_actor_hidden;
  int32_t actor_hidden[PPO_MAX_LAYERS];
  int32_t n_critic_hidden;
  int32_t critic_hidden[PPO_MAX_LAYERS];
  float output_max_value;   /* NetworkConfig.output_max_value (actor.py:30) */
  int32_t max_rows;         /* workspace rows = max(num_envs, minibatch) */
} ppo_net_cfg;

typedef struct ppo_ctx ppo_ctx;

int ppo_abi_version(void);
const char *ppo_last_error(void);

/* Context: owns activation workspace and split-K grad slabs on `device`; caller owns params. */
int ppo_ctx_create(const ppo_net_cfg *cfg, int device, ppo_ctx **out);
int ppo_ctx_destroy(ppo_ctx *ctx);
/* net = 0 actor, 1 critic, -1 both: number of fp32 parameters in the flat layout. */
int64_t ppo_param_count(const ppo_ctx *ctx, int net);
/* Offsets (floats) of every parameter tensor in the flat layout, in torch parameters() order
 * (actor then critic); every tensor starts 16-float (64-B) aligned, padding in between is zero
 * in gradients.  Writes min(count, max_tensors) offsets; returns the tensor count. */
int ppo_param_offsets(const ppo_ctx *ctx, int64_t *offsets, int max_tensors);
/* Bind the flat fp32 parameter buffer (device, ppo_param_count(ctx,-1) floats). */
int ppo_bind_params(ppo_ctx *ctx, float *params_d);

/* ---- A1: observation window + per-sample standardisation -------------------------------------
 * replaces EnvironmentHelper.step's window shift (running_gym_sequential_vectorized.py:53-58,
 * helper.py:51-57) and get_state/normalize_state/_normalize (:61-92).
 * window_d: (N, O, W) f64, the reference's timestep.observation.  obs_d: (N, O) new observation
 * (f64 if obs_is_f64 else f32).  reset_d (nullable): u8 per env; 1 -> all W slots := obs
 * (termination / reset), 0 -> shift left and append.  With reset_d == NULL and all_reset != 0
 * every env is reset (helper.py:59-64). */
int ppo_obs_window_push(double *window_d, const void *obs_d, int obs_is_f64,
                        const uint8_t *reset_d, int all_reset, int n, int o, int w, void *stream);
/* state_d: (N, W, O) f32 = permute(standardise_f64(window)).  bounds: n_bounds+1 ascending
 * feature-slice edges already clipped to O (Humanoid table :70-80); normalize=0 -> plain cast. */
int ppo_obs_normalize(const double *window_d, float *state_d, int n, int o, int w,
                      const int32_t *bounds, int n_bounds, int normalize, void *stream);

/* ---- A2-A4: rollout policy step -------------------------------------------------------------
 * replaces PPOAgent.get_state_value / act / Normal.sample / log_prob (ppo.py:22-26,
 * ppo_agent.py:24-43, linear/actor.py:25-30).  state_d: (n, W*O) f32.
 * eps_d (nullable): (n, A) f32 standard normals drawn by the host in reference RNG order
 * (parity mode); NULL -> counter-based Philox4x32-10 normals keyed by (seed, offset) (perf mode).
 * Outputs (each nullable): action (n, A) = fl(fl(eps*std)+mean); logp (n,) = sum_a log_prob;
 * value (n,) critic V(s); mean (n, A).  Only the networks whose outputs are requested run. */
int ppo_policy_step(ppo_ctx *ctx, const float *state_d, int n, const float *eps_d, uint64_t seed,
                    uint64_t offset, float *action_d, float *logp_d, float *value_d, float *mean_d,
                    void *stream);
/* Fused observe + act (A1-A4 in one launch in precision bf16 with the fused shapes; otherwise the
 * A1 kernels followed by ppo_policy_step): replaces EnvironmentHelper.step's window push
 * (running_gym_sequential_vectorized.py:53-58), get_state (:61-92) and PPOAgent.act /
 * get_state_value (ppo.py:22-26, ppo_agent.py:24-43) for one rollout step.
 * window_d (N, O, W) f64 is pushed with obs_d (N, O) f64 when obs_d != NULL (reset_d / all_reset as
 * ppo_obs_window_push), standardised as ppo_obs_normalize into state_d (N, W*O) f32, then the
 * policy outputs are produced as ppo_policy_step (each nullable; the actor runs when action, logp
 * or mean is requested, the critic when value is). */
int ppo_observe_act(ppo_ctx *ctx, double *window_d, const double *obs_d, const uint8_t *reset_d,
                    int all_reset, const int32_t *bounds, int n_bounds, int normalize,
                    float *state_d, int n, const float *eps_d, uint64_t seed, uint64_t offset,
                    float *action_d, float *logp_d, float *value_d, float *mean_d, void *stream);
/* Refresh the bf16 weight images the fused kernels (or the wide bf16-resident layered path,
 * csrc/wide_path.h) read from the bound f32 parameters; call after the parameters change outside
 * ppo_minibatch_grad (Adam steps, loads) and before ppo_observe_act.  No-op unless a bf16 path
 * with weight images is active (ppo_policy_step refreshes the wide path's images itself). */
int ppo_pack_weights(ppo_ctx *ctx, void *stream);
/* Philox sampling in ppo_policy_step uses offset + *counter_d when counter_d (a device uint64)
 * is set, read when the kernel runs rather than when it is launched: a rollout captured once in
 * a hipGraph replays with fresh noise after the host bumps the counter.  NULL restores plain
 * `offset`.  (No reference counterpart: the reference draws from the host generator.) */
int ppo_ctx_set_rng_counter(ppo_ctx *ctx, const uint64_t *counter_d);

/* How the fused update reads the staged records (ppo_stage_records /
 * ppo_gae_stage_records) of a minibatch: 1 (default, PPO_FUSED_DIRECT) = each row's 128-B record
 * through the row indices, one chunk ahead, inside the fused launch (the step tail gathers
 * nothing); 0 = the gathered copy written by the prep kernel or the previous step tail.  Bitwise
 * the same results; enable < 0 queries. */
int ppo_ctx_fused_direct(ppo_ctx *ctx, int enable);
/* GEMM precision of every fc-layer GEMM the ctx launches (rollout forward, update forward,
 * dgrad, wgrad): PPO_PREC_F32 (default; parity with the f32 reference) or PPO_PREC_BF16 (bf16
 * operands on v_mfma_f32_32x32x16_bf16, f32 accumulation, f32 activations / params / Adam in
 * HBM -- the "bf16 GEMMs with fp32 accumulate and fp32 master params" of SURVEY.md s8(d)).
 * Heads, losses, GAE and Adam stay f32 either way. */
int ppo_ctx_set_precision(ppo_ctx *ctx, int prec);

/* ---- A6/A9: per-env standardisation over T (ppo.py:66-69 rewards, :81-88 advantage/target) ----
 * x_d: time-major (T, N) (element (n,t) at t*N+n), f32 or f64 (is_f64).  x <- (x-mean_T)/std_T*scale
 * with the unbiased std (torch.std), in place. */
int ppo_normalize_rows(void *x_d, int is_f64, int n, int t, double scale, void *stream);

/* ---- A7/A8: GAE + value target -------------------------------------------------------------
 * replaces torchrl 0.6.0 generalized_advantage_estimate called at ppo.py:70-80.
 * All arrays time-major (T, N).  value_d / next_value_d f32; reward_d f64 or f32 (reward_is_f64);
 * done_d / terminated_d u8 (done_d nullable -> done = terminated); force_last_done=1 applies
 * ppo.py:72 (done[:, -1] = True).  Recurrence carried in f64, stored f32 (bit-exact with the
 * reference).  adv_d, vtarget_d: f32 outputs. */
int ppo_gae(const float *value_d, const float *next_value_d, const void *reward_d,
            int reward_is_f64, const uint8_t *done_d, const uint8_t *terminated_d,
            int force_last_done, int n, int t, double gamma, double lmbda, float *adv_d,
            float *vtarget_d, void *stream);

/* ---- A10: minibatch rows ---------------------------------------------------------------------
 * rows_d[j] = storage row of reference flat index perm_d[start + j] (f = n*T+t -> t*N+n), j < b.
 * Replaces memory.view(-1)[torch.randperm(N*T)][i*B:(i+1)*B] (ppo.py:99-106).  With shard_lo <
 * shard_hi only envs in [shard_lo, shard_hi) are kept (exact data-parallel):
 * they are compacted in order and the count is written to count_d (device int32). */
int ppo_perm_to_rows(const int64_t *perm_d, int64_t start, int b, int n_envs, int t,
                     int shard_lo, int shard_hi, int32_t *rows_d, int32_t *count_d,
                     void *stream);
/* Perf-mode shuffle: rows of a keyed bijection (cycle-walking Feistel) of [0, n_envs*t). */
int ppo_feistel_rows(uint64_t seed, uint64_t epoch, int64_t start, int b, int n_envs, int t,
                     int32_t *rows_d, void *stream);

/* ---- A11-A13: one minibatch loss + gradients -------------------------------------------------
 * replaces ppo.py:109-135 (actor/critic forward, Normal log_prob/entropy, huber critic loss,
 * clipped surrogate, both backward passes).  Buffers are time-major storage arrays indexed by
 * rows_d (b rows, or *count_d if count_d != NULL): states (rows, W*O) f32, actions (rows, A),
 * old_logp (rows,), adv (rows,), vtarget (rows,).  inv_b = 1/B_global, inv_ba = 1/(B_global*A)
 * (data-parallel ranks pass the global minibatch so an all-reduce SUM gives the mean-loss grad).
 * grad_d: flat fp32 gradient (layout above), overwritten.  loss_d: 2 floats, (actor, critic)
 * loss contributions of these rows, overwritten. */
int ppo_minibatch_grad(ppo_ctx *ctx, const float *states_d, const float *actions_d,
                       const float *old_logp_d, const float *adv_d, const float *vtarget_d,
                       const int32_t *rows_d, int b, const int32_t *count_d, float clip_lo,
                       float clip_hi, float entropy_coef, float inv_b, float inv_ba,
                       float *grad_d, float *loss_d, void *stream);

/* Staged minibatch path of the fused bf16 engine (ppo_ctx_fused_active != 0).  Same contract and
 * same results as ppo_minibatch_grad over the same storage arrays, with the per-row gather
 * reading one 128 B record per row instead of five scattered arrays:
 *   ppo_stage_records packs rows [0, n_rows) of the time-major storage arrays (the arguments of
 *   ppo_minibatch_grad) into ctx-owned records once per iteration (after GAE, before the epochs;
 *   the first call for a given size allocates and must not be inside a graph capture);
 *   ppo_minibatch_grad_staged(rows_d, b, count_d, ...) is ppo_minibatch_grad on those records.
 *   flags PPO_STAGED_WEIGHTS_CURRENT: the bf16 weight images are already current (the previous
 *   optimizer step was ppo_adam_pack), so the weight refresh is skipped; PPO_STAGED_ROWS_GATHERED:
 *   the previous step (ppo_adam_pack_gather) gathered rows_d already (count_d must be NULL). */
#define PPO_STAGED_WEIGHTS_CURRENT 1
#define PPO_STAGED_ROWS_GATHERED 2
int ppo_ctx_fused_active(const ppo_ctx *ctx);
int ppo_stage_records(ppo_ctx *ctx, const float *states_d, const float *actions_d,
                      const float *old_logp_d, const float *adv_d, const float *vtarget_d,
                      int64_t n_rows, void *stream);
/* ppo_gae (same arguments and outputs, ppo.py:70-80) and ppo_stage_records over its n*t rows in
 * ONE pass: each row's record is written as soon as its advantage / value target leave the scan.
 * Valid when nothing rewrites adv / vtarget between the two (ppo.py:81-88 advantage
 * normalisation off); adv_d / vtarget_d / records are byte-identical to the two calls. */
int ppo_gae_stage_records(ppo_ctx *ctx, const float *value_d, const float *next_value_d,
                          const void *reward_d, int reward_is_f64, const uint8_t *done_d,
                          const uint8_t *terminated_d, int force_last_done, int n, int t,
                          double gamma, double lmbda, float *adv_d, float *vtarget_d,
                          const float *states_d, const float *actions_d, const float *old_logp_d,
                          void *stream);
int ppo_minibatch_grad_staged(ppo_ctx *ctx, const int32_t *rows_d, int b, const int32_t *count_d,
                              float clip_lo, float clip_hi, float entropy_coef, float inv_b,
                              float inv_ba, float *grad_d, float *loss_d, int flags,
                              void *stream);

/* ppo_adam_pack that also gathers the NEXT minibatch's rows next_rows_d[0, next_b) from the
 * staged records (the data-parallel form of ppo_update_step_staged's tail: grad_d is the
 * all-reduced gradient).  The next ppo_minibatch_grad_staged then passes
 * PPO_STAGED_ROWS_GATHERED | PPO_STAGED_WEIGHTS_CURRENT. */
int ppo_adam_pack_gather(ppo_ctx *ctx, const float *g_d, float *m_d, float *v_d,
                         const float *sched_d, float neg_step_actor, float neg_step_critic,
                         float bc2_sqrt, float one_minus_beta1, float beta2,
                         float one_minus_beta2, float eps, const int32_t *next_rows_d,
                         int next_b, void *stream);
/* The minibatch row gather alone (ppo.py:106 `batch = memory[indices]` on the staged records):
 * rows_d (b int32) -> the ctx's gathered-minibatch workspace, so a later
 * ppo_minibatch_grad_staged(..., PPO_STAGED_ROWS_GATHERED) reads them.  The data-parallel loop
 * issues it while the gradient all-reduce is in flight (it depends on the row indices only). */
int ppo_gather_staged_rows(ppo_ctx *ctx, const int32_t *rows_d, int b, void *stream);

/* One whole optimizer step of the staged single-rank path (ppo.py:109-135 for one minibatch,
 * then both optimizers' step()), in at most three launches: [row gather / weight refresh],
 * the fused forward/backward, and a tail that folds the slabs into grad_d, applies Adam (as
 * ppo_adam_pack; sched_d or the host scalars) with the weight-image refresh, and gathers the
 * NEXT minibatch's rows next_rows_d[0, next_b) (NULL / 0: none).  flags:
 * PPO_STAGED_WEIGHTS_CURRENT (the images are current) | PPO_STAGED_ROWS_GATHERED (the previous
 * step gathered rows_d already).  Results equal ppo_minibatch_grad_staged + ppo_adam_pack. */
int ppo_update_step_staged(ppo_ctx *ctx, const int32_t *rows_d, int b, const int32_t *next_rows_d,
                           int next_b, float clip_lo, float clip_hi, float entropy_coef,
                           float inv_b, float inv_ba, float *grad_d, float *loss_d, float *m_d,
                           float *v_d, const float *sched_d, float neg_step_actor,
                           float neg_step_critic, float bc2_sqrt, float one_minus_beta1,
                           float beta2, float one_minus_beta2, float eps, int flags,
                           void *stream);

/* ---- A15: fused Adam over the flat buffer (torch.optim.Adam single-tensor path) ----------------
 * replaces optimizers['critic'].step() / optimizers['actor'].step() (ppo.py:122,135) and
 * torch.optim.Adam defaults (ppo_agent.py:15-18).  Elements [0, n_actor) use neg_step_actor,
 * [n_actor, n) use neg_step_critic.  Every scalar is computed by the host in double exactly as
 * adam.py does and rounded to f32 the way torch wraps a python scalar: neg_step = -(lr/(1-b1^k)),
 * one_minus_beta1 = 1-b1, one_minus_beta2 = 1-b2, bc2_sqrt = (1-b2^k)**0.5.  One launch updates
 * p, m, v in place. */
int ppo_adam(float *p_d, const float *g_d, float *m_d, float *v_d, int64_t n, int64_t n_actor,
             float neg_step_actor, float neg_step_critic, float one_minus_beta1, float beta2,
             float one_minus_beta2, float bc2_sqrt, float eps, void *stream);

/* ppo_adam with the step-dependent scalars in device memory: sched_d = {neg_step_actor,
 * neg_step_critic, bc2_sqrt} (f32, computed by the host as for ppo_adam), read when the kernel
 * runs -- lets a hipGraph-captured optimizer loop replay with a per-iteration schedule. */
int ppo_adam_sched(float *p_d, const float *g_d, float *m_d, float *v_d, int64_t n,
                   int64_t n_actor, const float *sched_d, float one_minus_beta1, float beta2,
                   float one_minus_beta2, float eps, void *stream);

/* ppo_adam on the ctx's bound parameters (both nets, n_actor = ppo_param_count(ctx, 0)) that
 * also writes the updated W0/W1 into the fused kernels' bf16 weight images (ppo_pack_weights'
 * values), so the next ppo_minibatch_grad_staged may pass PPO_STAGED_WEIGHTS_CURRENT.  sched_d
 * (nullable) as ppo_adam_sched; NULL -> the three host scalars.  Fused bf16 path only. */
int ppo_adam_pack(ppo_ctx *ctx, const float *g_d, float *m_d, float *v_d, const float *sched_d,
                  float neg_step_actor, float neg_step_critic, float bc2_sqrt,
                  float one_minus_beta1, float beta2, float one_minus_beta2, float eps,
                  void *stream);

/* ---- host physics pool transfers (no reference counterpart: the
 * reference steps MuJoCo in-process, running_gym_sequential_vectorized.py:21-59) ------------------
 * Page-lock a host region (the pool's shared-memory obs / reward / terminated / action arrays) so
 * ppo_memcpy_async moves it by DMA without a staging copy; kind 1 = host->device, 2 =
 * device->host, asynchronous on `stream`. */
int ppo_host_register(void *host, int64_t bytes);
int ppo_host_unregister(void *host);
int ppo_memcpy_async(void *dst, const void *src, int64_t bytes, int kind, void *stream);
/* Device address of registered host memory (zero-copy access from kernels over PCIe). */
int ppo_host_device_ptr(void *host, void **dev);

/* ---- measurement: per-kernel-class timing (no reference counterpart; replaces @timeit,
 * error_handling_utils.py:5-17, with device-side timing) -----------------------------------------
 * enable=1 (re)starts recording a HIP event pair around every launch the ctx issues, on the
 * launch's stream (up to `capacity` launches); enable=0 stops.  ppo_ctx_timing_read synchronises
 * on the recorded events and returns per class: summed kernel ms, launches, algorithmic FLOPs and
 * algorithmic bytes.  kclass < 0 returns the number of classes. */
int ppo_ctx_timing(ppo_ctx *ctx, int enable, int capacity);
int ppo_ctx_timing_read(ppo_ctx *ctx, int kclass, double *total_ms, int64_t *launches,
                        double *flops, double *bytes);
const char *ppo_kernel_class_name(int kclass);
/* The same records per kernel instantiation.  `name` is spelled as rocprofv3 demangles the
 * kernel (e.g. "gemm_f32_kernel<2, 2, 2, 2, 32, 0, 1, 1, 4, 4, 2>", without "void ppo::" and
 * the argument list), so a timed kernel maps to one row of a rocprof --stats file; the string
 * lives as long as the library.  index < 0 returns the number of kernels seen. */
int ppo_ctx_timing_kernel(ppo_ctx *ctx, int index, const char **name, int *kclass,
                          double *total_ms, int64_t *launches, double *flops, double *bytes);

/* Diagnostics (no reference counterpart): enable=1 makes the ctx's fused bf16 minibatch kernel
 * run its stamped instantiation, which sums s_memtime deltas per phase segment (wave 0 of each
 * workgroup, 11 slots) into a device buffer; enable=0 synchronises, copies the last launch's
 * (2 nets, G workgroups, 11) uint64 cycle sums to host_out (up to max_values) and returns the
 * number of values, then restores the product kernel.  ReLU networks only. */
int ppo_ctx_phase_stamps(ppo_ctx *ctx, int enable, uint64_t *host_out, int max_values);

/* ---- harness: synthetic VecEnv dynamics on device + Philox normals ---------------------------
 * The bench/test environment (physics is out of scope): obs' = base_obs + 0.1*a[:, o % A],
 * r = base_r - 0.01*sum_a a^2 (f64), terminated = base_term.  obs_out (N, O) f64, reward (N,) f64,
 * terminated (N,) u8.  Mirrors oracle/ppo_ref.py RefSyntheticEnv. */
int ppo_synthetic_env_step(const float *base_obs_d, const float *base_reward_d,
                           const uint8_t *base_term_d, const float *action_d, int n, int o, int a,
                           double *obs_out_d, double *reward_out_d, uint8_t *term_out_d,
                           void *stream);
int ppo_philox_normal(uint64_t seed, uint64_t offset, float *out_d, int64_t n, void *stream);
/* The same normals at offset + *counter_d (device uint64, read when the kernel runs; NULL: 0):
 * element i = the Philox normal ppo_policy_step / ppo_observe_act draw at index offset +
 * *counter_d + i, so a whole rollout's noise (T x N x A) comes from one launch ahead of the steps,
 * bitwise the in-kernel draws, and a graph-captured rollout replays with fresh noise. */
int ppo_philox_normal_ctr(uint64_t seed, uint64_t offset, const uint64_t *counter_d, float *out_d,
                          int64_t n, void *stream);
/* One step of the single evaluation env of Algorithm.test (base_algorithm.py:21-48) on the same
 * synthetic streams (env 0, base arrays (T+1, N, O) / (T, N) / (T, N)), with the reference's
 * host branch (:33-37) taken on the device: *step_d = k (device int32, zeroed by the test reset);
 * terminated -> window (O, W) f64 := base_obs[0, 0] in every slot (reset_environment(test),
 * helper.py:59-64) and k := 0; else shift + append base_obs[(k+1)%(T+1), 0] + 0.1 a[o % A]
 * (helper.py:51-57, :36-37) and k := k+1.  *reward_sum_d += base_reward[k%T, 0] - 0.01 sum a^2
 * (f64, the sequential sum(rewards) of :38,48); *term_out_d = terminated.  action_d: (A,) f32,
 * the flattened test-phase mean (agent.py:35-38). */
int ppo_synthetic_test_step(const float *base_obs_d, const float *base_reward_d,
                            const uint8_t *base_term_d, int t_len, int n_envs,
                            const float *action_d, int o, int a, int w, double *window_d,
                            int32_t *step_d, double *reward_sum_d, uint8_t *term_out_d,
                            void *stream);

/* ---- Native pipelined host-physics rollout ----------------------
 * The shared-memory worker pool of host_pool.HostPhysicsPool, described for the C driver:
 * groups of workers over contiguous env ranges [group_lo, group_hi), each released by bumping
 * ctrl[g][2] (generation; ctrl[g][0] = step) and finished when done[worker_lo..worker_hi) all
 * equal that generation.  action / obs / reward / term are the page-locked shared-memory arrays
 * (N, A) f32, (N, O) f64, (N,) f64, (N,) u8.  gen[] is updated in place. */
#define PPO_MAX_GROUPS 4
typedef struct ppo_host_pool_desc {
  int32_t groups;
  int32_t group_lo[PPO_MAX_GROUPS], group_hi[PPO_MAX_GROUPS];
  int32_t worker_lo[PPO_MAX_GROUPS], worker_hi[PPO_MAX_GROUPS];
  int64_t gen[PPO_MAX_GROUPS];
  int64_t *ctrl;
  int64_t *done;
  float *action;      /* host addresses (the workers' view) ... */
  double *obs;
  double *reward;
  uint8_t *term;
  float *action_dev;  /* ... and their device addresses (ppo_host_device_ptr) */
  double *obs_dev;
  double *reward_dev;
  uint8_t *term_dev;
} ppo_host_pool_desc;

/* One whole T-step rollout over a host-physics pool (ppo.py:13-60 driving
 * running_gym_sequential_vectorized.py:40-59), pipelined per group from one native thread:
 * the group's rewards / terminations of the last step read from the shared memory into the
 * rollout buffer, ppo_observe_act on its rows reading the observations straight from the shared
 * memory, its actions written back into the shared memory (all zero-copy over PCIe, one compute
 * stream), then -- host side -- release of the group's workers and the wait for them.  Buffers are the rollout buffer's
 * time-major arrays: states (T+1, N, W*O), actions (T, N, A), logp (T, N), values (T+1, N),
 * reward (T, N) f64, term (T, N) u8; obs_next (N, O) f64 scratch.  eps_d (T, N, A) or NULL
 * (Philox(seed, base_offset + row*A)).  The window must hold the reset observations. */
int ppo_host_rollout(ppo_ctx *ctx, ppo_host_pool_desc *pool, double *window_d,
                     const int32_t *bounds, int n_bounds, int normalize, float *states_d,
                     float *actions_d, float *logp_d, float *values_d, double *reward_d,
                     uint8_t *term_d, double *obs_next_d, int n, int obs_dim, int window,
                     int act_dim, int horizon, const float *eps_d, uint64_t seed,
                     uint64_t base_offset, void *stream);

/* ---- Windowed BiLSTM actor-critic --------------------------------
 * models/lstm/lstm_actor.py:9-48 + lstm_critic.py:9-41, the PPOAgent binding of
 * entities/agents/ppo_agent.py:2-3, selected by NetworkConfig.feature_extractor == "LSTM"
 * (features.py:53).  Actor: nn.LSTM(O, latent, actor_layers, bidirectional, batch_first) over the
 * (B, W, O) window, act() on its outputs flattened to (B, W*2*latent), mean = tanh(MLP_mu(.)),
 * std = 0.2*exp(tanh(MLP_ls(.))) per row (B, A) -- the reference's repeat_interleave at
 * lstm_actor.py:48 returns (B, B, A), the shape bug this engine fixes.  Critic: a one-layer
 * BiLSTM, value = MLP_v(act(Y[:, W-1, :])).  Every MLP is a NetworkBlock with
 * hidden[0..n_hidden-1] and act() between layers (network_block_creator.py:24-86).
 * Flat parameters: torch parameters() order of LSTMActor then LSTMCritic (nn.LSTM: per layer and
 * direction w_ih[4L][in], w_hh[4L][L], b_ih[4L], b_hh[4L]; gates i, f, g, o), each tensor
 * 16-float aligned (ppo_lstm_param_layout). */
typedef struct ppo_lstm_cfg {
  int32_t obs_dim;          /* NetworkConfig.input_shape (O) */
  int32_t window;           /* EnvironmentConfig.window_length (W) */
  int32_t act_dim;          /* NetworkConfig.output_shape (A), <= 32 */
  int32_t activation;       /* PPO_ACT_* (NetworkConfig.activation_class) */
  int32_t use_bias;         /* NetworkConfig.use_bias (the MLPs; nn.LSTM always has biases) */
  int32_t latent;           /* NetworkConfig.feature_extractor_latent_size, multiple of 4 */
  int32_t actor_layers;     /* NetworkConfig.num_feature_extractor_layers (critic: 1) */
  int32_t n_hidden;         /* NetworkConfig.num_linear_layers */
  int32_t hidden[PPO_MAX_LAYERS];  /* NetworkConfig.linear_hidden_shapes */
  int32_t max_rows;         /* workspace rows = max(num_envs, minibatch) */
} ppo_lstm_cfg;
typedef struct ppo_lstm_ctx ppo_lstm_ctx;

/* Replaces PPOAgent.initialize_networks' model construction (ppo_agent.py:11-13). */
int ppo_lstm_ctx_create(const ppo_lstm_cfg *cfg, int device, ppo_lstm_ctx **out);
int ppo_lstm_ctx_destroy(ppo_lstm_ctx *ctx);
/* Offsets (floats) of every parameter tensor in torch order; *total, *n_actor (the actor's
 * share, for the two Adam groups).  Returns the tensor count. */
int ppo_lstm_param_layout(const ppo_lstm_ctx *ctx, int64_t *offsets, int max_tensors,
                          int64_t *total, int64_t *n_actor);
int ppo_lstm_bind_params(ppo_lstm_ctx *ctx, float *params_d);
int ppo_lstm_set_precision(ppo_lstm_ctx *ctx, int prec);
/* LSTMActor.forward + LSTMCritic.forward (lstm_actor.py:41-48, lstm_critic.py:33-41) on
 * state_d[n][W*O]: mean[n][A], std[n][A], value[n]; optional copies of the top LSTM layers'
 * outputs [n][W][2*latent] (nullable outputs are skipped). */
int ppo_lstm_forward(ppo_lstm_ctx *ctx, const float *state_d, int n, float *mean_d, float *std_d,
                     float *value_d, float *actor_lstm_out_d, float *critic_lstm_out_d,
                     void *stream);
/* PPO rollout step with the LSTM agent (ppo.py:22-26): action = eps*std + mean (eps from
 * eps_d, or Philox(seed, offset + i) when eps_d is null), log_prob summed over actions, V(s). */
int ppo_lstm_policy_step(ppo_lstm_ctx *ctx, const float *state_d, int n, const float *eps_d,
                         uint64_t seed, uint64_t offset, float *action_d, float *logp_d,
                         float *value_d, void *stream);
/* One minibatch of ppo.py:108-135 for the LSTM agent: the same arguments and gradient layout
 * contract as ppo_minibatch_grad (rows_d index the rollout rows), grad_d = the flat gradient. */
int ppo_lstm_minibatch_grad(ppo_lstm_ctx *ctx, const float *states_d, const float *actions_d,
                            const float *logp_d, const float *adv_d, const float *vt_d,
                            const int32_t *rows_d, int b, float *grad_d, float *loss_d,
                            float clip_lo, float clip_hi, float entropy_coef, float inv_b,
                            float inv_ba, void *stream);
/* bf16 forward steps s > 0 as one launch per step (the recurrent projection h W_hh^T on MFMA with
 * the cell in its epilogue: lstm_step_fwd_kernel; latent a multiple of 64) instead of the
 * projection GEMM + lstm_cell_fwd_kernel pair; bitwise the same results.  enable < 0 queries;
 * default PPO_LSTM_FUSED_STEP (1). */
int ppo_lstm_fused_step(ppo_lstm_ctx *ctx, int enable);
/* Per-launch event timing of this context (as ppo_ctx_timing / ppo_ctx_timing_kernel). */
int ppo_lstm_timing(ppo_lstm_ctx *ctx, int enable, int capacity);
int ppo_lstm_timing_kernel(ppo_lstm_ctx *ctx, int index, const char **name, int *kclass,
                           double *total_ms, int64_t *launches, double *flops, double *bytes);

/* ---- Pixel-observation actor-critic (BASELINE.json configs[4]) ----------------------------
 * dm_control cheetah-run pixel observations: u8 frames (H, W, C) = (84, 84, 3), HWC.  The
 * reference has NO pixel / CNN path (running_dm_control.py:56-91 is state-observation humanoid),
 * so this model is the engine's own declaration: each net is the Nature-DQN
 * encoder -- Conv2d(3, 32, 8, 4) ReLU, Conv2d(32, 64, 4, 2) ReLU, Conv2d(64, 64, 3, 1) ReLU,
 * flatten (torch CHW order, 3136 features) -- followed by the reference's NetworkBlock heads:
 * actor mean = output_max_value * tanh(MLP(features)) with the state-independent actor_logstd of
 * models/linear/actor.py:9-30, critic value = MLP(features) (models/critic.py:6-25); actor and
 * critic keep separate encoders (they have separate optimizers, ppo_agent.py:15-22).  Pixels are
 * scaled by 1/255 (x / 255.f).  Flat parameters, torch parameters() order with 16-float aligned
 * tensors:  actor: actor_logstd[A], encoder.{0,2,4}.weight [co][ci][k][k] + .bias,
 * actor.first_layers.* / last_layer.*;  critic: encoder.*, network.*  (ppo_cnn_param_layout).
 * The convolutions are implicit GEMMs on MFMA (csrc/conv.h): exact f32 operands in PPO_PREC_F32,
 * bf16 operands with f32 accumulation in PPO_PREC_BF16. */
typedef struct ppo_cnn_cfg {
  int32_t height, width, channels;  /* pixel frame: 84, 84, 3 (the compiled encoder geometry) */
  int32_t act_dim;                  /* NetworkConfig.output_shape (A), <= 32 */
  int32_t activation;               /* PPO_ACT_* of the MLP hidden layers (the encoder: ReLU) */
  int32_t use_bias;                 /* NetworkConfig.use_bias of the actor MLP */
  int32_t n_hidden;                 /* NetworkConfig.num_linear_layers (actor and critic) */
  int32_t hidden[PPO_MAX_LAYERS];   /* NetworkConfig.linear_hidden_shapes */
  float output_max_value;           /* NetworkConfig.output_max_value (actor.py:30) */
  int32_t max_rows;                 /* workspace rows = max(num_envs, minibatch) */
} ppo_cnn_cfg;
typedef struct ppo_cnn_ctx ppo_cnn_ctx;

/* Replaces PPOAgent.initialize_networks' model construction (ppo_agent.py:11-13). */
int ppo_cnn_ctx_create(const ppo_cnn_cfg *cfg, int device, ppo_cnn_ctx **out);
int ppo_cnn_ctx_destroy(ppo_cnn_ctx *ctx);
int ppo_cnn_param_layout(const ppo_cnn_ctx *ctx, int64_t *offsets, int max_tensors,
                         int64_t *total, int64_t *n_actor);
int ppo_cnn_bind_params(ppo_cnn_ctx *ctx, float *params_d);
int ppo_cnn_set_precision(ppo_cnn_ctx *ctx, int prec);
int ppo_cnn_set_rng_counter(ppo_cnn_ctx *ctx, const uint64_t *counter_d);
/* Actor.forward + Critic.forward on frames_d[n][H*W*C] u8: mean[n][A], value[n]; optionally the
 * encoder outputs (the flattened features [n][3136], f32) of both nets.  Nullable outputs are
 * skipped. */
int ppo_cnn_forward(ppo_cnn_ctx *ctx, const uint8_t *frames_d, int n, float *mean_d,
                    float *value_d, float *feat_actor_d, float *feat_critic_d, void *stream);
/* The PPO rollout step (ppo.py:22-26) on pixel frames: action = eps*std + mean (eps from eps_d,
 * or Philox(seed, offset + counter + i) when eps_d is null), log_prob summed over actions, V(s). */
int ppo_cnn_policy_step(ppo_cnn_ctx *ctx, const uint8_t *frames_d, int n, const float *eps_d,
                        uint64_t seed, uint64_t offset, float *action_d, float *logp_d,
                        float *value_d, float *mean_d, void *stream);
/* One minibatch of ppo.py:108-135 with the pixel actor-critic: frames_d = the rollout buffer's
 * frames [(T+1)*N][H*W*C] u8, rows_d the minibatch's storage rows (t*N + n), the other arrays as
 * ppo_minibatch_grad; grad_d = the flat gradient, loss_d[2] = (actor, critic) loss. */
int ppo_cnn_minibatch_grad(ppo_cnn_ctx *ctx, const uint8_t *frames_d, const float *actions_d,
                           const float *logp_d, const float *adv_d, const float *vt_d,
                           const int32_t *rows_d, int b, float *grad_d, float *loss_d,
                           float clip_lo, float clip_hi, float entropy_coef, float inv_b,
                           float inv_ba, void *stream);
/* Per-launch event timing of this context (as ppo_ctx_timing / ppo_ctx_timing_kernel). */
int ppo_cnn_timing(ppo_cnn_ctx *ctx, int enable, int capacity);
int ppo_cnn_timing_kernel(ppo_cnn_ctx *ctx, int index, const char **name, int *kclass,
                          double *total_ms, int64_t *launches, double *flops, double *bytes);
/* Synthetic pixel VecEnv step (bench / test harness; physics is out of scope): frame t of env n,
 *   pix[y][x][c] = (mix32(seed, t, n, (y*W + x)*C + c) + q[(2c + ((x + y) & 1)) % A]) & 255,
 *   q[j] = clamp(floor(8 * action[n][j]), -64, 63)   (q = 0 when action_d is NULL: the reset frame)
 * written to frames_out_d[n][H*W*C]; with base_reward_d / base_term_d (T, N) and t >= 1 also
 * reward_out[n] = base_reward[t-1][n] - 0.01 * sum_a a^2 (f64, a summed in order) and
 * term_out[n] = base_term[t-1][n] (the state-env formulas of ppo_synthetic_env_step). */
int ppo_synthetic_pixel_step(uint32_t seed, int t, const float *action_d, int n, int h, int w,
                             int c, int a, uint8_t *frames_out_d, const float *base_reward_d,
                             const uint8_t *base_term_d, double *reward_out_d,
                             uint8_t *term_out_d, void *stream);

/* ---- (e) data-parallel gradient exchange (csrc/comm.hip) ----------------
 * The reference has no distributed code; the engine shards envs over the GPUs of one node (one
 * process per GPU) and sums the flat actor+critic gradient of every optimizer step (ppo.py:120-135)
 * with ONE in-place RCCL all-reduce, issued on the caller's compute stream -- so a hipGraph
 * capture of the optimizer loop records it like a kernel.  RCCL is resolved at run time (the
 * instance torch.distributed loaded, else librccl.so.1, or $PPO_RCCL_LIB); without it only these
 * calls fail (PPO_EHIP, message in ppo_last_error).
 *   ppo_comm_unique_id   rank 0 draws the 128-byte id; the host broadcasts it (torch.distributed)
 *   ppo_comm_create      every rank, with the same id, its rank and its device (collective call)
 *   ppo_comm_allreduce   buf_d[0, n) f32 := SUM over ranks, in place, ordered on `stream`
 *   ppo_comm_check       the communicator's asynchronous error state (0 = healthy)
 *   ppo_comm_query       what RCCL itself reports: rank count (ncclCommCount), this rank
 *                        (ncclCommUserRank) and the device the communicator was built on
 *   ppo_ctx_set_comm / ppo_allreduce_grads   SURVEY.md s8(b)'s ctx-owned form: the ctx keeps the
 *                        communicator (not owned: ppo_comm_destroy after the ctx) and
 *                        ppo_allreduce_grads(ctx, flat, n, stream) sums n <= ppo_param_count(ctx, -1)
 *                        floats of the flat gradient layout. */
#define PPO_COMM_ID_BYTES 128
typedef struct ppo_comm ppo_comm;
int ppo_comm_version(void); /* NCCL_VERSION_CODE of the RCCL in use, 0 if none */
int ppo_comm_unique_id(uint8_t *id_out);
int ppo_comm_create(const uint8_t *id, int nranks, int rank, int device, ppo_comm **out);
int ppo_comm_destroy(ppo_comm *comm);
int ppo_comm_allreduce(ppo_comm *comm, float *buf_d, int64_t n, void *stream);
int ppo_comm_check(ppo_comm *comm);
int ppo_comm_query(ppo_comm *comm, int *nranks_out, int *rank_out, int *device_out);
int ppo_ctx_set_comm(ppo_ctx *ctx, ppo_comm *comm);
int ppo_allreduce_grads(ppo_ctx *ctx, float *flat_d, int64_t n, void *stream);

/* Logged-loss share of the entropy bonus (ppo.py:128-132 `- entropy * entropy_eps`): the loss_d
 * actor value a minibatch entry point writes is -(sum of the rows' clipped surrogate) * inv_b -
 * share * entropy_eps * H.  Data-parallel ranks each see the same H (replicated log-std), so with
 * the per-rank losses SUMMED for logging, rank 0 passes 1 and the others 0 and the sum carries the
 * bonus once.  Default 1.  Gradients are unaffected (the per-row log-std term uses inv_ba). */
int ppo_ctx_loss_entropy_share(ppo_ctx *ctx, float share);
int ppo_lstm_loss_entropy_share(ppo_lstm_ctx *ctx, float share);
int ppo_cnn_loss_entropy_share(ppo_cnn_ctx *ctx, float share);

/* ---- wide layered path (bf16-resident activations; csrc/wide_gemm.h) ----------------------------
 * One bf16 MFMA GEMM of the wide path on caller buffers (kernel-level parity tests and tuning).
 * The products of network_block_creator.py:74-86 (Linear layers) and their autograd backward
 * (ppo.py:109-135 loss.backward()), on bf16 operands with f32 accumulation:
 *   kind 0 FWD    C[m][n] bf16 = act(sum_k A[m][k] B[n][k] + bias[n])   (rows >= *count_d: 0)
 *   kind 1 DGRAD  C[m][n] bf16 = act'(aux[m][n]) * sum_k A[m][k] B[n][k] (aux: the layer output,
 *                 bf16, C may alias it); colsum_d (nullable) [ceil(m / tile)][n] f32 column sums
 *                 of C before rounding, one row per row tile
 *   kind 2 F32    C[m][n] f32 = sum_k A[m][k] B[n][k]
 *   kind 3 WGRAD  C[split][m][n] f32 = sum over the split's rows k of A[k][m] B[k][n] (split-K
 *                 over *count_d (or k) rows, `splits` slabs of m*ldc floats)
 * A, B bf16; NT kinds need k % 64 == 0 and operand rows readable up to the padded extents
 * (round_up(m or n, tile) rows of k elements); act = PPO_ACT_*. */
int ppo_wide_gemm(int kind, int m, int n, int k, const void *a_d, int64_t lda, const void *b_d,
                  int64_t ldb, void *c_d, int64_t ldc, const float *bias_d, const void *aux_d,
                  float *colsum_d, int act, int splits, const int32_t *count_d, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PPO_ENGINE_H */
