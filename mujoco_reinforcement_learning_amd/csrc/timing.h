// Per-launch device timing for bench.py's live roofline (replaces the reference's host-side
// @timeit, error_handling_utils.py:5-17).  While a ctx has timing enabled, every kernel an entry
// point launches goes through hipExtLaunchKernelGGL with an event pair attached to its dispatch
// packet, so a record is the kernel's own duration (no host launch gap), on the launch stream.
// Records carry the kernel's rocprofv3 name, its class, and its algorithmic FLOPs and bytes.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace ppo {

enum {
  KC_GEMM_FWD = 0,
  KC_GEMM_DGRAD,
  KC_GEMM_WGRAD,
  KC_UPDATE_HEAD,
  KC_POLICY_HEAD,
  KC_REDUCE,
  KC_GATHER,
  KC_GAE,
  KC_ADAM,
  KC_ROWS,   // row normalisation (reward / advantage / value target)
  KC_OBS,    // observation window push + normalisation
  KC_PERM,   // minibatch row selection
  KC_ENV,    // synthetic VecEnv step + Philox normals (bench harness)
  KC_FUSED,  // persistent fused minibatch forward + loss + backward (bf16)
  KC_LSTM,   // BiLSTM cell steps and elementwise glue (bilstm.hip)
  KC_CONV,   // implicit-GEMM convolutions of the pixel encoder (cnn_engine.hip)
  KC_COUNT
};

struct KernelTotals {  // one per kernel instantiation seen while timing
  const char *name;
  int cls;
  double ms, fl, by;
  int64_t n;
};

struct Timing {
  bool on = false;
  int capacity = 0;
  int used = 0;
  hipEvent_t *ev = nullptr;  // 2 per record
  int *cls = nullptr;
  const char **kname = nullptr;
  double *flops = nullptr, *bytes = nullptr;
  double ms[KC_COUNT] = {}, fl[KC_COUNT] = {}, by[KC_COUNT] = {};
  int64_t n[KC_COUNT] = {};
  std::vector<KernelTotals> per_kernel;
};

// The ctx timing an entry point records into for the duration of the call (set by TimingScope
// for ctx entry points, by FreeTimingScope for the ctx-free ones).
extern thread_local Timing *g_tim;
// The most recently enabled ctx timing: ctx-free entry points (ppo_gae, ppo_adam, ...) record
// into it while it is on.
extern Timing *g_free_tim;

// Interned "kernel<targs>" names spelled as rocprofv3 demangles them (minus "void ppo::" and
// the argument list); pointers stay valid for the life of the library.
const char *intern_name(const char *fmt, ...);

inline bool tim_active() { return g_tim != nullptr; }

// Shared bodies of the per-context timing entry points (ppo_ctx_timing / ppo_cnn_timing, ...):
// enable (re)allocates `capacity` event pairs and clears the totals; read folds pending records.
int timing_enable(Timing &t, int enable, int capacity);
int timing_read_class(Timing &t, int kclass, double *total_ms, int64_t *launches, double *flops,
                      double *bytes);
int timing_read_kernel(Timing &t, int index, const char **name, int *kclass, double *total_ms,
                       int64_t *launches, double *flops, double *bytes);

struct FreeTimingScope {
  FreeTimingScope() { g_tim = (g_free_tim && g_free_tim->on) ? g_free_tim : nullptr; }
  ~FreeTimingScope() { g_tim = nullptr; }
};

struct TimRec {
  int cls;
  const char *name;  // may be null when timing is off
  double flops, bytes;
};

// Launch `kernel`; when timing is active, with the next event pair on its dispatch packet.
template <typename F, typename... Args>
inline void launch_k(const TimRec &rec, F kernel, dim3 grid, dim3 block, uint32_t shm,
                     hipStream_t st, Args... args) {
  Timing *t = g_tim;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  // a launch being captured into a hipGraph (graph-replayed rollout) is not event-timed
  if (t && t->used < t->capacity && hipStreamIsCapturing(st, &cap) == hipSuccess &&
      cap == hipStreamCaptureStatusNone) {
    const int i = t->used++;
    t->cls[i] = rec.cls;
    t->kname[i] = rec.name;
    t->flops[i] = rec.flops;
    t->bytes[i] = rec.bytes;
    hipExtLaunchKernelGGL(kernel, grid, block, shm, st, t->ev[2 * i], t->ev[2 * i + 1], 0,
                          args...);
  } else {
    kernel<<<grid, block, shm, st>>>(args...);
  }
}

}  // namespace ppo
