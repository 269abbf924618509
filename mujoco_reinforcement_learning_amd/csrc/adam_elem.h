// One element of the engine's Adam step (torch.optim.Adam, amsgrad=False, weight_decay=0:
// reference ppo.py:122/:135 via agent.optimizers[...].step()), shared by adam_kernel,
// adam_sched_kernel and adam_pack_kernel so every optimizer path rounds identically.
#pragma once

#include <hip/hip_runtime.h>

namespace ppo {

// w1 = 1 - beta1 (torch's lerp weight), b2 = beta2, omb2 = 1 - beta2; ns = -lr / (1 - beta1^t)
// of this element's net, bc2_sqrt = sqrt(1 - beta2^t).  Returns the new parameter.
__device__ __forceinline__ float adam_elem(float p, float gi, float &m, float &v, float ns,
                                           float w1, float b2, float omb2, float bc2_sqrt,
                                           float eps) {
  float mi = m;
  // torch.lerp: weight < 0.5 -> start + w*(end-start), else end - (1-w)*(end-start)
  mi = (w1 < 0.5f) ? fmaf(w1, gi - mi, mi) : fmaf(w1 - 1.f, gi - mi, gi);
  // torch's vectorised addcmul (self + value*t1*t2) is built with FP contraction: one FMA
  const float vi = fmaf(omb2 * gi, gi, v * b2);
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  m = mi;
  v = vi;
  return p + (ns * mi) / denom;
}

}  // namespace ppo
