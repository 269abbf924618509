/* Host-side synthetic dynamics of the host physics pool's workers (host_pool.py), compiled with
 * gcc into libppo_hostenv.so.  It stands in for gymnasium's MuJoCo env.step on the worker's env
 * slice -- the one call a real MuJoCo pool makes here (mujoco / gymnasium are not installed in
 * this image) -- and is bit-identical to synthetic_env_step_kernel and to host_pool.step_slice's
 * numpy form (built with -ffp-contract=off: every a*b+c below rounds twice, like numpy):
 *   obs'      = base_obs[t+1] + 0.1 * a[:, o % A]      (f64)
 *   reward    = base_reward[t] - 0.01 * sum_a a^2      (f64, summed in order)
 *   terminated = base_terminated[t]                                                      */
#include <stdint.h>

void ppo_host_step_slice(const float *base_obs, const float *base_reward,
                         const uint8_t *base_term, const float *action, double *obs,
                         double *reward, uint8_t *term, int64_t n, int o, int a, int t,
                         int64_t lo, int64_t hi) {
  const float *bo = base_obs + ((int64_t)(t + 1) * n) * o;
  const float *br = base_reward + (int64_t)t * n;
  const uint8_t *bt = base_term + (int64_t)t * n;
  for (int64_t e = lo; e < hi; ++e) {
    const float *ae = action + e * a;
    for (int k = 0; k < o; ++k)
      obs[e * o + k] = (double)bo[e * o + k] + 0.1 * (double)ae[k % a];
    double ctrl = 0.0;
    for (int j = 0; j < a; ++j) ctrl = ctrl + (double)ae[j] * (double)ae[j];
    reward[e] = (double)br[e] - 0.01 * ctrl;
    term[e] = bt[e];
  }
}
