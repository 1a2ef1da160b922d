/* duck_ppo.h — C ABI of the learner-side kernels of the PPO outer loop (libduck.so).
 *
 *   duck_gae   brax losses.compute_gae (the advantage/value-target recursion brax PPO runs in
 *                its loss; the reference reaches it through ppo.train at common/runner.py:104-118)
 *
 * Same conventions as duck.h: DEVICE pointers, float32, time-major [T][B] arrays (B = number of
 * trajectories, contiguous), `stream` a hipStream_t, negative return codes on error.
 */
#ifndef DUCK_PPO_H_
#define DUCK_PPO_H_

#ifdef __cplusplus
extern "C" {
#endif

/* vs[t][b], adv[t][b] from truncation/termination/reward/value [T][B] and bootstrap [B]:
 *   delta_t = (r_t + discount (1 - term_t) v_{t+1} - v_t)(1 - trunc_t),  v_T = bootstrap
 *   acc_t   = delta_t + discount (1 - term_t)(1 - trunc_t) lambda acc_{t+1},  vs_t = acc_t + v_t
 *   adv_t   = (r_t + discount (1 - term_t) vs_{t+1} - v_t)(1 - trunc_t),  vs_T = bootstrap */
int duck_gae(int T, int B, const float* truncation, const float* termination, const float* reward,
             const float* value, const float* bootstrap, float lambda_, float discount, float* vs, float* adv,
             void* stream);

#ifdef __cplusplus
}
#endif
#endif
