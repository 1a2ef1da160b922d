/* duck_oracle.h — CPU restatement (fp64) of the Open Duck Joystick hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This library is the parity checker and the CPU baseline;
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product path (open_duck_playground_amd, libduck.so) never links or calls it.
 *
 * What it restates (no reference physics can run in this container):
 *   - mjx.step / mj_step for this model class (reference call sites:
 *     playground/open_duck_mini_v2/joystick.py:258 (init -> forward) and :420
 *     (mjx_env.step -> 10 x mjx.step)): kinematics, com-based inertia, CRB mass
 *     matrix, MJX-style collision (plane-convex 4-point manifold, convex-convex SAT),
 *     pyramidal contact / joint limit / dof friction rows, MJX Newton solver (1 iteration,
 *     zoom line search), site sensors, semi-implicit Euler.
 *   - Joystick.reset / step / _get_obs / _get_reward / _get_termination
 *     (joystick.py:206-725), common/rewards.py, custom_rewards.py,
 *     poly_reference_motion.py and randomize.py.
 * Parity status: physics "unpinned" by any reference test (the reference has none and
 * mujoco/mjx are not installed); rewards/reference-motion pinned by golden vectors from
 * the reference's own NumPy twins (tests/golden/).
 */
#ifndef DUCK_ORACLE_H_
#define DUCK_ORACLE_H_

#include <stdint.h>

#include "../include/duck_env.h"
#include "../include/duck_model.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_model oracle_model;

/* physics data of one env (subset of mjData) */
typedef struct oracle_data {
  double qpos[DUCK_MAXQ], qvel[DUCK_MAXV], qacc_warmstart[DUCK_MAXV], ctrl[DUCK_MAXU];
  double qacc[DUCK_MAXV], qacc_smooth[DUCK_MAXV], qfrc_smooth[DUCK_MAXV], qfrc_bias[DUCK_MAXV],
      qfrc_passive[DUCK_MAXV], qfrc_actuator[DUCK_MAXV], qfrc_constraint[DUCK_MAXV];
  double actuator_force[DUCK_MAXU];
  double sensordata[DUCK_MAXSENSORDATA];
  double xpos[DUCK_MAXBODY][3], xquat[DUCK_MAXBODY][4], xmat[DUCK_MAXBODY][9];
  double xipos[DUCK_MAXBODY][3], ximat[DUCK_MAXBODY][9];
  double site_xpos[DUCK_MAXSITE][3], site_xmat[DUCK_MAXSITE][9];
  double geom_xpos[DUCK_MAXGEOM][3], geom_xmat[DUCK_MAXGEOM][9];
  double qM[DUCK_MAXV][DUCK_MAXV];
  /* contacts: fixed slots, DUCK_CON_PER_PAIR per pair, dist > 0 = inactive */
  int ncon;
  double con_dist[DUCK_MAXCON], con_pos[DUCK_MAXCON][3], con_frame[DUCK_MAXCON][9];
  int con_geom1[DUCK_MAXCON], con_geom2[DUCK_MAXCON];
  int nefc;
  double efc_force[128];
  int solver_niter;
} oracle_data;

oracle_model* oracle_model_create(const duck_model_desc* desc);
void oracle_model_destroy(oracle_model* m);
/* apply one env's domain-randomisation parameters (duck_dr_layout) to a model copy */
oracle_model* oracle_model_randomized(const oracle_model* m, const double* dr);
void oracle_dr_sample(const oracle_model* m, uint64_t seed, int64_t env_id, double* dr_out);

void oracle_forward(const oracle_model* m, oracle_data* d);
void oracle_step(const oracle_model* m, oracle_data* d, int nsubstep);

/* threefry2x32-20 (Salmon et al. 2011), exposed for known-answer tests */
void oracle_threefry2x32(const uint32_t key[2], const uint32_t ctr[2], uint32_t out[2]);

/* Joystick env on one env: fstate/istate are this env's columns (stride 1). */
int oracle_env_reset(const oracle_model* m, const duck_env_config* cfg, const duck_refmotion* ref,
                     uint64_t seed, int64_t env_id, double* fstate, int32_t* istate, double* obs, double* priv);
/* brute-force check of the height-field prism decomposition: every penetrating prism's exact
 * separating-axis depth, normal, deepest hull vertex and strip index */
int oracle_hfield_prisms(const oracle_model* m, const oracle_data* d, int g_hf, int g_cvx, int max, double* depth,
                         double* normal, double* point, int* index);
/* test aid: counts of the axis class that gave each prism contact (top, sides, bottom, hull faces,
 * top-edge pairs, vertical-edge pairs, bottom-edge pairs) since the last reset, then [7 + class]
 * the class that separated a prism whose own 5 faces do not */
void oracle_hfield_axis_wins(long long out[14], int reset);
void oracle_set_trace(double* buf); /* test aid: record substep inputs of oracle_env_step */
void oracle_set_ls_floor(double floor); /* test aid: the HIP line search's fp32 stop rule (0 = off) */
void oracle_set_hdump(double* buf); /* test aid: dump the next solve's first Newton Hessian and row margins */
void oracle_set_hf_band_scale(double s); /* test aid: scales HF_POINT_BAND (0: the plain weighted centroid) */
double oracle_get_hf_band_scale(void);
/* test aids: injected contact-generation defects (0 point band scale, 1 witness band scale, 2 depth
 * tie scale, 3 manifold start rank) */
void oracle_set_hf_defect(int which, double value);
double oracle_get_hf_defect(int which);
/* test aid: the height-field 4-slot choice (collide_hfield_convex's) over caller-given candidates */
int oracle_hfield_select(const double* depth, const double* point, const double* normal, int n, int idx[4]);
void oracle_set_hf_tie_last(double band); /* test aid: height-field SAT near-ties resolve to the last axis in the band */
void oracle_set_hf_tie_first(double band); /* test aid: height-field SAT near-ties resolve to the first axis in the band */
int oracle_hfield_contacts(const oracle_model* m, const oracle_data* d, int g_hf, int g_cvx, int max, double* depth,
                           double* normal, double* point); /* test aid: the prism contacts before the manifold selection */
void oracle_set_con_override(const double* buf); /* test aid: replace the contact set after collision (7 doubles per slot) */
void oracle_set_force_start(int mode);  /* test aid: Newton start 1 warm, 2 smooth, 0 the cheaper */
void oracle_last_start_costs(double out[2]); /* test aid: costs at qacc_warmstart, qacc_smooth */
int oracle_env_step(const oracle_model* m, const duck_env_config* cfg, const duck_refmotion* ref,
                    double* fstate, int32_t* istate, const double* action, double* obs, double* priv,
                    double* reward, double* done, oracle_data* d_out);

/* reward/reference-motion pieces, exposed for golden-vector tests */
void oracle_reference_motion(const duck_refmotion* ref, double dx, double dy, double dtheta, int i, double out[40]);
double oracle_reward_imitation(const double base_qpos[7], const double base_qvel[6], const double* joints_qpos,
                               const double* joints_qvel, const double contacts[2], const double* ref,
                               const double cmd[7], int nu);
void oracle_rewards(const double cmd[7], const double local_linvel[3], const double gyro[3],
                    const double* actuator_force, const double* action, const double* last_act,
                    const double* joints_qpos, const double* joints_qvel, const double* default_act, int nu,
                    double tracking_sigma, double out[5]);
void oracle_standing_rewards(const double cmd[7], const double upvector[3], const double* actuator_force,
                             const double* action, const double* last_act, const double* joints_qpos,
                             const double* joints_qvel, const double* default_act, int nu, double out[6]);

/* batched CPU baseline: n_envs independent envs, OpenMP over envs.
 * fstate/istate are SoA with stride n_envs (duck_env.h); models[e] per env (or one shared). */
int oracle_batch_step(const oracle_model* const* models, int n_models, const duck_env_config* cfg,
                      const duck_refmotion* ref, int n_envs, double* fstate, int32_t* istate,
                      const double* actions, double* obs, double* priv, double* reward, double* done,
                      int n_threads);
int oracle_batch_reset(const oracle_model* const* models, int n_models, const duck_env_config* cfg,
                       const duck_refmotion* ref, int n_envs, uint64_t seed, int64_t env_offset,
                       double* fstate, int32_t* istate, double* obs, double* priv, int n_threads);

/* test aid: iteration counts of this thread's line searches since the last reset (tools/ls_divergence.py) */
int oracle_ls_trace(int* out, int cap, int reset);

#ifdef __cplusplus
}
#endif
#endif
