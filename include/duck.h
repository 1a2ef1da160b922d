/* duck.h — C ABI of the MI355X Open Duck Joystick simulator (libduck.so).
 *
 * This is the drop-in boundary for the reference's hot path. Each entry point replaces
 * one reference interface (file:line under /root/reference):
 *
 *   duck_create        OpenDuckMiniV2Env.__init__ + Joystick._post_init
 *                        (playground/open_duck_mini_v2/base.py:44-132, joystick.py:121-204);
 *                        the model arrives pre-compiled (duck_model.h), like mjx.put_model (base.py:61)
 *   duck_reset         Joystick.reset(rng) -> State          (joystick.py:206-321)
 *   duck_step          Joystick.step(state, action) -> State (joystick.py:323-481), optionally
 *                        wrapped by EpisodeWrapper + BraxAutoResetWrapper (common/runner.py:117)
 *   duck_randomize     randomize.domain_randomize(model, rng) (common/randomize.py:26-146)
 *   duck_physics_step  mjx_env.step(model, data, ctrl, n_substeps) (joystick.py:420);
 *                        n_substeps = 0 is mjx_env.init's mjx.forward (joystick.py:258)
 *
 * Conventions: all array arguments are DEVICE pointers (HIP/torch allocations on the
 * handle's device), float32 unless stated, `stream` is a hipStream_t (NULL = default).
 * Per-env state is struct-of-arrays with the layout of duck_env.h (fstate/istate);
 * obs/priv/action are row-major [n_envs][k]. The caller owns every buffer; the handle owns
 * only device-resident model constants. No call allocates, synchronises or throws; errors
 * are returned as negative codes with a thread-local message in duck_last_error().
 * Calls on one handle are not thread-safe; work is ordered on `stream`.
 */
#ifndef DUCK_H_
#define DUCK_H_

#include <stddef.h>
#include <stdint.h>

#include "duck_env.h"
#include "duck_model.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct duck_sim duck_sim;

enum { DUCK_OK = 0, DUCK_EINVAL = -1, DUCK_EUNSUPPORTED = -2, DUCK_EHIP = -3, DUCK_EDEVICE = -4 };

/* library version (major*10000 + minor*100 + patch) */
int duck_version(void);
/* sha1 of the sources, headers and compile flags this library was built from */
const char* duck_build_id(void);
/* message of the last failing call on this thread ("" if none) */
const char* duck_last_error(void);
/* per-env state layout for a model/config/task (same as duck_layout_make) */
int duck_layout_get(int nq, int nv, int nu, int imitation, int task, duck_layout* out);
/* size in floats of the per-env debug record written by duck_physics_step(aux) */
int duck_aux_size(const duck_sim* sim);
/* debug: per-stage cycle counters of a -DDUCK_STAGE_PROF build (32 + 1024 x uint64: 32 stage counters, then per-wave cycles of the last launch; optionally
 * reset); DUCK_EUNSUPPORTED in a regular build */
int duck_debug_stage_cycles(const duck_sim* sim, unsigned long long* out, int reset);

/* Identity of a kernel specialisation: FNV-1a 64 over the float32-rounded model values the
 * kernels bake at compile time (everything in duck_model_desc except the height-field
 * elevation, which duck_create uploads). Host-only. */
uint64_t duck_model_fingerprint(const duck_model_desc* model);
/* 1 if this library holds kernels compiled for `model` (same fingerprint), else 0 */
int duck_model_supported(const duck_model_desc* model);

/* Create a simulator for `model`. The kernels are specialised on the model at build time
 * (like MJX specialises its XLA program at jit time); a model none of this library's
 * variants was compiled for is rejected with DUCK_EUNSUPPORTED. `ref` may be NULL
 * when cfg->use_imitation == 0. `device` is the HIP device ordinal. */
int duck_create(const duck_model_desc* model, const duck_env_config* cfg, const duck_refmotion* ref, int device,
                duck_sim** out);
void duck_destroy(duck_sim* sim);

/* Joystick.reset for envs [env_offset, env_offset + n_envs): key derived from
 * (seed, global env id). `mask` (uint8 [n_envs], nullable) restricts the reset to envs
 * with mask != 0. Writes fstate/istate/obs/priv. */
int duck_reset(duck_sim* sim, int n_envs, float* fstate, int32_t* istate, const uint8_t* mask, uint64_t seed,
               int64_t env_offset, const float* dr, float* obs, float* priv, void* stream);

/* Step kernel selection for duck_step (the same stage code, a different work split):
 * THROUGHPUT runs 16 envs per workgroup, each env's substeps on one 16-lane team (the batch
 * rate at >= 4 envs per SIMD); LATENCY runs 4 envs per workgroup with each substep's stages
 * split over its 4 waves (the shortest env-step: strong scaling over GPUs, <= 4 envs per CU);
 * PAIRED runs 8 envs per workgroup, each set of 4 on a pair of waves that split the stages
 * (the shortest env-step at 4-8 envs per CU: 4,096 envs over 2 GPUs). AUTO (the default) picks
 * LATENCY while n_envs <= 4 x the device's CU count, LATENCY_X2 (where compiled, below) or else PAIRED
 * while n_envs <= 8 x, else THROUGHPUT.
 * Every mode gives the same results bit for bit (every scene; tests/test_gpu_env.py), so a run's
 * trajectories do not depend on the batch size or the GPU count that picked the kernel; bench.py
 * and the PPO runner still record which kernel ran. A model whose LDS budget does not fit a
 * latency split (model blob + hot state in LDS next to the env slices) is compiled without it:
 * duck_set_step_mode refuses that mode with DUCK_EUNSUPPORTED and AUTO skips it.
 * LATENCY_X2 (round 6) is the LATENCY kernel compiled for two waves per SIMD (<= 256 registers per
 * lane), so that two of its 4-env workgroups share a CU: the shortest env-step at 4-8 envs per CU in
 * the plane-floor scenes without backlash, the only models it is compiled for (elsewhere its register
 * spills make it slower than PAIRED); AUTO takes it there instead of PAIRED. */
enum { DUCK_STEP_AUTO = 0, DUCK_STEP_THROUGHPUT = 1, DUCK_STEP_LATENCY = 2, DUCK_STEP_PAIRED = 3,
       DUCK_STEP_LATENCY_X2 = 4 };
int duck_set_step_mode(duck_sim* sim, int mode);
/* the kernel duck_step would launch for n_envs envs: DUCK_STEP_THROUGHPUT, _LATENCY, _PAIRED or _LATENCY_X2 */
int duck_step_kernel_for(const duck_sim* sim, int n_envs);
/* debug: latency-mode event waits that gave up (a broken cross-wave schedule; must stay 0) */
int duck_debug_lat_timeouts(const duck_sim* sim, unsigned* out, int reset);

/* Sticky device error word of the handle (bits DUCK_DEVERR_*), set by a kernel that could not
 * complete its step correctly. It lives in host-mapped memory: duck_reset / duck_step /
 * duck_physics_step read it on entry WITHOUT synchronising and return DUCK_EDEVICE while it is
 * non-zero (so a failure surfaces at the first call after the failing launch has been written,
 * at the latest after the caller's next synchronisation). `clear` resets it. No reference
 * counterpart: MJX has no failure mode of this kind (its NaN guard is joystick.py:483-485). */
enum { DUCK_DEVERR_LAT_TIMEOUT = 1 };
int duck_device_error(duck_sim* sim, unsigned* out, int clear);

/* Joystick.step (+ wrappers if cfg->auto_reset). `dr` (nullable) = per-env randomised
 * model values (duck_dr_layout, SoA [k][n_envs]) written by duck_randomize. `reward`,
 * `done` are [n_envs]. `scratch` (nullable unless feet can collide) = n_envs*nv*nv floats
 * for the rare dense-Hessian path. */
int duck_step(duck_sim* sim, int n_envs, float* fstate, int32_t* istate, const float* dr, const float* action,
              float* obs, float* priv, float* reward, float* done, float* scratch, void* stream);

/* domain_randomize: fill dr (SoA [duck_dr_layout.nfloat][n_envs]) for global env ids
 * [env_offset, env_offset + n_envs). */
int duck_randomize(duck_sim* sim, int n_envs, float* dr, uint64_t seed, int64_t env_offset, void* stream);

/* mjx_env.step on raw physics state (SoA [k][n_envs]): qpos [nq], qvel/qacc_warmstart [nv],
 * ctrl [nu]. n_substeps = 0 runs one forward pass without integration. `aux` (nullable)
 * receives the last substep's forward record (duck_aux_size floats per env, SoA). */
int duck_physics_step(duck_sim* sim, int n_envs, float* qpos, float* qvel, float* qacc_warmstart, const float* ctrl,
                      const float* dr, int n_substeps, float* aux, float* scratch, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DUCK_H_ */
