// duck_env_kernels.h — Joystick env kernels for MI355X (gfx950), templated on the model.
//
// One launch per env-step runs the whole of Joystick.step (joystick.py:323-481):
// imitation phase + reference motion, action delay, push, motor-target rate limit, 10
// fused physics substeps (duck_team.h: 16 lanes per env; duck_physics.h: one lane per env),
// contacts, obs, termination, rewards, info bookkeeping, and (optionally) the training
// wrappers EpisodeWrapper + BraxAutoResetWrapper. Per-env state never leaves LDS between
// substeps; HBM sees one read and one write of the state per env-step.
//
// Included by one variant_*.hip per compiled model (after its generated header), which
// instantiates the kernels and exports a VariantOps table; duck_capi.hip dispatches.
#pragma once
#include "duck_common.h"
#include "duck_physics.h"
#include "duck_team.h"

// per-step RNG slot map (identical to oracle/duck_oracle.c)
enum { SLOT_ACTION_DELAY = 0, SLOT_PUSH_THETA = 1, SLOT_PUSH_MAG = 2, SLOT_GYRO = 3, SLOT_ACCEL = 6,
       SLOT_GRAVITY = 9, SLOT_IMU_IDX = 12, SLOT_QPOS = 13, SLOT_QVEL = 29, SLOT_CMD = 45 };
enum { RSLOT_DXY = 0, RSLOT_YAW = 2, RSLOT_QSCALE = 3, RSLOT_QVEL = 19, RSLOT_CMD = 25, RSLOT_PUSH = 33,
       RSLOT_OBS = 64 };
#define KEY_TAG_ENV 0x5EEDu
#define KEY_TAG_DR 0xD0D0u
#define PI_F 3.14159265358979323846f

struct KArgs {
  int n;
  float* fs;
  int32_t* is;
  const float* dr;
  const float* action;
  float* obs;
  float* priv;
  float* reward;
  float* done;
  float* scratch;
  const uint8_t* mask;
  uint64_t seed;
  int64_t env_offset;
  const float* frames;
  const float* hfield;
  RefMeta ref;
  duck_env_config cfg;
  duck_layout lay;
  duck_dr_layout drl;
  unsigned* err;  // the handle's sticky device error word (host-mapped; duck_device_error)
};

// Launch geometry: 16 lanes per env (a team), 16 envs (4 waves) per workgroup, so 4096 envs are
// exactly one workgroup per CU.
constexpr int WG = 16;
constexpr int EPW = 4;
constexpr int TPB = WG * TEAM;
static_assert(TPB == TPB_TEAM, "load_model_tables assumes the kernels' block size");
constexpr int SW = 1;  // slice stride (contiguous per-env slices)

// this lane's env within the workgroup (-1: idle lane) and its rank in the env's team
DK int local_env(int& lane) {
  lane = threadIdx.x % TEAM;
  return threadIdx.x / TEAM;
}

template <class Md, int LAT = 0>
DK Slice<SW> env_slice(float* lds, int t) {
  return Slice<SW>{(lds_float*)(lds + t * TLay<Md, LAT>::STRIDE)};
}

template <class Md>
DK void phys_step(Slice<SW> L, int lane, bool integrate, bool want_out, float* aux, int aux_stride, float* scratch,
                  int sstride, const float* hfield) {
  TPhys<Md>::step(L.p, lane, integrate, want_out, aux, aux_stride, scratch, sstride, hfield);
}

// the physics_kernel (mjx_env.step / mjx.forward parity entry) runs its substeps through one
// out-of-line copy: no values hoisted across substeps, one call site for both modes, so the
// test harness stays well inside the register file (two inlined copies plus the rare-path calls
// needed 512 VGPRs + 86 spilled, the pressure under which the allocator misplaced split copies
// ahead of an exec restore)
template <class Md>
__device__ __noinline__ void phys_step_dni(Slice<SW> L, int lane, bool integrate, bool want_out, float* aux,
                                           int aux_stride, float* scratch, int sstride, const float* hfield) {
  phys_step<Md>(L, lane, integrate, want_out, aux, aux_stride, scratch, sstride, hfield);
}

template <int WG>
struct Col {  // SoA accessor for env e
  float* p;
  int n;
  DK float& operator[](int k) const { return p[(size_t)k * n]; }
};
struct LCol {  // the env's hot state staged in LDS (step_kernel, team mode)
  lds_float* p;
  DK lds_float& operator[](int k) const { return p[k]; }
};

// PolyReferenceMotion.get_reference_motion (poly_reference_motion.py:148-168)
DK int nearest(const float* g, int n, float v) {
  int best = 0;
  float bd = fabsf(g[0] - v);
  for (int i = 1; i < 16; i++) {
    if (i >= n) break;
    const float d = fabsf(g[i] - v);
    if (d < bd) { bd = d; best = i; }
  }
  return best;
}
DK void reference_motion(const KArgs& A, float dx, float dy, float dth, int i, float* out) {
  const RefMeta& R = A.ref;
  dx = fminf(fmaxf(dx, R.dx_range[0]), R.dx_range[1]);
  dy = fminf(fmaxf(dy, R.dy_range[0]), R.dy_range[1]);
  dth = fminf(fmaxf(dth, R.dtheta_range[0]), R.dtheta_range[1]);
  const int ix = nearest(R.dxs, R.n_dx, dx), iy = nearest(R.dys, R.n_dy, dy), it = nearest(R.dthetas, R.n_dtheta, dth);
  // t = (i % nb) / nb takes nb values: the table holds the polynomials pre-evaluated there
  const int nb = R.nb;
  const int ph = ((i % nb) + nb) % nb;
  const float4* f = reinterpret_cast<const float4*>(
      A.frames + ((size_t)((ix * R.n_dy + iy) * R.n_dtheta + it) * nb + ph) * 40);
#pragma unroll
  for (int d = 0; d < 10; d++) {
    const float4 v = f[d];
    out[4 * d] = v.x; out[4 * d + 1] = v.y; out[4 * d + 2] = v.z; out[4 * d + 3] = v.w;
  }
}

DK float nan_to_num(float x) {
  if (isnan(x)) return 0.0f;
  if (isinf(x)) return x > 0 ? 3.4028234663852886e38f : -3.4028234663852886e38f;
  return x;
}

template <class RT>
DK void sample_command(const duck_env_config& c, const RT& r, int slot, float* cmd) {
  const float f = c.head_range_factor;
  cmd[0] = r.uniform(slot + 0, c.lin_vel_x[0], c.lin_vel_x[1]);
  cmd[1] = r.uniform(slot + 1, c.lin_vel_y[0], c.lin_vel_y[1]);
  cmd[2] = r.uniform(slot + 2, c.ang_vel_yaw[0], c.ang_vel_yaw[1]);
  cmd[3] = r.uniform(slot + 3, c.neck_pitch_range[0] * f, c.neck_pitch_range[1] * f);
  cmd[4] = r.uniform(slot + 4, c.head_pitch_range[0] * f, c.head_pitch_range[1] * f);
  cmd[5] = r.uniform(slot + 5, c.head_yaw_range[0] * f, c.head_yaw_range[1] * f);
  cmd[6] = r.uniform(slot + 6, c.head_roll_range[0] * f, c.head_roll_range[1] * f);
  if (r.u(slot + 7) < 0.1f)
    for (int k = 0; k < 7; k++) cmd[k] = 0.0f;
}

// per-env model values: nominal (constexpr) or this env's domain-randomised record
template <class Md, int WG>
DK void load_dyn(const KArgs& A, int e, Slice<WG> L) {
  using Ly = Lay<Md>;
  Phys<Md, WG>::set_nominal(L);
  if (A.dr) {
    const duck_dr_layout& D = A.drl;
    const int n = A.n;
#pragma unroll
    for (int k = 0; k < 3; k++) L[Ly::DIPOS + k] = A.dr[(size_t)(D.base_ipos + k) * n + e];
#pragma unroll
    for (int b = 0; b < Md::NB; b++) L[Ly::DMASS + b] = A.dr[(size_t)(D.body_mass + b) * n + e];
#pragma unroll
    for (int a = 0; a < Md::NU; a++) {
      L[Ly::DFRIC + Md::actuator_dof[a]] = A.dr[(size_t)(D.frictionloss + a) * n + e];
      L[Ly::DARM + Md::actuator_dof[a]] = A.dr[(size_t)(D.armature + a) * n + e];
      L[Ly::DQ0 + Md::actuator_qadr[a]] = A.dr[(size_t)(D.qpos0 + a) * n + e];
      L[Ly::DKP + a] = A.dr[(size_t)(D.kp + a) * n + e];
    }
  }
}

// load_dyn with the team's lanes: nominal block from the LDS model blob, then the env's DR record
template <class Md, int LAT = 0>
DK void load_dyn_team(const KArgs& A, int e, Slice<SW> L, int lane) {
  using Ly = Lay<Md>;
  using TP = TPhys<Md, LAT>;
  constexpr int NDYN = Md::NB + 3 + 2 * Md::NV + Md::NQ + Md::NU;
  static_assert(Ly::DKP + Md::NU - Ly::DMASS == NDYN, "contiguous per-env model block");
  for (int k = lane; k < NDYN; k += TEAM) L[Ly::DMASS + k] = TP::tf(Md::B_NOM + k);
  if (A.dr) {
    TSYNC();
    const duck_dr_layout& D = A.drl;
    const int n = A.n;
    if (lane < 3) L[Ly::DIPOS + lane] = A.dr[(size_t)(D.base_ipos + lane) * n + e];
    for (int b = lane; b < Md::NB; b += TEAM) L[Ly::DMASS + b] = A.dr[(size_t)(D.body_mass + b) * n + e];
    if (lane < Md::NU) {
      const int a = lane, o = Md::B_ACT + 12 * a, dof = TP::ti(o + 5), qadr = TP::ti(o + 4);
      L[Ly::DFRIC + dof] = A.dr[(size_t)(D.frictionloss + a) * n + e];
      L[Ly::DARM + dof] = A.dr[(size_t)(D.armature + a) * n + e];
      L[Ly::DQ0 + qadr] = A.dr[(size_t)(D.qpos0 + a) * n + e];
      L[Ly::DKP + a] = A.dr[(size_t)(D.kp + a) * n + e];
    }
  }
}

// Joystick._get_obs (joystick.py:487-620) / Standing._get_obs (standing.py:462-575); reads the
// last forward's outputs from the slice
// Observation sinks: GObs writes obs/priv rows in HBM directly; SObs stages the privileged row
// (whose prefix is the state row) in the env slice's dead H/row storage, from where the team
// stores both rows with coalesced 16-lane stores (step_kernel)
struct GObs {
  float* obs;
  float* priv;
  int obs_size;
  DK void operator()(int k, float v) const {
    if (k < obs_size) obs[k] = v;
    priv[k] = v;
  }
};
template <int WG>
struct SObs {
  Slice<WG> L;
  int base;
  DK void operator()(int k, float v) const { L[base + k] = v; }
};

template <class Md, int WG, class FA, class OS, class RT>
DK void write_obs(const KArgs& A, int e, Slice<WG> L, const FA& F, const OS& out, const RT& r, int slot_base,
                  int imitation_i) {
  using Ly = Lay<Md>;
  const duck_env_config& c = A.cfg;
  const duck_layout& Lo = A.lay;
  constexpr int NU = Md::NU;
  float gyro[3], acc[3], grav[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    gyro[k] = L[Ly::SENS + c.sens_gyro + k];
    acc[k] = L[Ly::SENS + c.sens_accelerometer + k];
    grav[k] = -L[Ly::IMUR + k];
  }
  float ngrav[3];
#pragma unroll
  for (int k = 0; k < 3; k++)
    ngrav[k] = grav[k] + (2.0f * r.u(slot_base + SLOT_GRAVITY + k) - 1.0f) * c.noise_level * c.noise_gravity;
  // IMU delay history (joystick.py:521-530); the delayed sample is never emitted
#pragma unroll
  for (int k = 8; k >= 3; k--) F[Lo.imu_history + k] = F[Lo.imu_history + k - 3];
#pragma unroll
  for (int k = 0; k < 3; k++) F[Lo.imu_history + k] = ngrav[k];
  int o = 0;
  auto put = [&](float v) { out(o++, v); };
#pragma unroll
  for (int k = 0; k < 3; k++) put(gyro[k] + (2.0f * r.u(slot_base + SLOT_GYRO + k) - 1.0f) * c.noise_level * c.noise_gyro);
#pragma unroll
  for (int k = 0; k < 3; k++)
    put(acc[k] + (2.0f * r.u(slot_base + SLOT_ACCEL + k) - 1.0f) * c.noise_level * c.noise_accelerometer);
#pragma unroll
  for (int k = 0; k < 7; k++) put(F[Lo.command + k]);
  for (int a = 0; a < NU; a++) {
    float ja = L[Ly::QPOS + c.actuator_qposadr[a]];
    if (c.backlash_qposadr[a] >= 0) ja += L[Ly::QPOS + c.backlash_qposadr[a]];
    put(ja + (2.0f * r.u(slot_base + SLOT_QPOS + a) - 1.0f) * c.noise_level * c.qpos_noise_scale[a] - c.default_actuator[a]);
  }
  for (int a = 0; a < NU; a++) {
    const float jv = L[Ly::QVEL + c.actuator_qveladr[a]];
    put((jv + (2.0f * r.u(slot_base + SLOT_QVEL + a) - 1.0f) * c.noise_level * c.noise_joint_vel) * c.dof_vel_scale);
  }
  for (int a = 0; a < NU; a++) put(F[Lo.last_act + a]);
  for (int a = 0; a < NU; a++) put(F[Lo.last_last_act + a]);
  for (int a = 0; a < NU; a++) put(F[Lo.last_last_last_act + a]);
  const bool joystick = Lo.task == DUCK_TASK_JOYSTICK;
  if (joystick)
    for (int a = 0; a < NU; a++) put(F[Lo.motor_targets + a]);
  put(L[Ly::OCON]);
  put(L[Ly::OCON + 1]);
  if (joystick) {
    put(F[Lo.imitation_phase]);
    put(F[Lo.imitation_phase + 1]);
  }
  int p = o;
  auto pp = [&](float v) { out(p++, v); };
#pragma unroll
  for (int k = 0; k < 3; k++) pp(gyro[k]);
#pragma unroll
  for (int k = 0; k < 3; k++) pp(acc[k]);
#pragma unroll
  for (int k = 0; k < 3; k++) pp(grav[k]);
#pragma unroll
  for (int k = 0; k < 3; k++) pp(L[Ly::SENS + c.sens_local_linvel + k]);
#pragma unroll
  for (int k = 0; k < 3; k++) pp(L[Ly::SENS + c.sens_global_angvel + k]);
  for (int a = 0; a < NU; a++) {
    float ja = L[Ly::QPOS + c.actuator_qposadr[a]];
    if (c.backlash_qposadr[a] >= 0) ja += L[Ly::QPOS + c.backlash_qposadr[a]];
    pp(ja - c.default_actuator[a]);
  }
  for (int a = 0; a < NU; a++) pp(L[Ly::QVEL + c.actuator_qveladr[a]]);
  pp(L[Ly::QPOS + 2]);
  for (int a = 0; a < NU; a++) pp(L[Ly::AF + a]);
  pp(L[Ly::OCON]);
  pp(L[Ly::OCON + 1]);
#pragma unroll
  for (int k = 0; k < 3; k++) pp(L[Ly::SENS + c.sens_left_foot_linvel + k]);
#pragma unroll
  for (int k = 0; k < 3; k++) pp(L[Ly::SENS + c.sens_right_foot_linvel + k]);
  pp(F[Lo.feet_air_time]);
  pp(F[Lo.feet_air_time + 1]);
  if (Lo.imitation)
    for (int k = 0; k < 40; k++) pp(F[Lo.ref_motion + k]);
  if (joystick) {
    pp((float)imitation_i);
    pp(F[Lo.imitation_phase]);
    pp(F[Lo.imitation_phase + 1]);
  }
}

// write_obs with the team's lanes splitting the rows (step_kernel): lane a < NU takes actuator
// a's entries, lanes 0-2 the 3-vectors, lanes 0-1 the pairs; same values at the same offsets
template <class Md, class FA, class OS, class RT>
DK void write_obs_team(const KArgs& A, int lane, Slice<SW> L, const FA& F, const OS& out, const RT& r,
                       int imitation_i) {
  using Ly = Lay<Md>;
  const duck_env_config& c = A.cfg;
  const duck_layout& Lo = A.lay;
  constexpr int NU = Md::NU;
  static_assert(NU <= TEAM, "an actuator per lane");
  const bool joystick = Lo.task == DUCK_TASK_JOYSTICK;
  const float nl = c.noise_level;
  // state row offsets (joystick.py:544-560 / standing.py)
  const int OQ = 13, OV = OQ + NU, O1 = OV + NU, O2 = O1 + NU, O3 = O2 + NU, OM = O3 + NU;
  const int OC = joystick ? OM + NU : OM;  // contacts
  const int P = OC + 2 + (joystick ? 2 : 0);  // privileged row continues after the state row
  const int PQ = P + 15, PV = PQ + NU, PZ = PV + NU, PA = PZ + 1, PC = PA + NU, PF = PC + 2, PT = PF + 6, PR = PT + 2;
  const int PI = PR + (Lo.imitation ? 40 : 0);
  if (lane < 3) {
    const int k = lane;
    const float gyro = L[Ly::SENS + c.sens_gyro + k], acc = L[Ly::SENS + c.sens_accelerometer + k];
    const float grav = -L[Ly::IMUR + k];
    const float ngrav = grav + (2.0f * r.u(SLOT_GRAVITY + k) - 1.0f) * nl * c.noise_gravity;
    // IMU delay history (joystick.py:521-530): shift by one sample, the delayed one is never emitted
    const float h0 = F[Lo.imu_history + k], h1 = F[Lo.imu_history + 3 + k];
    F[Lo.imu_history + 6 + k] = h1;
    F[Lo.imu_history + 3 + k] = h0;
    F[Lo.imu_history + k] = ngrav;
    out(k, gyro + (2.0f * r.u(SLOT_GYRO + k) - 1.0f) * nl * c.noise_gyro);
    out(3 + k, acc + (2.0f * r.u(SLOT_ACCEL + k) - 1.0f) * nl * c.noise_accelerometer);
    out(P + k, gyro);
    out(P + 3 + k, acc);
    out(P + 6 + k, grav);
    out(P + 9 + k, L[Ly::SENS + c.sens_local_linvel + k]);
    out(P + 12 + k, L[Ly::SENS + c.sens_global_angvel + k]);
    out(PF + k, L[Ly::SENS + c.sens_left_foot_linvel + k]);
    out(PF + 3 + k, L[Ly::SENS + c.sens_right_foot_linvel + k]);
  }
  if (lane < 7) out(6 + lane, F[Lo.command + lane]);
  if (lane < NU) {
    const int a = lane;
    float ja = L[Ly::QPOS + c.actuator_qposadr[a]];
    if (c.backlash_qposadr[a] >= 0) ja += L[Ly::QPOS + c.backlash_qposadr[a]];
    const float jv = L[Ly::QVEL + c.actuator_qveladr[a]];
    out(OQ + a, ja + (2.0f * r.u(SLOT_QPOS + a) - 1.0f) * nl * c.qpos_noise_scale[a] - c.default_actuator[a]);
    out(OV + a, (jv + (2.0f * r.u(SLOT_QVEL + a) - 1.0f) * nl * c.noise_joint_vel) * c.dof_vel_scale);
    out(O1 + a, F[Lo.last_act + a]);
    out(O2 + a, F[Lo.last_last_act + a]);
    out(O3 + a, F[Lo.last_last_last_act + a]);
    if (joystick) out(OM + a, F[Lo.motor_targets + a]);
    out(PQ + a, ja - c.default_actuator[a]);
    out(PV + a, jv);
    out(PA + a, L[Ly::AF + a]);
  }
  if (lane < 2) {
    const float con = L[Ly::OCON + lane];
    out(OC + lane, con);
    out(PC + lane, con);
    out(PT + lane, F[Lo.feet_air_time + lane]);
    if (joystick) {
      const float ph = F[Lo.imitation_phase + lane];
      out(OC + 2 + lane, ph);
      out(PI + 1 + lane, ph);
    }
  }
  if (lane == 0) {
    out(PZ, L[Ly::QPOS + 2]);
    if (joystick) out(PI, (float)imitation_i);
  }
  if (Lo.imitation)
    for (int k = lane; k < 40; k += TEAM) out(PR + k, F[Lo.ref_motion + k]);
}

template <class Md, int WG>
__global__ void __launch_bounds__(TPB) reset_kernel(KArgs A) {
  using Ly = Lay<Md>;
  {
    extern __shared__ float lds_t[];
    load_model_tables<Md>(lds_t);
  }
  int lane;
  const int t = local_env(lane);
  if (t < 0) return;
  const int e = blockIdx.x * WG + t;
  if (e >= A.n) return;
  if (A.mask && !A.mask[e]) return;
  extern __shared__ float lds[];
  const Slice<SW> L = env_slice<Md>(lds, t);
  const duck_env_config& c = A.cfg;
  const duck_layout& Lo = A.lay;
  constexpr int NQ = Md::NQ, NV = Md::NV, NU = Md::NU;
  Col<0> F{A.fs + e, A.n};
  auto iset = [&](int k, int32_t v) { A.is[(size_t)k * A.n + e] = v; };
  for (int k = 0; k < Lo.nfloat; k++) F[k] = 0.0f;
  for (int k = 0; k < Lo.nint; k++) iset(k, 0);
  Rng r;
  derive_key(A.seed, A.env_offset + e, KEY_TAG_ENV, r.k0, r.k1);
  r.ctr = 0;
  load_dyn<Md, SW>(A, e, L);
  // Joystick.reset (joystick.py:206-258)
  for (int i = 0; i < NQ; i++) L[Ly::QPOS + i] = c.init_qpos[i];
  for (int i = 0; i < NV; i++) { L[Ly::QVEL + i] = 0.0f; L[Ly::WARM + i] = 0.0f; }
  L[Ly::QPOS + 0] += r.uniform(RSLOT_DXY + 0, -0.05f, 0.05f);
  L[Ly::QPOS + 1] += r.uniform(RSLOT_DXY + 1, -0.05f, 0.05f);
  {
    const float yaw = r.uniform(RSLOT_YAW, -3.14f, 3.14f);
    float s, co;
    sincosf(0.5f * yaw, &s, &co);
    const float qy[4] = {co, 0.0f, 0.0f, s};
    float q[4] = {L[Ly::QPOS + 3], L[Ly::QPOS + 4], L[Ly::QPOS + 5], L[Ly::QPOS + 6]};
    qmul(q, q, qy);
    for (int k = 0; k < 4; k++) L[Ly::QPOS + 3 + k] = q[k];
  }
  for (int a = 0; a < NU; a++) L[Ly::QPOS + c.actuator_qposadr[a]] *= r.uniform(RSLOT_QSCALE + a, 0.5f, 1.5f);
  // base velocity U(+-0.05) (joystick.py:247-249); U(+-0.5) for Standing (standing.py:247-249)
  const float vr = Lo.task == DUCK_TASK_STANDING ? 0.5f : 0.05f;
  for (int k = 0; k < 6; k++) L[Ly::QVEL + k] = r.uniform(RSLOT_QVEL + k, -vr, vr);
  for (int a = 0; a < NU; a++) L[Ly::CTRL + a] = L[Ly::QPOS + c.actuator_qposadr[a]];
  phys_step<Md>(L, lane, false, true, nullptr, 0, A.scratch ? A.scratch + e : nullptr, A.n, A.hfield);
  float cmd[7];
  sample_command(c, r, RSLOT_CMD, cmd);
  const float push_interval = r.uniform(RSLOT_PUSH, c.push_interval_range[0], c.push_interval_range[1]);
  iset(Lo.push_interval, (int32_t)rintf(push_interval / c.ctrl_dt));
  iset(Lo.rng_key, (int32_t)r.k0);
  iset(Lo.rng_key + 1, (int32_t)r.k1);
  iset(Lo.rng_ctr, 1);
  for (int k = 0; k < 7; k++) F[Lo.command + k] = cmd[k];
  // info["motor_targets"]: home ctrl (joystick.py:285) / zeros (standing.py:279)
  for (int a = 0; a < NU; a++) F[Lo.motor_targets + a] = Lo.task == DUCK_TASK_STANDING ? 0.0f : c.default_actuator[a];
  if (Lo.imitation) {
    float ref[40];
    reference_motion(A, cmd[0], cmd[1], cmd[2], 0, ref);
    for (int k = 0; k < 40; k++) F[Lo.ref_motion + k] = ref[k];
  }
  for (int i = 0; i < NQ; i++) { F[Lo.qpos + i] = L[Ly::QPOS + i]; F[Lo.first_qpos + i] = L[Ly::QPOS + i]; }
  for (int i = 0; i < NV; i++) {
    F[Lo.qvel + i] = L[Ly::QVEL + i]; F[Lo.first_qvel + i] = L[Ly::QVEL + i];
    F[Lo.qacc_warmstart + i] = L[Ly::WARM + i]; F[Lo.first_qacc_warmstart + i] = L[Ly::WARM + i];
  }
  for (int a = 0; a < NU; a++) { F[Lo.ctrl + a] = L[Ly::CTRL + a]; F[Lo.first_ctrl + a] = L[Ly::CTRL + a]; }
  write_obs<Md, SW>(A, e, L, F, GObs{A.obs + (size_t)e * Lo.obs_size, A.priv + (size_t)e * Lo.priv_size, Lo.obs_size},
                    r, RSLOT_OBS, 0);
  for (int k = 0; k < Lo.obs_size; k++) F[Lo.first_obs + k] = A.obs[(size_t)e * Lo.obs_size + k];
  for (int k = 0; k < Lo.priv_size; k++) F[Lo.first_priv + k] = A.priv[(size_t)e * Lo.priv_size + k];
}

// the per-env values step_env reads from HBM besides the hot state: integer counters, the RNG
// key, this lane's action. Loaded by one batch of independent loads issued together with the
// hot-state loads, so the step waits for one memory round trip instead of three
struct StepPre {
  int32_t step, push_step, push_interval, ep_steps, imitation_i;
  uint32_t k0, k1, ctr;
  float act;
};
template <class Md>
DK StepPre step_prefetch(const KArgs& A, int e, int lane) {
  static_assert(Md::NU <= TEAM, "an actuator per lane");
  const duck_layout& Lo = A.lay;
  const int n = A.n, ec = e < n ? e : 0;
  auto ig = [&](int k) { return A.is[(size_t)k * n + ec]; };
  StepPre P;
  P.step = ig(Lo.step);
  P.push_step = ig(Lo.push_step);
  P.push_interval = ig(Lo.push_interval);
  P.ep_steps = ig(Lo.ep_steps);
  P.imitation_i = ig(Lo.imitation_i);
  P.k0 = (uint32_t)ig(Lo.rng_key);
  P.k1 = (uint32_t)ig(Lo.rng_key + 1);
  P.ctr = (uint32_t)ig(Lo.rng_ctr);
  P.act = A.action[(size_t)ec * Md::NU + (lane < Md::NU ? lane : 0)];
  return P;
}

// for (i = l0; i < N; i += TS) f(i) with the trip count unrolled at compile time (l0 < TS): straight-line
// code instead of a loop whose trip count depends on the lane (team mode: l0 = lane, TS = TEAM)
template <int N, int TS, class Fn>
DK void strided_for(int l0, Fn&& f) {
#pragma unroll
  for (int s = 0; s < (N + TS - 1) / TS; s++) {
    const int i = l0 + TS * s;
    if (TS * (s + 1) <= N || i < N) f(i);
  }
}

// Joystick.step body for env e (joystick.py:323-481 + wrappers); F = the env's hot state
// (LDS-staged or the global row), G = the global row (auto-reset snapshot)
template <class Md, class FA, bool STAGE_OBS, class RT, int LAT = 0>
DK void step_env(const KArgs& A, int e, int lane, Slice<SW> L, const FA& F, const Col<0>& G, const RT& r,
                 const StepPre& P) {
  using Ly = Lay<Md>;
  const duck_env_config& c = A.cfg;
  const duck_layout& Lo = A.lay;
  constexpr int NQ = Md::NQ, NV = Md::NV, NU = Md::NU;
  const int n = A.n;
  STAGE_T0();
  auto iset = [&](int k, int32_t v) { A.is[(size_t)k * n + e] = v; };
  const float dt = c.ctrl_dt;
  // every integer counter was read up front (step_prefetch; a global load issued after the obs
  // stores would wait for them: vmcnt counts stores too on CDNA)
  const int step_prev = P.step, push_step = P.push_step, push_interval = P.push_interval;
  int ep_steps = P.ep_steps;
  if (c.auto_reset && F[Lo.done] != 0.0f) ep_steps = 0;
  int imitation_i = P.imitation_i;
  if (Lo.imitation) {  // joystick.py:325-355
    const int nb = A.ref.nb;
    imitation_i = (imitation_i + 1) % nb;
    const float ph = ((float)imitation_i / (float)nb) * 2.0f * PI_F;
    F[Lo.imitation_phase] = cosf(ph);
    F[Lo.imitation_phase + 1] = sinf(ph);
    float ref[40];
    reference_motion(A, F[Lo.command], F[Lo.command + 1], F[Lo.command + 2], imitation_i, ref);
    for (int k = 0; k < 40; k++) F[Lo.ref_motion + k] = ref[k];
  } else {
    imitation_i = 0;
  }
  // action delay (joystick.py:362-376): history = [a_t, a_{t-1}, a_{t-2}]
  const int didx = r.randint(SLOT_ACTION_DELAY, c.action_min_delay, c.action_max_delay);
  float arate = 0.0f;
  for (int a = STAGE_OBS ? lane : 0; a < NU; a += STAGE_OBS ? TEAM : 1) {
    const float act = STAGE_OBS ? P.act : A.action[(size_t)e * NU + a];
    const float h1 = F[Lo.action_history + a], h2 = F[Lo.action_history + NU + a];
    F[Lo.action_history + a] = act;
    F[Lo.action_history + NU + a] = h1;
    F[Lo.action_history + 2 * NU + a] = h2;
    const float ad = didx == 0 ? act : (didx == 1 ? h1 : h2);
    float mt = c.default_actuator[a] + ad * c.action_scale;  // joystick.py:404-417
    if (c.use_motor_speed_limits) {
      const float prev = F[Lo.motor_targets + a], lim = c.max_motor_velocity * dt;
      mt = fminf(fmaxf(mt, prev - lim), prev + lim);
    }
    L[Ly::CTRL + a] = mt;
    const float la = F[Lo.last_act + a];
    arate += (act - la) * (act - la);
  }
  // push (joystick.py:381-400)
  const float theta = r.uniform(SLOT_PUSH_THETA, 0.0f, 2.0f * PI_F);
  const float mag = r.uniform(SLOT_PUSH_MAG, c.push_magnitude_range[0], c.push_magnitude_range[1]);
  // jp.mod(push_step + 1, interval) == 0 (joystick.py:388-390); an interval that rounds to 0 steps
  // never pushes (XLA integer remainder by zero returns the dividend), and never divides by zero here
  const float gate = (push_interval != 0 && (push_step + 1) % push_interval == 0) ? 1.0f : 0.0f;
  const float push[2] = {cosf(theta) * gate * (float)c.push_enable, sinf(theta) * gate * (float)c.push_enable};
  if constexpr (STAGE_OBS) {  // team: lane-split copies, sums by DPP
    arate = tsum(arate);
    strided_for<NQ, TEAM>(lane, [&](int i) { L[Ly::QPOS + i] = F[Lo.qpos + i]; });
    strided_for<NV, TEAM>(lane, [&](int i) {
      L[Ly::QVEL + i] = F[Lo.qvel + i] + (i == 0 ? push[0] * mag : (i == 1 ? push[1] * mag : 0.0f));
      L[Ly::WARM + i] = F[Lo.qacc_warmstart + i];
    });
    load_dyn_team<Md, LAT>(A, e, L, lane);
    TSYNC();
  } else {
    for (int i = 0; i < NQ; i++) L[Ly::QPOS + i] = F[Lo.qpos + i];
    for (int i = 0; i < NV; i++) { L[Ly::QVEL + i] = F[Lo.qvel + i]; L[Ly::WARM + i] = F[Lo.qacc_warmstart + i]; }
    L[Ly::QVEL + 0] += push[0] * mag;
    L[Ly::QVEL + 1] += push[1] * mag;
    load_dyn<Md, SW>(A, e, L);
  }
  // physics (joystick.py:420)
  float* scr = A.scratch ? A.scratch + e : nullptr;
  STAGE_MARK(29);
  if constexpr (LAT) {
    // wave 0's share of each substep (the paired kernel: wave A's); the other waves run theirs in
    // step_kernel_lat. The env code below reads the last substep's state and sensors: wait for Euler
    using TPL = TPhys<Md, LAT>;
    (void)scr;
    LAT_T(43, 5);
    for (int s = 0; s < c.n_substeps; s++) {
      if constexpr (LAT == 2) TPL::lat2_a(L.p, lane, s, A.hfield);
      else TPL::lat_r0(L.p, lane, s);
    }
    TPL::ev_wait(TPL::EV_EULER, c.n_substeps);
    LAT_T(44, 5);
  } else {
    for (int s = 0; s < c.n_substeps; s++)
      phys_step<Md>(L, lane, true, s == c.n_substeps - 1, nullptr, 0, scr, n, A.hfield);
  }
  STAGE_RESET();
  for (int a = STAGE_OBS ? lane : 0; a < NU; a += STAGE_OBS ? TEAM : 1) {
    F[Lo.motor_targets + a] = L[Ly::CTRL + a];
    F[Lo.ctrl + a] = L[Ly::CTRL + a];
  }
  const float con[2] = {L[Ly::OCON], L[Ly::OCON + 1]};
  // feet bookkeeping (joystick.py:424-435)
  for (int k = 0; k < 2; k++) {
    F[Lo.feet_air_time + k] = F[Lo.feet_air_time + k] + dt;
    F[Lo.swing_peak + k] = fmaxf(F[Lo.swing_peak + k], L[Ly::FOOTZ + k]);
  }
  if constexpr (STAGE_OBS) {
    static_assert(DUCK_OBS_SIZE(NU) + 15 + 3 * NU + 1 + 2 + 6 + 2 + 40 + 1 + 2 <= Ly::SCR_OBS && Ly::SCR_OBS <= Ly::HSZ + 4 * Ly::NROW,
                  "privileged row must fit in the H/row storage");
    write_obs_team<Md>(A, lane, L, F, SObs<SW>{L, Ly::H}, r, imitation_i);
    TSYNC();
  } else {
    write_obs<Md, SW>(A, e, L, F, GObs{A.obs + (size_t)e * Lo.obs_size, A.priv + (size_t)e * Lo.priv_size, Lo.obs_size},
                      r, 0, imitation_i);
  }
  STAGE_MARK(30);
  // team mode: the per-actuator / per-dof loops below are split over the team's lanes and
  // their sums combined by DPP row reductions (single-lane mode: TS = 1, plain loops)
  constexpr int TS = STAGE_OBS ? TEAM : 1;
  const int l0 = STAGE_OBS ? lane : 0;
  auto red = [&](float v) {
    if constexpr (STAGE_OBS) return tsum(v);
    else return v;
  };
  // termination (joystick.py:483-485)
  float nanp = 0.0f;
  strided_for<NQ, TS>(l0, [&](int i) { nanp += isnan(L[Ly::QPOS + i]) ? 1.0f : 0.0f; });
  strided_for<NV, TS>(l0, [&](int i) { nanp += isnan(L[Ly::QVEL + i]) ? 1.0f : 0.0f; });
  const bool nan = red(nanp) > 0.0f;
  float done = (L[Ly::SENS + c.sens_upvector + 2] < 0.0f || nan) ? 1.0f : 0.0f;
  // rewards (joystick.py:622-669, common/rewards.py:11-125, custom_rewards.py:4-148)
  float cmd[7];
  for (int k = 0; k < 7; k++) cmd[k] = F[Lo.command + k];
  const float lv0 = L[Ly::SENS + c.sens_local_linvel], lv1 = L[Ly::SENS + c.sens_local_linvel + 1];
  const float gz = L[Ly::SENS + c.sens_gyro + 2];
  const float sigma = c.tracking_sigma;
  const float ex = (cmd[0] - lv0) * (cmd[0] - lv0);
  const float ey = fmaxf(fabsf(lv1 - cmd[1]) - 0.1f, 0.0f);
  const float r_lin = nan_to_num(expf(-(ex + ey * ey) / sigma));
  const float r_ang = nan_to_num(expf(-((cmd[2] - gz) * (cmd[2] - gz)) / sigma));
  const bool standing = Lo.task == DUCK_TASK_STANDING;
  float torq = 0.0f, pc = 0.0f, vc = 0.0f, lpc = 0.0f, lvc = 0.0f, hp = 0.0f;
  for (int a = l0; a < NU; a += TS) {
    const float f = L[Ly::AF + a];
    const float q = L[Ly::QPOS + c.actuator_qposadr[a]], qd = fabsf(L[Ly::QVEL + c.actuator_qveladr[a]]);
    const float dq = fabsf(q - c.default_actuator[a]);
    torq += f * f;
    pc += dq;
    vc += qd;
    if (standing) {
      if (a < 5 || a >= NU - 5) {  // legs: qpos[:5] and qpos[9:]
        lpc += dq;
        lvc += qd;
      } else {  // head joints qpos[5:9] vs cmd[3:]
        const float d = q - cmd[3 + a - 5];
        hp += d * d;
      }
    }
  }
  torq = red(torq);
  pc = red(pc);
  vc = red(vc);
  const float cn = sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1] + cmd[2] * cmd[2]);
  const float r_still = nan_to_num(pc + vc) * (cn < 0.01f ? 1.0f : 0.0f);
  float imit = 0.0f;
  if (Lo.imitation) {
    const int R0 = Lo.ref_motion;
    float lxy = 0.0f, axy = 0.0f;
    for (int k = 0; k < 2; k++) {
      const float dv = L[Ly::QVEL + k] - F[R0 + 34 + k], dw = L[Ly::QVEL + 3 + k] - F[R0 + 37 + k];
      lxy += dv * dv;
      axy += dw * dw;
    }
    const float dz = L[Ly::QVEL + 2] - F[R0 + 36], dwz = L[Ly::QVEL + 5] - F[R0 + 39];
    const float lin_xy = expf(-8.0f * lxy), lin_z = expf(-8.0f * dz * dz);
    const float ang_xy = expf(-2.0f * axy) * 0.5f, ang_z = expf(-2.0f * dwz * dwz) * 0.5f;
    float jp = 0.0f, jv = 0.0f;
    for (int k = l0; k < 5; k += TS) {
      const float q1 = L[Ly::QPOS + c.actuator_qposadr[k]] - F[R0 + k];
      const float q2 = L[Ly::QPOS + c.actuator_qposadr[NU - 5 + k]] - F[R0 + 11 + k];
      const float v1 = L[Ly::QVEL + c.actuator_qveladr[k]] - F[R0 + 16 + k];
      const float v2 = L[Ly::QVEL + c.actuator_qveladr[NU - 5 + k]] - F[R0 + 27 + k];
      jp += q1 * q1 + q2 * q2;
      jv += v1 * v1 + v2 * v2;
    }
    jp = red(jp);
    jv = red(jv);
    float contact_r = 0.0f;
    for (int k = 0; k < 2; k++) contact_r += (con[k] == (F[R0 + 32 + k] > 0.5f ? 1.0f : 0.0f)) ? 1.0f : 0.0f;
    float rr = lin_xy + lin_z + ang_xy + ang_z + (-jp * 15.0f) + (-jv * 1e-3f) + contact_r;
    rr *= cn > 0.01f ? 1.0f : 0.0f;
    imit = nan_to_num(rr);
  }
  float terms[7];
  if (standing) {
    // Standing._get_reward (standing.py:584-606): orientation, torques, action_rate, alive,
    // stand_still(ignore_head=True), head_pos (common/rewards.py:45-46,93-117,131-147)
    lpc = red(lpc);
    lvc = red(lvc);
    hp = red(hp);
    const float ux = L[Ly::SENS + c.sens_upvector], uy = L[Ly::SENS + c.sens_upvector + 1];
    terms[0] = nan_to_num(ux * ux + uy * uy) * c.scale_orientation;
    terms[1] = nan_to_num(torq) * c.scale_torques;
    terms[2] = nan_to_num(arate) * c.scale_action_rate;
    terms[3] = 1.0f * c.scale_alive;
    terms[4] = nan_to_num(lpc + lvc) * (cn < 0.01f ? 1.0f : 0.0f) * c.scale_stand_still;
    terms[5] = nan_to_num(hp) * (cn > 0.01f ? 1.0f : 0.0f) * c.scale_head_pos;
    terms[6] = 0.0f;
  } else {
    terms[0] = r_lin * c.scale_tracking_lin_vel;
    terms[1] = r_ang * c.scale_tracking_ang_vel;
    terms[2] = nan_to_num(torq) * c.scale_torques;
    terms[3] = nan_to_num(arate) * c.scale_action_rate;
    terms[4] = 1.0f * c.scale_alive;
    terms[5] = imit * c.scale_imitation;
    terms[6] = r_still * c.scale_stand_still;
  }
  float sum = 0.0f;
  for (int k = 0; k < 7; k++) sum += terms[k];
  const float reward = fminf(fmaxf(sum * dt, 0.0f), 10000.0f);
  // info bookkeeping (joystick.py:449-477)
  F[Lo.push] = push[0];
  F[Lo.push + 1] = push[1];
  int step = step_prev + 1;
  iset(Lo.push_step, push_step + 1);
  strided_for<NU, TS>(l0, [&](int a) {
    F[Lo.last_last_last_act + a] = F[Lo.last_last_act + a];
    F[Lo.last_last_act + a] = F[Lo.last_act + a];
    F[Lo.last_act + a] = F[Lo.action_history + a];  // this step's action
  });
  if (step > 500) {
    float nc[7];
    sample_command(c, r, SLOT_CMD, nc);
    for (int k = 0; k < 7; k++) F[Lo.command + k] = nc[k];
  }
  if (done != 0.0f || step > 500) step = 0;
  iset(Lo.step, step);
  iset(Lo.imitation_i, imitation_i);
  for (int k = 0; k < 2; k++) {
    F[Lo.feet_air_time + k] = F[Lo.feet_air_time + k] * (con[k] != 0.0f ? 0.0f : 1.0f);
    F[Lo.last_contact + k] = con[k];
    F[Lo.swing_peak + k] = F[Lo.swing_peak + k] * (con[k] != 0.0f ? 0.0f : 1.0f);
  }
  // metrics: reward/<k> = term, cost/<k> = -term (joystick.py:467-474, standing.py:424-431)
  const float scales[7] = {standing ? c.scale_orientation : c.scale_tracking_lin_vel,
                           standing ? c.scale_torques : c.scale_tracking_ang_vel,
                           standing ? c.scale_action_rate : c.scale_torques,
                           standing ? c.scale_alive : c.scale_action_rate,
                           standing ? c.scale_stand_still : c.scale_alive,
                           standing ? c.scale_head_pos : c.scale_imitation,
                           standing ? 0.0f : c.scale_stand_still};
  for (int k = 0; k < 7; k++) F[Lo.metrics + k] = scales[k] > 0.0f ? terms[k] : -terms[k];
  F[Lo.metrics + DUCK_M_SWING_PEAK] = 0.5f * (F[Lo.swing_peak] + F[Lo.swing_peak + 1]);
  iset(Lo.rng_ctr, (int32_t)(r.ctr + 1));
  // training wrappers: EpisodeWrapper + BraxAutoResetWrapper
  float trunc = 0.0f;
  bool restore = false;
  if (c.auto_reset) {
    ep_steps += 1;
    if (ep_steps >= c.episode_length) { trunc = 1.0f - done; done = 1.0f; }
    restore = done != 0.0f;
    iset(Lo.ep_steps, ep_steps);
  }
  if (restore) {
    for (int i = l0; i < NQ; i += TS) F[Lo.qpos + i] = G[Lo.first_qpos + i];
    for (int i = l0; i < NV; i += TS) { F[Lo.qvel + i] = G[Lo.first_qvel + i]; F[Lo.qacc_warmstart + i] = G[Lo.first_qacc_warmstart + i]; }
    for (int a = l0; a < NU; a += TS) F[Lo.ctrl + a] = G[Lo.first_ctrl + a];
    if constexpr (STAGE_OBS) {
      TSYNC();
      for (int k = lane; k < Lo.priv_size; k += TEAM) L[Ly::H + k] = G[Lo.first_priv + k];  // state = its prefix
    } else {
      for (int k = 0; k < Lo.obs_size; k++) A.obs[(size_t)e * Lo.obs_size + k] = G[Lo.first_obs + k];
      for (int k = 0; k < Lo.priv_size; k++) A.priv[(size_t)e * Lo.priv_size + k] = G[Lo.first_priv + k];
    }
  } else {
    strided_for<NQ, TS>(l0, [&](int i) { F[Lo.qpos + i] = L[Ly::QPOS + i]; });
    strided_for<NV, TS>(l0, [&](int i) { F[Lo.qvel + i] = L[Ly::QVEL + i]; F[Lo.qacc_warmstart + i] = L[Ly::WARM + i]; });
  }
  F[Lo.reward] = reward;
  F[Lo.done] = done;
  F[Lo.truncation] = trunc;
  A.reward[e] = reward;
  A.done[e] = done;
  STAGE_MARK(31);
  if constexpr (STAGE_OBS) {  // coalesced rows: lane k of the team stores elements k, k + 16, ...
    TSYNC();
    float* priv = A.priv + (size_t)e * Lo.priv_size;
    float* obs = A.obs + (size_t)e * Lo.obs_size;
    // the staged row is read in one batch (compile-time trip count over the largest row), then
    // stored: one LDS round trip instead of one per element group; obs is the row's prefix
    constexpr int PMAX = DUCK_OBS_SIZE(NU) + 15 + 3 * NU + 1 + 2 + 6 + 2 + 40 + 1 + 2;
    constexpr int NKP = (PMAX + TEAM - 1) / TEAM, NKO = (DUCK_OBS_SIZE(NU) + TEAM - 1) / TEAM;
    float pv[NKP];
#pragma unroll
    for (int kk = 0; kk < NKP; kk++) {
      const int k = lane + TEAM * kk;
      pv[kk] = L[Ly::H + (k < PMAX ? k : PMAX - 1)];
    }
#pragma unroll
    for (int kk = 0; kk < NKP; kk++) {
      const int k = lane + TEAM * kk;
      if (k < Lo.priv_size) priv[k] = pv[kk];
    }
#pragma unroll
    for (int kk = 0; kk < NKO; kk++) {
      const int k = lane + TEAM * kk;
      if (k < Lo.obs_size) obs[k] = pv[kk];
    }
  }
  STAGE_MARK(34);
}


template <class Md, int WG>
__global__ void __launch_bounds__(TPB) step_kernel(KArgs A) {
  STAGE_T0();
#ifdef DUCK_ANY_PROF
  const unsigned long long kstart = clock64(), kwall = wall_clock64();
#endif
  using TL = TLay<Md>;
  {
    extern __shared__ float lds_t[];
    load_model_tables<Md>(lds_t);
  }
  STAGE_MARK(14);
  int lane;
  const int t = local_env(lane);
  if (t < 0) return;
  const int e = blockIdx.x * WG + t;
  const int n = A.n;
  extern __shared__ float lds[];
  if constexpr (TL::ES_LDS) {
    // hot state <-> LDS by the whole workgroup, field-major: a wave instruction moves 4 fields
    // x 16 consecutive envs (four 64-B segments of the [field][env] rows) instead of 16 fields x
    // 4 envs; the step's 64 random draws are made by each team in parallel into the same region
    const int j = threadIdx.x % WG, ej = blockIdx.x * WG + j;
    lds_float* esj = (lds_float*)(lds + TL::ES + j * TL::ESTRIDE);
    const StepPre P = step_prefetch<Md>(A, e, lane);
    {
      // compile-time trip count: all of the thread's loads are in flight before the first store
      // waits (one memory round trip; a runtime-bounded loop costs one per unrolled group)
      constexpr int NK = (TL::HOT + TPB / WG - 1) / (TPB / WG);
      const int ejc = ej < n ? ej : 0;
      float hv[NK];
#pragma unroll
      for (int kk = 0; kk < NK; kk++) {
        const int k = (int)threadIdx.x / WG + (TPB / WG) * kk;
        hv[kk] = A.fs[(size_t)(k < TL::HOT ? k : TL::HOT - 1) * n + ejc];
      }
#pragma unroll
      for (int kk = 0; kk < NK; kk++) {
        const int k = (int)threadIdx.x / WG + (TPB / WG) * kk;
        if (ej < n && k < TL::HOT) esj[k] = hv[kk];
      }
    }
    __syncthreads();
    STAGE_MARK(32);
    if (e < n) {
      const Slice<SW> L = env_slice<Md>(lds, t);
      const Col<0> G{A.fs + e, n};  // global row: the auto-reset snapshot (first_*) stays in HBM
      const duck_layout& Lo = A.lay;
      lds_float* esp = (lds_float*)(lds + TL::ES + t * TL::ESTRIDE);
      RngTab rt;
      rt.k0 = P.k0;
      rt.k1 = P.k1;
      rt.ctr = P.ctr;
      rt.tab = esp + TL::HOT;
      rt.fill(esp + TL::HOT, lane);
      TSYNC();
      STAGE_MARK(33);
      step_env<Md, LCol, true>(A, e, lane, L, LCol{esp}, G, rt, P);
      STAGE_RESET();
    }
    __syncthreads();
    {
      constexpr int NK = (TL::HOT + TPB / WG - 1) / (TPB / WG);
      float hv[NK];
#pragma unroll
      for (int kk = 0; kk < NK; kk++) {
        const int k = (int)threadIdx.x / WG + (TPB / WG) * kk;
        hv[kk] = esj[k < TL::HOT ? k : TL::HOT - 1];
      }
#pragma unroll
      for (int kk = 0; kk < NK; kk++) {
        const int k = (int)threadIdx.x / WG + (TPB / WG) * kk;
        if (ej < n && k < TL::HOT) A.fs[(size_t)k * n + ej] = hv[kk];
      }
    }
  } else {
    if (e >= n) return;
    const Slice<SW> L = env_slice<Md>(lds, t);
    const Col<0> G{A.fs + e, n};
    const duck_layout& Lo = A.lay;
    Rng r;
    r.k0 = (uint32_t)A.is[(size_t)Lo.rng_key * n + e];
    r.k1 = (uint32_t)A.is[(size_t)(Lo.rng_key + 1) * n + e];
    r.ctr = (uint32_t)A.is[(size_t)Lo.rng_ctr * n + e];
    step_env<Md, Col<0>, true>(A, e, lane, L, G, G, r, step_prefetch<Md>(A, e, lane));
    STAGE_RESET();  // (no staged hot state to store: mark 15 counts nothing on this path)
  }
  STAGE_MARK(15);
#ifdef DUCK_ANY_PROF
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 256) {
    const int w = 4 * blockIdx.x + threadIdx.x / 64;
    g_stage_cycles[DUCK_NSTAGE + w] = clock64() - kstart;
    g_stage_cycles[DUCK_NSTAGE + 1024 + w] = kwall;
    g_stage_cycles[DUCK_NSTAGE + 2048 + w] = wall_clock64();
  }
#endif
}

// Latency mode (duck_set_step_mode / DUCK_STEP_LATENCY, or AUTO at <= 4 envs per CU): 4 envs per
// workgroup and the stages of each substep split over its waves (TPhys::lat_r0 .. lat_r3,
// duck_team.h): wave 0 runs the env code and kinematics / com_pos / rne / actuation, wave 1 crb, the
// warm start, the Newton solve, sensors and Euler, wave 2 collision and the constraint rows, wave 3
// the smooth acceleration (M's factorization and solve). Same stage code and arithmetic as step_kernel, so the
// results are the same bit for bit (test_gpu_env.py::test_latency_mode_matches_throughput_mode);
// one env-step of a small batch takes the critical path through the waves instead of the sum.
// (the body of step_kernel_lat and step_kernel_lat_x2 below)
template <class Md, int LAT>
__device__ __forceinline__ void step_lat_body(KArgs A) {
  using TL = TLay<Md, LAT>;
  using TPL = TPhys<Md, LAT>;
  constexpr int WGL = TL::NWG;
  static_assert(TL::TAB_LDS && TL::ES_LDS, "latency mode: the model blob and the hot state in LDS");
  static_assert(TPB == 4 * 64 && WGL * TEAM == 64 * (LAT == 2 ? 2 : 1),
                "latency modes: 4 waves, one set of 4 teams per wave (paired: per pair of waves)");
  extern __shared__ float lds[];
  LAT_T(40, 5);
  TPL::ev_init((int)threadIdx.x);
  load_model_tables<Md, LAT>(lds);  // (ends with a workgroup barrier: the event counters are 0 before any wait)
  LAT_T(41, 5);
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  // the paired kernel: waves 2w and 2w + 1 work env set w (envs 4w .. 4w + 3 of the workgroup)
  const int t = (LAT == 2 ? 4 * (wave >> 1) : 0) + ((int)threadIdx.x & 63) / TEAM, lane = (int)threadIdx.x % TEAM;
  const int e = blockIdx.x * WGL + t;
  const int n = A.n;
  const int j = threadIdx.x % WGL, ej = blockIdx.x * WGL + j;
  lds_float* esj = (lds_float*)(lds + TL::ES + j * TL::ESTRIDE);
  const StepPre P = step_prefetch<Md>(A, e, lane);
  constexpr int NK = (TL::HOT + TPB / WGL - 1) / (TPB / WGL);
  {
    const int ejc = ej < n ? ej : 0;
    float hv[NK];
#pragma unroll
    for (int kk = 0; kk < NK; kk++) {
      const int k = (int)threadIdx.x / WGL + (TPB / WGL) * kk;
      hv[kk] = A.fs[(size_t)(k < TL::HOT ? k : TL::HOT - 1) * n + ejc];
    }
#pragma unroll
    for (int kk = 0; kk < NK; kk++) {
      const int k = (int)threadIdx.x / WGL + (TPB / WGL) * kk;
      if (ej < n && k < TL::HOT) esj[k] = hv[kk];
    }
  }
  __syncthreads();
  LAT_T(42, 5);
  if (e < n) {
    const Slice<SW> L = env_slice<Md, LAT>(lds, t);
    const int ns = A.cfg.n_substeps;
    float* scr = A.scratch ? A.scratch + e : nullptr;
    auto env_code = [&]() {
      const Col<0> G{A.fs + e, n};
      lds_float* esp = (lds_float*)(lds + TL::ES + t * TL::ESTRIDE);
      RngTab rt;
      rt.k0 = P.k0;
      rt.k1 = P.k1;
      rt.ctr = P.ctr;
      rt.tab = esp + TL::HOT;
      rt.fill(esp + TL::HOT, lane);
      TSYNC();
      step_env<Md, LCol, true, RngTab, LAT>(A, e, lane, L, LCol{esp}, G, rt, P);
      LAT_T(45, 5);
    };
    if constexpr (LAT == 2) {
      // the paired kernel: waves 2w (A: the env code and its share of each substep) and 2w + 1 (B)
      if ((wave & 1) == 0) {
        env_code();
      } else {
        for (int s = 0; s < ns; s++) TPL::lat2_b(L.p, lane, s, true, s == ns - 1, scr, n);
      }
    } else {
      if (wave == 0) {
        env_code();
      } else if (wave == 1) {
        for (int s = 0; s < ns; s++) TPL::lat_r1(L.p, lane, s, true, s == ns - 1, scr, n);
      } else if (wave == 2) {
        for (int s = 0; s < ns; s++) TPL::lat_r2(L.p, lane, s, A.hfield);
      } else {
        for (int s = 0; s < ns; s++) TPL::lat_r3(L.p, lane, s);
      }
    }
  }
  __syncthreads();
  LAT_T(46, 5);
  // a cross-wave wait that gave up: this workgroup's results are not valid. Raise the sticky error
  // word (the next duck_* call on the handle returns DUCK_EDEVICE) and store NaN qpos, which the
  // termination check turns into done, as the reference does for NaN physics (joystick.py:483-485)
  const bool timed_out = TPL::ev_timed_out(LAT == 2 ? j / LAT_WG : 0);  // env ej's set
  if (threadIdx.x == 0 && A.err && (TPL::ev_timed_out(0) || (LAT == 2 && TPL::ev_timed_out(1))))
    __hip_atomic_fetch_or(A.err, (unsigned)DUCK_DEVERR_LAT_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  {
    float hv[NK];
#pragma unroll
    for (int kk = 0; kk < NK; kk++) {
      const int k = (int)threadIdx.x / WGL + (TPB / WGL) * kk;
      hv[kk] = esj[k < TL::HOT ? k : TL::HOT - 1];
      if (timed_out && k >= A.lay.qpos && k < A.lay.qpos + Md::NQ) hv[kk] = __builtin_nanf("");
    }
#pragma unroll
    for (int kk = 0; kk < NK; kk++) {
      const int k = (int)threadIdx.x / WGL + (TPB / WGL) * kk;
      if (ej < n && k < TL::HOT) A.fs[(size_t)k * n + ej] = hv[kk];
    }
  }
}

template <class Md, int LAT>
__global__ void __launch_bounds__(TPB) step_kernel_lat(KArgs A) {
  step_lat_body<Md, LAT>(A);
}

// Two latency workgroups per CU (DUCK_STEP_LATENCY_X2, round 6): the four-wave latency kernel capped at
// 256 VGPR + AGPR per lane (amdgpu_waves_per_eu(2, 2)), so that a CU holds two of its workgroups -- two
// waves per SIMD, each hiding the other's stalls -- where the LDS allows (2 x lds_bytes_lat <= 160 KiB).
// Measured (profiles/r06_two_waves.txt): flat, 2 VGPRs spilled, C2 at 2,048 envs 0.1692 ms per env-step
// against 0.1744 (paired) and 0.2822 (latency, two rounds); the rough scenes spill 86-114 VGPRs and lose
// to the paired kernel (C4 0.387 vs 0.335 ms, C5 0.427 vs 0.370), and at <= 1,024 envs (one workgroup
// per CU anyway) the spills cost 6 % against the uncapped kernel. So it is compiled for plane-floor
// models without backlash hinges only (lat_x2_pays) and AUTO takes it at 4-8 envs per CU there.
// Its stage code is instantiated with LAT = LAT_X2, which every LAT test treats as LAT = 1 (same work
// split, same layout): a separate TPhys instantiation, so that its out-of-line rare paths (newton_dense,
// collide_hulls_rare) are compiled within the 256-register budget too -- shared with the uncapped kernel
// they would take its budget and hold this one at one wave per SIMD.
constexpr int LAT_X2 = 5;
template <class Md>
struct LatX2 {
  static_assert(TLay<Md, LAT_X2>::LDS_FLOATS == TLay<Md, 1>::LDS_FLOATS && TLay<Md, LAT_X2>::NWG == LAT_WG,
                "LAT_X2 is the LAT = 1 layout");
  static constexpr bool PAYS = TLay<Md, 1>::FITS && 2 * (size_t)TLay<Md, 1>::LDS_FLOATS * 4 <= 160 * 1024 &&
                               Md::FLOOR_TYPE == 0 && Md::NV <= 20;
};
template <class Md>
__global__ void __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(2, 2))) step_kernel_lat_x2(KArgs A) {
  if constexpr (LatX2<Md>::PAYS) step_lat_body<Md, LAT_X2>(A);
}

template <class Md, int WG>
__global__ void __launch_bounds__(TPB) physics_kernel(KArgs A, float* qpos_g, float* qvel_g, float* warm_g,
                                                     const float* ctrl_g, int nsub, float* aux) {
  using Ly = Lay<Md>;
  {
    extern __shared__ float lds_t[];
    load_model_tables<Md>(lds_t);
  }
  int lane;
  const int t = local_env(lane);
  if (t < 0) return;
  const int e = blockIdx.x * WG + t;
  const int n = A.n;
  if (e >= n) return;
  extern __shared__ float lds[];
  const Slice<SW> L = env_slice<Md>(lds, t);
  for (int i = 0; i < Md::NQ; i++) L[Ly::QPOS + i] = qpos_g[(size_t)i * n + e];
  for (int i = 0; i < Md::NV; i++) { L[Ly::QVEL + i] = qvel_g[(size_t)i * n + e]; L[Ly::WARM + i] = warm_g[(size_t)i * n + e]; }
  for (int a = 0; a < Md::NU; a++) L[Ly::CTRL + a] = ctrl_g[(size_t)a * n + e];
  load_dyn<Md, SW>(A, e, L);
  float* ax = aux ? aux + e : nullptr;
  float* scr = A.scratch ? A.scratch + e : nullptr;
  // nsub = 0: one forward (mjx.forward), no integration
  const int ns = nsub > 0 ? nsub : 1;
  for (int s = 0; s < ns; s++) phys_step_dni<Md>(L, lane, nsub > 0, s == ns - 1, ax, n, scr, n, A.hfield);
  for (int i = 0; i < Md::NQ; i++) qpos_g[(size_t)i * n + e] = L[Ly::QPOS + i];
  for (int i = 0; i < Md::NV; i++) { qvel_g[(size_t)i * n + e] = L[Ly::QVEL + i]; warm_g[(size_t)i * n + e] = L[Ly::WARM + i]; }
}

// domain_randomize (randomize.py:39-106), absolute randomised values per env
template <class Md>
__global__ void randomize_kernel(int n, float* dr, duck_dr_layout D, uint64_t seed, int64_t env_offset) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  Rng r;
  derive_key(seed, env_offset + e, KEY_TAG_DR, r.k0, r.k1);
  r.ctr = 0;
  int slot = 0;
  auto W = [&](int k, float v) { dr[(size_t)k * n + e] = v; };
  W(D.floor_friction, r.uniform(slot++, 0.5f, 1.0f));
  float fl[Md::NU], arm[Md::NU], ip[3], ms[Md::NB], q0[Md::NU], kp[Md::NU];
  for (int a = 0; a < Md::NU; a++) fl[a] = r.uniform(slot++, 0.9f, 1.1f);
  for (int a = 0; a < Md::NU; a++) arm[a] = r.uniform(slot++, 1.0f, 1.05f);
  for (int k = 0; k < 3; k++) ip[k] = r.uniform(slot++, -0.05f, 0.05f);
  for (int b = 0; b < Md::NB; b++) ms[b] = r.uniform(slot++, 0.9f, 1.1f);
  const float dmass = r.uniform(slot++, -0.1f, 0.1f);
  for (int a = 0; a < Md::NU; a++) q0[a] = r.uniform(slot++, -0.03f, 0.03f);
  for (int a = 0; a < Md::NU; a++) kp[a] = r.uniform(slot++, 0.9f, 1.1f);
  for (int a = 0; a < Md::NU; a++) {
    W(D.frictionloss + a, fl[a] * Md::dof_frictionloss[Md::actuator_dof[a]]);
    W(D.armature + a, arm[a] * Md::dof_armature[Md::actuator_dof[a]]);
    W(D.qpos0 + a, q0[a] + Md::qpos0[Md::actuator_qadr[a]]);
    W(D.kp + a, kp[a] * Md::actuator_kp[a]);
  }
  for (int k = 0; k < 3; k++) W(D.base_ipos + k, ip[k] + Md::body_ipos[1][k]);
  for (int b = 0; b < Md::NB; b++) W(D.body_mass + b, ms[b] * Md::body_mass[b] + (b == 1 ? dmass : 0.0f));
}

// --------------------------------------------------------------------------------------
// host side
// --------------------------------------------------------------------------------------
template <class Md>
static bool matches(const duck_model_desc* m) {
  // the header bakes every model value the kernels read: a model binds to this variant only if
  // it hashes to the same float32 values (duck_model_fingerprint, codegen.model_fingerprint)
  return duck_model_fingerprint(m) == Md::FINGERPRINT;
}

template <class Md>
static size_t lds_bytes() {
  static_assert(WG == TEAM_WG, "team workgroup size");
  return (size_t)TLay<Md>::LDS_FLOATS * sizeof(float);
}
// 0 = the split does not fit this model's LDS and is not compiled (TLay::FITS)
template <class Md>
static size_t lds_bytes_lat() {
  return TLay<Md, 1>::FITS ? (size_t)TLay<Md, 1>::LDS_FLOATS * sizeof(float) : 0;
}
template <class Md>
static size_t lds_bytes_lat2() {
  return TLay<Md, 2>::FITS ? (size_t)TLay<Md, 2>::LDS_FLOATS * sizeof(float) : 0;
}
template <class Md>
static size_t lds_bytes_lat_x2() {
  return LatX2<Md>::PAYS ? (size_t)TLay<Md, 1>::LDS_FLOATS * sizeof(float) : 0;
}

template <class Md>
static int aux_size_of() {
  return aux_size<Md>();
}

static KArgs make_args(duck_sim* s, int n) {
  KArgs A;
  memset(&A, 0, sizeof(A));
  A.n = n;
  A.cfg = s->cfg;
  A.lay = s->lay;
  A.drl = s->drl;
  A.ref = s->ref;
  A.frames = s->frames_d;
  A.hfield = s->hfield_d;
  A.err = s->err_d;
  return A;
}

template <class Md>
static int launch_reset(duck_sim* s, int n, float* fs, int32_t* is, const uint8_t* mask, uint64_t seed,
                        int64_t env_offset, const float* dr, float* obs, float* priv, hipStream_t st) {
  KArgs A = make_args(s, n);
  A.fs = fs; A.is = is; A.mask = mask; A.seed = seed; A.env_offset = env_offset; A.dr = dr;
  A.obs = obs; A.priv = priv;
  const dim3 grid((A.n + WG - 1) / WG), block(TPB);
  hipLaunchKernelGGL((reset_kernel<Md, WG>), grid, block, lds_bytes<Md>(), st, A);
  HIPCHECK(hipGetLastError());
  return DUCK_OK;
}

template <class Md>
static int launch_step(duck_sim* s, int n, float* fs, int32_t* is, const float* dr, const float* action, float* obs,
                       float* priv, float* reward, float* done, float* scratch, hipStream_t st) {
  KArgs A = make_args(s, n);
  A.fs = fs; A.is = is; A.dr = dr; A.action = action; A.obs = obs; A.priv = priv;
  A.reward = reward; A.done = done; A.scratch = scratch;
  if (s->lay.first_qpos != TLay<Md>::HOT) return duck_fail(DUCK_EINVAL, "state layout does not match the kernel's hot-state size");
  // the kernel for this batch (step_kernel_choice: AUTO takes the latency kernel while the batch
  // leaves a CU per 4 envs, the paired one while it leaves a CU per 8 -- each latency workgroup takes a
  // whole CU, one wave of 512 registers per SIMD)
  static_assert(LAT_WG == LAT_WG_HOST, "latency workgroup size");
  const int k = step_kernel_choice(s, n);
  if (k == DUCK_STEP_LATENCY || k == DUCK_STEP_PAIRED || k == DUCK_STEP_LATENCY_X2) {
    const int wgl = k == DUCK_STEP_PAIRED ? 2 * LAT_WG : LAT_WG;
    const dim3 grid((A.n + wgl - 1) / wgl), block(TPB);
    if (k == DUCK_STEP_LATENCY_X2) {
      if constexpr (LatX2<Md>::PAYS)
        hipLaunchKernelGGL((step_kernel_lat_x2<Md>), grid, block, lds_bytes_lat_x2<Md>(), st, A);
      else
        return duck_fail(DUCK_EUNSUPPORTED, "the two-workgroups-per-CU latency kernel is not compiled for this model");
    } else if (k == DUCK_STEP_PAIRED) {
      if constexpr (TLay<Md, 2>::FITS)
        hipLaunchKernelGGL((step_kernel_lat<Md, 2>), grid, block, lds_bytes_lat2<Md>(), st, A);
      else
        return duck_fail(DUCK_EUNSUPPORTED, "the paired latency kernel does not fit this model in LDS");
    } else {
      if constexpr (TLay<Md, 1>::FITS)
        hipLaunchKernelGGL((step_kernel_lat<Md, 1>), grid, block, lds_bytes_lat<Md>(), st, A);
      else
        return duck_fail(DUCK_EUNSUPPORTED, "the latency kernel does not fit this model in LDS");
    }
    HIPCHECK(hipGetLastError());
    return DUCK_OK;
  }
  const dim3 grid((A.n + WG - 1) / WG), block(TPB);
  hipLaunchKernelGGL((step_kernel<Md, WG>), grid, block, lds_bytes<Md>(), st, A);
  HIPCHECK(hipGetLastError());
  return DUCK_OK;
}

template <class Md>
static int launch_randomize(duck_sim* s, int n, float* dr, uint64_t seed, int64_t env_offset, hipStream_t st) {
  const dim3 grid((n + 255) / 256), block(256);
  hipLaunchKernelGGL((randomize_kernel<Md>), grid, block, 0, st, n, dr, s->drl, seed, env_offset);
  HIPCHECK(hipGetLastError());
  return DUCK_OK;
}

template <class Md>
static int launch_physics(duck_sim* s, int n, float* qpos, float* qvel, float* warm, const float* ctrl, const float* dr,
                          int nsub, float* aux, float* scratch, hipStream_t st) {
  const dim3 grid((n + WG - 1) / WG), block(TPB);
  KArgs A = make_args(s, n);
  A.dr = dr;
  A.scratch = scratch;
  hipLaunchKernelGGL((physics_kernel<Md, WG>), grid, block, lds_bytes<Md>(), st, A, qpos, qvel, warm, ctrl, nsub, aux);
  HIPCHECK(hipGetLastError());
  return DUCK_OK;
}

static int lat_timeouts_of(unsigned* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lat_timeouts), sizeof(unsigned));
  if (e == hipSuccess && reset) {
    const unsigned z = 0;
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_lat_timeouts), &z, sizeof(unsigned));
  }
  return e == hipSuccess ? DUCK_OK : duck_fail(DUCK_EHIP, hipGetErrorString(e));
}

static int stage_cycles_of(unsigned long long* out, int reset) {
#ifdef DUCK_ANY_PROF
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stage_cycles), sizeof(unsigned long long) * (DUCK_NSTAGE + 3 * 1024));
  static unsigned long long wg[DUCK_NSTAGE * 256];
  if (e == hipSuccess) e = hipMemcpyFromSymbol(wg, HIP_SYMBOL(g_stage_wg), sizeof(wg));
  for (int k = 0; k < DUCK_NSTAGE && e == hipSuccess; k++)
    for (int b = 0; b < 256; b++) out[k] += wg[k * 256 + b];
  if (e == hipSuccess && reset) {
    static unsigned long long z[DUCK_NSTAGE * 256 > DUCK_NSTAGE + 3 * 1024 ? DUCK_NSTAGE * 256 : DUCK_NSTAGE + 3 * 1024] = {0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_stage_cycles), z, sizeof(unsigned long long) * (DUCK_NSTAGE + 3 * 1024));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_stage_wg), z, sizeof(wg));
  }
  return e == hipSuccess ? 0 : DUCK_EHIP;
#else
  (void)out;
  (void)reset;
  return DUCK_EUNSUPPORTED;
#endif
}

// one VariantOps table per compiled model (a host function, so the device pass skips it)
#define DUCK_DEFINE_VARIANT(NAME, MODEL)                                                        \
  const VariantOps* duck_variant_##NAME() {                                                     \
    static const VariantOps ops = {#NAME,               matches<MODEL>,         aux_size_of<MODEL>, \
                                   lds_bytes<MODEL>,    MODEL::FLOOR_TYPE,      launch_reset<MODEL>, \
                                   launch_step<MODEL>,  launch_randomize<MODEL>, launch_physics<MODEL>, \
                                   stage_cycles_of,     lat_timeouts_of,        lds_bytes_lat<MODEL>, \
                                   lds_bytes_lat2<MODEL>, lds_bytes_lat_x2<MODEL>};                     \
    return &ops;                                                                                \
  }
