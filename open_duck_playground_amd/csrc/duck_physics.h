// duck_physics.h — fused mjx.step for one env per lane (CDNA4, fp32).
//
// Replaces `mjx_env.step(model, data, ctrl, n_substeps)` (joystick.py:420) and
// `mjx_env.init` -> `mjx.forward` (joystick.py:258) for the Open Duck model class. Per
// substep, inside one lane and without touching HBM:
//   kinematics -> com/cinert/cdof -> RNE bias -> CRB mass matrix (tree-sparse)
//   -> actuation/passive -> smooth acceleration (sparse LDL')
//   -> collision (plane/convex 4-point manifold, convex/convex SAT) -> constraint rows
//   (dof friction, joint limits, pyramidal contacts) -> MJX Newton (1 iteration, zoom
//   line search) -> sensors (last substep) -> semi-implicit Euler.
//
// Memory plan: every per-env array lives in a per-lane LDS slice (element k of lane t at
// lds[k*WG + t]: consecutive lanes hit consecutive banks). Each stage is a separate
// non-inlined function that reads/writes the slice with compile-time offsets (the model
// structure is constexpr, generated/duck_model_*.h), so registers only hold a stage's
// temporaries: no spills, bounded code size.
//
// Contact Jacobians are never materialised: a contact row is a 6-vector a = [r x u; u]
// in the foot's com-based spatial frame, J.x = a . (sum_chain cdof_i x_i), and J'DJ is
// accumulated as one 6x6 block per foot projected onto the foot's dof chain.
#pragma once
#include "duck_math.h"

#define DNI __device__ __noinline__
// compiler-only barrier: stops the scheduler from hoisting a whole unrolled loop's LDS
// loads into registers at once (which spills); costs no instruction
#define SCHED_FENCE() asm volatile("" ::: "memory")

// LDS-qualified pointer: keeps every slice access a ds_read/ds_write (a generic float*
// passed into a non-inlined stage would compile to flat_load/flat_store through the
// vector-memory pipe)
typedef __attribute__((address_space(3))) float lds_float;

// optional per-stage cycle counters (build with -DDUCK_STAGE_PROF; read by duck_debug_stage_cycles);
// -DDUCK_WAVE_PROF records only the per-wave launch cycles (no stage marks perturbing wave 0)
#if defined(DUCK_STAGE_PROF) || defined(DUCK_WAVE_PROF)
#define DUCK_ANY_PROF 1
#endif
#ifdef DUCK_ANY_PROF
static __device__ unsigned long long g_stage_cycles[32 + 1024];
#endif
#ifdef DUCK_STAGE_PROF
// g_stage_cycles: [0, 32) stage counters; [32, 32 + 1024) cycles of each of the first 1024 waves
// of the last step_kernel launch (wave = 4 * workgroup + wave-in-workgroup), for the launch tail
#define STAGE_T0() unsigned long long _t0 = wall_clock64(), _c0 = clock64()
#define STAGE_RESET() (_c0 = clock64())
#define STAGE_MARK(k)                                                             \
  do {                                                                            \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                            \
    const unsigned long long _c1 = clock64();                                     \
    if (threadIdx.x == 0) atomicAdd(&g_stage_cycles[k], _c1 - _c0);               \
    _c0 = _c1;                                                                    \
    (void)_t0;                                                                    \
  } while (0)
#else
#define STAGE_T0() \
  do {             \
  } while (0)
#define STAGE_MARK(k) \
  do {                \
  } while (0)
#define STAGE_RESET() \
  do {                \
  } while (0)
#endif

template <int WG>
struct Slice {
  lds_float* p;
  DK lds_float& operator[](int k) const { return p[k * WG]; }
};

// Per-lane LDS layout (floats)
template <class Md>
struct Lay {
  static constexpr int NB = Md::NB, NV = Md::NV, NQ = Md::NQ, NU = Md::NU;
  static constexpr int NCON = 4 * Md::NPAIR;
  static constexpr int R_LIM = Md::NFRIC, R_CON = Md::NFRIC + Md::NLIM;
  static constexpr int NROW = R_CON + 4 * NCON;
  // state
  static constexpr int QPOS = 0, QVEL = QPOS + NQ, WARM = QVEL + NV, CTRL = WARM + NV, QACC = CTRL + NU;
  static constexpr int QSM = QACC + NV, FSM = QSM + NV, SRCH = FSM + NV, GRAD = SRCH + NV, MA = GRAD + NV;
  // per-env model values (domain randomisation)
  static constexpr int DMASS = MA + NV, DIPOS = DMASS + NB, DARM = DIPOS + 3, DFRIC = DARM + NV;
  static constexpr int DQ0 = DFRIC + NV, DKP = DQ0 + NQ;
  // bodies
  static constexpr int XPOS = DKP + NU, XQ = XPOS + 3 * NB, XMAT = XQ + 4 * NB, CIN = XMAT + 9 * NB;
  static constexpr int CVEL = CIN + 10 * NB, COM = CVEL + 6 * NB;
  static constexpr int CDOF = COM + 3, CDD1 = CDOF + 6 * NV;
  // matrices
  static constexpr int M = CDD1 + 18, H = M + Md::NM;
  // RNE accumulators live in the H + row storage (dead until smooth()/make_rows())
  static constexpr int CACC = H, CFRC = CACC + 6 * NB;
  static_assert(12 * NB <= Md::NM + 4 * NROW, "RNE scratch must fit in H + rows");
  // constraint rows, NROWS apart: the rows, or more when the hull/hull SAT scratch that reuses the
  // H + row storage (6 floats per hull edge and face) needs it (a model without dof friction rows)
  static constexpr int SAT_SCRATCH = 6 * (Md::NHE + Md::NHF);
  static constexpr int NROWS =
      (Md::NM + 4 * NROW + Md::NLIM >= SAT_SCRATCH) ? NROW : (SAT_SCRATCH - Md::NM - Md::NLIM + 3) / 4;
  static constexpr int JA = H + Md::NM, JV = JA + NROWS, RD = JV + NROWS, AREF = RD + NROWS;
  static constexpr int LSGN = AREF + NROWS;
  static constexpr int CR = LSGN + Md::NLIM, CFR = CR + 3 * NCON, CDIST = CFR + 9 * NCON;
  // Newton 6x6 foot blocks live in CIN's storage (composite inertias are dead after crb())
  static constexpr int KL = CIN, KR = KL + 21, KLR = KR + 21, FL = KLR + 36, FR = FL + 6;
  static_assert(FR + 6 <= CIN + 10 * NB, "Newton blocks must fit in CIN");
  // outputs of the last forward
  static constexpr int AF = CDIST + NCON, SENS = AF + NU, OCON = SENS + Md::NSENSORDATA, IMUR = OCON + 2,
                       FOOTZ = IMUR + 3, FLAGS = FOOTZ + 2;
  static constexpr int TOTAL = FLAGS + 2;
};

// solref/solimp -> (k, b, imp) (mjx constraint._kbi / MuJoCo mj_makeImpedance)
DK void kbi(const float* solref, const float* solimp, float pos, float dt, float& k, float& b, float& imp) {
  const float timeconst = fmaxf(solref[0], 2.0f * dt);
  const float dampratio = solref[1];
  const float dmin = fminf(fmaxf(solimp[0], 0.0001f), 0.9999f), dmax = fminf(fmaxf(solimp[1], 0.0001f), 0.9999f);
  const float width = fmaxf(1e-15f, solimp[2]), mid = fminf(fmaxf(solimp[3], 0.0001f), 0.9999f);
  const float power = fmaxf(1.0f, solimp[4]);
  k = 1.0f / (dmax * dmax * timeconst * timeconst * dampratio * dampratio);
  b = 2.0f / (dmax * timeconst);
  const float x = fabsf(pos) / width;
  float y;
  if (power == 2.0f) {
    const float ya = (1.0f / mid) * x * x;
    const float yb = 1.0f - (1.0f / (1.0f - mid)) * (1.0f - x) * (1.0f - x);
    y = x < mid ? ya : yb;
  } else {
    const float ya = (1.0f / powf(mid, power - 1.0f)) * powf(x, power);
    const float yb = 1.0f - (1.0f / powf(1.0f - mid, power - 1.0f)) * powf(1.0f - x, power);
    y = x < mid ? ya : yb;
  }
  float im = dmin + y * (dmax - dmin);
  im = fminf(fmaxf(im, dmin), dmax);
  imp = x > 1.0f ? dmax : im;
}

// argmax with a tie band (first index within tol of the max) — same rule as the oracle
template <int N>
DK int argmax_tol(const float* v, float tol) {
  float mx = v[0];
#pragma unroll
  for (int i = 1; i < N; i++) mx = fmaxf(mx, v[i]);
  int r = N - 1;
#pragma unroll
  for (int i = N - 1; i >= 0; i--) r = (v[i] >= mx - tol) ? i : r;
  return r;
}
#define MANIFOLD_TOL 2e-8f

template <int N>
DK void pick3(const float (*P)[3], int k, float* out) {
  out[0] = P[0][0]; out[1] = P[0][1]; out[2] = P[0][2];
#pragma unroll
  for (int i = 1; i < N; i++) {
    const bool s = (i == k);
    out[0] = s ? P[i][0] : out[0];
    out[1] = s ? P[i][1] : out[1];
    out[2] = s ? P[i][2] : out[2];
  }
}
template <int N>
DK float pick1(const float* P, int k) {
  float o = P[0];
#pragma unroll
  for (int i = 1; i < N; i++) o = (i == k) ? P[i] : o;
  return o;
}

// mjx collision_convex._manifold_points: 4 polygon points of ~maximal area
template <int N>
DK void manifold_points(const float (*poly)[3], const bool* mask, const float* nrm, int idx[4]) {
  float dm[N], s[N], s2[2 * N];
#pragma unroll
  for (int k = 0; k < N; k++) dm[k] = mask[k] ? 0.0f : -1e6f;
  const int a = argmax_tol<N>(dm, 0.0f);
  float pa[3];
  pick3<N>(poly, a, pa);
#pragma unroll
  for (int k = 0; k < N; k++) {
    const float dx = pa[0] - poly[k][0], dy = pa[1] - poly[k][1], dz = pa[2] - poly[k][2];
    s[k] = dx * dx + dy * dy + dz * dz + dm[k];
  }
  const int b = argmax_tol<N>(s, MANIFOLD_TOL);
  float pb[3];
  pick3<N>(poly, b, pb);
  float amb[3] = {pa[0] - pb[0], pa[1] - pb[1], pa[2] - pb[2]}, ab[3];
  cross3(ab, nrm, amb);
#pragma unroll
  for (int k = 0; k < N; k++) {
    const float ap[3] = {pa[0] - poly[k][0], pa[1] - poly[k][1], pa[2] - poly[k][2]};
    s[k] = fabsf(dot3(ap, ab)) + dm[k];
  }
  const int c = argmax_tol<N>(s, MANIFOLD_TOL);
  float pc[3];
  pick3<N>(poly, c, pc);
  float amc[3] = {pa[0] - pc[0], pa[1] - pc[1], pa[2] - pc[2]};
  float bmc[3] = {pb[0] - pc[0], pb[1] - pc[1], pb[2] - pc[2]};
  float ac[3], bc[3];
  cross3(ac, nrm, amc);
  cross3(bc, nrm, bmc);
#pragma unroll
  for (int k = 0; k < N; k++) {
    const float bp[3] = {pb[0] - poly[k][0], pb[1] - poly[k][1], pb[2] - poly[k][2]};
    const float ap[3] = {pa[0] - poly[k][0], pa[1] - poly[k][1], pa[2] - poly[k][2]};
    s2[k] = fabsf(dot3(bp, bc)) + dm[k];
    s2[N + k] = fabsf(dot3(ap, ac)) + dm[k];
  }
  int d = argmax_tol<2 * N>(s2, MANIFOLD_TOL);
  d = d >= N ? d - N : d;
  idx[0] = a; idx[1] = b; idx[2] = c; idx[3] = d;
}

// mjx math.make_frame: rows (n, t1, t2)
DK void make_frame(float* fr, const float* nin) {
  float n[3] = {nin[0], nin[1], nin[2]};
  const float nn = sqrtf(dot3(n, n));
  if (nn > 1e-15f) { n[0] /= nn; n[1] /= nn; n[2] /= nn; }
  float b[3];
  const bool y = (-0.5f < n[1]) && (n[1] < 0.5f);
  b[0] = 0.0f; b[1] = y ? 1.0f : 0.0f; b[2] = y ? 0.0f : 1.0f;
  const float nb = dot3(n, b);
  b[0] -= n[0] * nb; b[1] -= n[1] * nb; b[2] -= n[2] * nb;
  const float bn = sqrtf(dot3(b, b));
  if (bn > 1e-15f) { b[0] /= bn; b[1] /= bn; b[2] /= bn; }
  float c[3];
  cross3(c, n, b);
  fr[0] = n[0]; fr[1] = n[1]; fr[2] = n[2];
  fr[3] = b[0]; fr[4] = b[1]; fr[5] = b[2];
  fr[6] = c[0]; fr[7] = c[1]; fr[8] = c[2];
}

template <class Md>
DK constexpr int cgeom_slot(int g) {
  return g == Md::FLOOR_GEOM ? 0 : (g == Md::LFOOT_GEOM ? 1 : 2);
}

template <class Md, int WG>
struct Phys {
  using Ly = Lay<Md>;
  using S = Slice<WG>;
  static constexpr int NV = Md::NV, NB = Md::NB, NQ = Md::NQ, NU = Md::NU;
  static constexpr int NCON = Ly::NCON, NFRIC = Md::NFRIC, NLIM = Md::NLIM, NROW = Ly::NROW;

  // ---------------- per-env model values ----------------
  static DK void set_nominal(S L) {
#pragma unroll
    for (int b = 0; b < NB; b++) L[Ly::DMASS + b] = Md::body_mass[b];
#pragma unroll
    for (int k = 0; k < 3; k++) L[Ly::DIPOS + k] = Md::body_ipos[1][k];
#pragma unroll
    for (int i = 0; i < NV; i++) { L[Ly::DARM + i] = Md::dof_armature[i]; L[Ly::DFRIC + i] = Md::dof_frictionloss[i]; }
#pragma unroll
    for (int i = 0; i < NQ; i++) L[Ly::DQ0 + i] = Md::qpos0[i];
#pragma unroll
    for (int a = 0; a < NU; a++) L[Ly::DKP + a] = Md::actuator_kp[a];
  }

  // ---------------- mj_kinematics ----------------
  static DNI void kinematics(S L) {
#pragma unroll
    for (int b = 1; b < NB; b++) {
      float p[3], q[4];
      if (b == 1) {
        p[0] = L[Ly::QPOS + 0]; p[1] = L[Ly::QPOS + 1]; p[2] = L[Ly::QPOS + 2];
        q[0] = L[Ly::QPOS + 3]; q[1] = L[Ly::QPOS + 4]; q[2] = L[Ly::QPOS + 5]; q[3] = L[Ly::QPOS + 6];
      } else {
        const int pa = Md::body_parentid[b];
        if (pa == 0) {
#pragma unroll
          for (int k = 0; k < 3; k++) p[k] = Md::body_pos[b][k];
#pragma unroll
          for (int k = 0; k < 4; k++) q[k] = Md::body_quat[b][k];
        } else {
          float R[9], pq[4], t[3];
#pragma unroll
          for (int k = 0; k < 9; k++) R[k] = L[Ly::XMAT + 9 * pa + k];
#pragma unroll
          for (int k = 0; k < 4; k++) pq[k] = L[Ly::XQ + 4 * pa + k];
          mulmv3(t, R, Md::body_pos[b]);
#pragma unroll
          for (int k = 0; k < 3; k++) p[k] = L[Ly::XPOS + 3 * pa + k] + t[k];
          qmul(q, pq, Md::body_quat[b]);
        }
#pragma unroll
        for (int jj = 0; jj < 2; jj++) {
          if (jj < Md::body_jntnum[b]) {
            const int j = Md::body_jntadr[b] + jj;
            const int a = Md::jnt_qposadr[j];
            float s, c;
            sincosf(0.5f * (L[Ly::QPOS + a] - L[Ly::DQ0 + a]), &s, &c);
            const float ql[4] = {c, Md::jnt_axis[j][0] * s, Md::jnt_axis[j][1] * s, Md::jnt_axis[j][2] * s};
            qmul(q, q, ql);
          }
        }
      }
      qnormalize(q);
      float R[9];
      q2m(R, q);
#pragma unroll
      for (int k = 0; k < 3; k++) L[Ly::XPOS + 3 * b + k] = p[k];
#pragma unroll
      for (int k = 0; k < 4; k++) L[Ly::XQ + 4 * b + k] = q[k];
#pragma unroll
      for (int k = 0; k < 9; k++) L[Ly::XMAT + 9 * b + k] = R[k];
    }
  }

  // ---------------- mj_comPos: subtree com, cinert, cdof ----------------
  static DNI void com_pos(S L) {
    float com[3] = {0.0f, 0.0f, 0.0f}, msum = 0.0f;
#pragma unroll
    for (int b = 1; b < NB; b++) {
      if (Md::body_weldid[b] == 0) continue;
      SCHED_FENCE();
      float R[9], t[3], ip[3];
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = L[Ly::XMAT + 9 * b + k];
#pragma unroll
      for (int k = 0; k < 3; k++) ip[k] = (b == 1) ? L[Ly::DIPOS + k] : Md::body_ipos[b][k];
      mulmv3(t, R, ip);
      const float m = L[Ly::DMASS + b];
      msum += m;
#pragma unroll
      for (int k = 0; k < 3; k++) com[k] += m * (L[Ly::XPOS + 3 * b + k] + t[k]);
    }
    const float inv = 1.0f / msum;
#pragma unroll
    for (int k = 0; k < 3; k++) { com[k] *= inv; L[Ly::COM + k] = com[k]; }
#pragma unroll
    for (int b = 1; b < NB; b++) {
      if (Md::body_weldid[b] == 0) continue;
      SCHED_FENCE();
      float R[9], t[3], ip[3], Ri[9];
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = L[Ly::XMAT + 9 * b + k];
#pragma unroll
      for (int k = 0; k < 3; k++) ip[k] = (b == 1) ? L[Ly::DIPOS + k] : Md::body_ipos[b][k];
      mulmv3(t, R, ip);
      mulmm3(Ri, R, Md::body_imat[b]);
      const float* I = Md::body_inertia[b];
      float rot[9];
#pragma unroll
      for (int a = 0; a < 3; a++)
#pragma unroll
        for (int c = 0; c < 3; c++)
          rot[3 * a + c] = Ri[3 * a] * I[0] * Ri[3 * c] + Ri[3 * a + 1] * I[1] * Ri[3 * c + 1] + Ri[3 * a + 2] * I[2] * Ri[3 * c + 2];
      const float d[3] = {L[Ly::XPOS + 3 * b] + t[0] - com[0], L[Ly::XPOS + 3 * b + 1] + t[1] - com[1],
                          L[Ly::XPOS + 3 * b + 2] + t[2] - com[2]};
      const float m = L[Ly::DMASS + b], dd = dot3(d, d);
      const int o = Ly::CIN + 10 * b;
      L[o + 0] = rot[0] + m * (dd - d[0] * d[0]);
      L[o + 1] = rot[4] + m * (dd - d[1] * d[1]);
      L[o + 2] = rot[8] + m * (dd - d[2] * d[2]);
      L[o + 3] = rot[1] - m * d[0] * d[1];
      L[o + 4] = rot[2] - m * d[0] * d[2];
      L[o + 5] = rot[5] - m * d[1] * d[2];
      L[o + 6] = m * d[0]; L[o + 7] = m * d[1]; L[o + 8] = m * d[2];
      L[o + 9] = m;
    }
#pragma unroll
    for (int j = 0; j < Md::NJ; j++) {
      SCHED_FENCE();
      const int b = Md::jnt_bodyid[j], da = Md::jnt_dofadr[j];
      const float off[3] = {com[0] - L[Ly::XPOS + 3 * b], com[1] - L[Ly::XPOS + 3 * b + 1], com[2] - L[Ly::XPOS + 3 * b + 2]};
      if (Md::jnt_type[j] == 0) {
#pragma unroll
        for (int k = 0; k < 3; k++)
#pragma unroll
          for (int q = 0; q < 6; q++) L[Ly::CDOF + 6 * (da + k) + q] = (q == 3 + k) ? 1.0f : 0.0f;
#pragma unroll
        for (int k = 0; k < 3; k++) {
          const float ax[3] = {L[Ly::XMAT + 9 * b + k], L[Ly::XMAT + 9 * b + 3 + k], L[Ly::XMAT + 9 * b + 6 + k]};
          float t[3];
          cross3(t, ax, off);
          const int o = Ly::CDOF + 6 * (da + 3 + k);
          L[o] = ax[0]; L[o + 1] = ax[1]; L[o + 2] = ax[2]; L[o + 3] = t[0]; L[o + 4] = t[1]; L[o + 5] = t[2];
        }
      } else {
        float R[9], ax[3], t[3];
#pragma unroll
        for (int k = 0; k < 9; k++) R[k] = L[Ly::XMAT + 9 * b + k];
        mulmv3(ax, R, Md::jnt_axis[j]);
        cross3(t, ax, off);
        const int o = Ly::CDOF + 6 * da;
        L[o] = ax[0]; L[o + 1] = ax[1]; L[o + 2] = ax[2]; L[o + 3] = t[0]; L[o + 4] = t[1]; L[o + 5] = t[2];
      }
    }
  }

  // ---------------- mj_comVel + mj_rne (flg_acc = 0): cvel, FSM = -bias ----------------
  static DNI void rne(S L) {
#pragma unroll
    for (int b = 1; b < NB; b++) {
      if (Md::body_weldid[b] == 0) continue;
      SCHED_FENCE();
      const int pa = Md::body_parentid[b];
      float cv[6], ca[6];
#pragma unroll
      for (int k = 0; k < 6; k++) {
        cv[k] = (pa == 0) ? 0.0f : L[Ly::CVEL + 6 * pa + k];
        ca[k] = (pa == 0) ? ((k >= 3) ? -Md::gravity[k - 3] : 0.0f) : L[Ly::CACC + 6 * pa + k];
      }
      const int da = Md::body_dofadr[b];
      if (b == 1) {
#pragma unroll
        for (int i = 0; i < 3; i++) {
          const float v = L[Ly::QVEL + i];
#pragma unroll
          for (int k = 0; k < 6; k++) cv[k] += L[Ly::CDOF + 6 * i + k] * v;
        }
        float cvt[6];
#pragma unroll
        for (int k = 0; k < 6; k++) cvt[k] = cv[k];
#pragma unroll
        for (int i = 3; i < 6; i++) {
          float cd[6], cdd[6];
#pragma unroll
          for (int k = 0; k < 6; k++) cd[k] = L[Ly::CDOF + 6 * i + k];
          cross_motion(cdd, cvt, cd);
          const float v = L[Ly::QVEL + i];
#pragma unroll
          for (int k = 0; k < 6; k++) { L[Ly::CDD1 + 6 * (i - 3) + k] = cdd[k]; ca[k] += cdd[k] * v; cv[k] += cd[k] * v; }
        }
      } else {
#pragma unroll
        for (int jj = 0; jj < 2; jj++) {
          if (jj < Md::body_dofnum[b]) {
            const int i = da + jj;
            float cd[6], cdd[6];
#pragma unroll
            for (int k = 0; k < 6; k++) cd[k] = L[Ly::CDOF + 6 * i + k];
            cross_motion(cdd, cv, cd);
            const float v = L[Ly::QVEL + i];
#pragma unroll
            for (int k = 0; k < 6; k++) { ca[k] += cdd[k] * v; cv[k] += cd[k] * v; }
          }
        }
      }
      float I[10], f[6], t1[6], t2[6];
#pragma unroll
      for (int k = 0; k < 10; k++) I[k] = L[Ly::CIN + 10 * b + k];
      mul_inert_vec(f, I, ca);
      mul_inert_vec(t1, I, cv);
      cross_force(t2, cv, t1);
#pragma unroll
      for (int k = 0; k < 6; k++) {
        L[Ly::CFRC + 6 * b + k] = f[k] + t2[k];
        L[Ly::CVEL + 6 * b + k] = cv[k];
        L[Ly::CACC + 6 * b + k] = ca[k];
      }
    }
#pragma unroll
    for (int b = NB - 1; b > 1; b--) {
      if (Md::body_weldid[b] == 0) continue;
      const int pa = Md::body_parentid[b];
#pragma unroll
      for (int k = 0; k < 6; k++) L[Ly::CFRC + 6 * pa + k] += L[Ly::CFRC + 6 * b + k];
    }
#pragma unroll
    for (int i = 0; i < NV; i++) {
      SCHED_FENCE();
      const int b = Md::dof_bodyid[i];
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < 6; k++) s += L[Ly::CDOF + 6 * i + k] * L[Ly::CFRC + 6 * b + k];
      L[Ly::FSM + i] = -s;  // -qfrc_bias, completed by smooth()
    }
  }

  // ---------------- mj_crb: composite inertia (in place) and sparse M ----------------
  static DNI void crb(S L) {
#pragma unroll
    for (int b = NB - 1; b > 1; b--) {
      if (Md::body_weldid[b] == 0) continue;
      const int pa = Md::body_parentid[b];
#pragma unroll
      for (int k = 0; k < 10; k++) L[Ly::CIN + 10 * pa + k] += L[Ly::CIN + 10 * b + k];
    }
#pragma unroll
    for (int i = 0; i < NV; i++) {
      SCHED_FENCE();
      float cd[6], buf[6], I[10];
#pragma unroll
      for (int k = 0; k < 6; k++) cd[k] = L[Ly::CDOF + 6 * i + k];
#pragma unroll
      for (int k = 0; k < 10; k++) I[k] = L[Ly::CIN + 10 * Md::dof_bodyid[i] + k];
      mul_inert_vec(buf, I, cd);
#pragma unroll
      for (int j = 0; j <= i; j++) {
        if (Md::M_adr[i][j] >= 0) {
          SCHED_FENCE();
          float s = 0.0f;
#pragma unroll
          for (int k = 0; k < 6; k++) s += L[Ly::CDOF + 6 * j + k] * buf[k];
          if (j == i) s += L[Ly::DARM + i];
          L[Ly::M + Md::M_adr[i][j]] = s;
        }
      }
    }
  }

  // ---------------- actuation + passive + smooth acceleration ----------------
  static DNI void smooth(S L) {
#pragma unroll
    for (int i = 0; i < NV; i++) L[Ly::FSM + i] += -Md::dof_damping[i] * L[Ly::QVEL + i];
#pragma unroll
    for (int a = 0; a < NU; a++) {
      float c = L[Ly::CTRL + a];
      if (Md::actuator_ctrllimited[a]) c = fminf(fmaxf(c, Md::actuator_ctrlrange[a][0]), Md::actuator_ctrlrange[a][1]);
      const float g = Md::actuator_gear[a], kp = L[Ly::DKP + a];
      const float len = g * L[Ly::QPOS + Md::actuator_qadr[a]], vel = g * L[Ly::QVEL + Md::actuator_dof[a]];
      float f = kp * c + (-kp * len - Md::actuator_kv[a] * vel);
      if (Md::actuator_forcelimited[a]) f = fminf(fmaxf(f, Md::actuator_forcerange[a][0]), Md::actuator_forcerange[a][1]);
      L[Ly::AF + a] = f;
      L[Ly::FSM + Md::actuator_dof[a]] += g * f;
    }
#pragma unroll
    for (int k = 0; k < Md::NM; k++) L[Ly::H + k] = L[Ly::M + k];
  }

  // ---------------- collision (mjx collision_driver, 4 slots per pair) ----------------
  static DK void geom_frame(S L, int g, float* gp, float* gR) {
    const int b = Md::cgeom_body[g];
    if (Md::body_weldid[b] == 0) {
      float bq[4] = {Md::body_quat[b][0], Md::body_quat[b][1], Md::body_quat[b][2], Md::body_quat[b][3]}, BR[9], t[3];
      q2m(BR, bq);
      mulmv3(t, BR, Md::geom_pos[g]);
#pragma unroll
      for (int k = 0; k < 3; k++) gp[k] = Md::body_pos[b][k] + t[k];
      mulmm3(gR, BR, Md::geom_mat[g]);
    } else {
      float R[9], t[3];
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = L[Ly::XMAT + 9 * b + k];
      mulmv3(t, R, Md::geom_pos[g]);
#pragma unroll
      for (int k = 0; k < 3; k++) gp[k] = L[Ly::XPOS + 3 * b + k] + t[k];
      mulmm3(gR, R, Md::geom_mat[g]);
    }
  }

  static DK void store_contact(S L, int slot, float dist, const float* pos, const float* fr) {
    L[Ly::CDIST + slot] = dist;
#pragma unroll
    for (int a = 0; a < 3; a++) L[Ly::CR + 3 * slot + a] = pos[a] - L[Ly::COM + a];
#pragma unroll
    for (int a = 0; a < 9; a++) L[Ly::CFR + 9 * slot + a] = fr[a];
  }

  // plane (floor) vs convex hull: mjx collision_convex.plane_convex
  static DNI void collide_plane_hull(S L, int gs, int slot0) {
    float pp[3], PR[9], cp[3], CR[9];
    geom_frame(L, 0, pp, PR);
    geom_frame(L, gs, cp, CR);
    const float n[3] = {PR[2], PR[5], PR[8]};
    const float dif[3] = {pp[0] - cp[0], pp[1] - cp[1], pp[2] - cp[2]};
    float pl[3], nl[3];
    mulmtv3(pl, CR, dif);
    mulmtv3(nl, CR, n);
    constexpr int NH = Md::NHV;
    float support[NH];
    bool mask[NH];
    float smax = -1e30f;
#pragma unroll
    for (int k = 0; k < NH; k++) {
      const float t[3] = {pl[0] - Md::hull_vert[k][0], pl[1] - Md::hull_vert[k][1], pl[2] - Md::hull_vert[k][2]};
      support[k] = dot3(t, nl);
      smax = fmaxf(smax, support[k]);
    }
    const float thr = fmaxf(smax - 1e-3f, 0.0f);
#pragma unroll
    for (int k = 0; k < NH; k++) mask[k] = support[k] > thr;
    int idx[4];
    manifold_points<NH>(Md::hull_vert, mask, nl, idx);
    float fr[9];
    make_frame(fr, n);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      bool unique = true;
#pragma unroll
      for (int e = 0; e < c; e++) unique = unique && (idx[e] != idx[c]);
      const float dist = unique ? -pick1<NH>(support, idx[c]) : 1.0f;
      float v[3], vw[3], pos[3];
      pick3<NH>(Md::hull_vert, idx[c], v);
      mulmv3(vw, CR, v);
#pragma unroll
      for (int a = 0; a < 3; a++) pos[a] = cp[a] + vw[a] - 0.5f * dist * n[a];
      store_contact(L, slot0 + c, dist, pos, fr);
    }
  }

  // convex vs convex (foot/foot): SAT over face normals and edge pairs, then a 4-point
  // manifold against the reference face or one edge-edge point (oracle collide_convex_convex).
  // Single-lane debug build (-DDUCK_TEAM=0) only: it tests every edge pair and keeps the exact
  // maximum, without the Minkowski-face filter and tie tolerance of TPhys::collide_hulls_team and
  // the oracle, so near-tied axes may resolve differently there.
  static DNI void collide_hulls(S L, int s1, int s2, int slot0) {
    constexpr int NH = Md::NHV;
    const float nofr[9] = {0, 0, 1, 0, 1, 0, -1, 0, 0};
    float zero[3];
#pragma unroll
    for (int a = 0; a < 3; a++) zero[a] = L[Ly::COM + a];
#pragma unroll
    for (int c = 0; c < 4; c++) store_contact(L, slot0 + c, 1.0f, zero, nofr);
    float p1[3], R1[9], p2[3], R2[9];
    geom_frame(L, s1, p1, R1);
    geom_frame(L, s2, p2, R2);
    float c1[3], c2[3], t[3];
    mulmv3(t, R1, Md::hull_center);
#pragma unroll
    for (int a = 0; a < 3; a++) c1[a] = p1[a] + t[a];
    mulmv3(t, R2, Md::hull_center);
#pragma unroll
    for (int a = 0; a < 3; a++) c2[a] = p2[a] + t[a];
    const float cc[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
    if (dot3(cc, cc) > 4.0f * Md::hull_radius * Md::hull_radius) return;
    float V1[NH][3], V2[NH][3];
#pragma unroll
    for (int k = 0; k < NH; k++) {
      mulmv3(t, R1, Md::hull_vert[k]);
      V1[k][0] = p1[0] + t[0]; V1[k][1] = p1[1] + t[1]; V1[k][2] = p1[2] + t[2];
      mulmv3(t, R2, Md::hull_vert[k]);
      V2[k][0] = p2[0] + t[0]; V2[k][1] = p2[1] + t[1]; V2[k][2] = p2[2] + t[2];
    }
    const float(*HV)[3] = Md::hull_vert_d();
    const float(*HN)[3] = Md::hull_face_normal_d();
    const int(*HE)[2] = Md::hull_edge_d();
    float best = -1e30f, bu[3] = {0.0f, 0.0f, 1.0f};
    int btype = -1, bi = 0, bj = 0;
    for (int side = 0; side < 2; side++) {
      for (int f = 0; f < Md::NHF; f++) {
        float u[3];
        mulmv3(u, side == 0 ? R1 : R2, HN[f]);
        if (side == 1) { u[0] = -u[0]; u[1] = -u[1]; u[2] = -u[2]; }
        float mx1 = -1e30f, mn2 = 1e30f;
#pragma unroll
        for (int k = 0; k < NH; k++) {
          mx1 = fmaxf(mx1, dot3(u, V1[k]));
          mn2 = fminf(mn2, dot3(u, V2[k]));
        }
        const float sep = mn2 - mx1;
        if (sep > 0.0f) return;
        if (sep > best) { best = sep; bu[0] = u[0]; bu[1] = u[1]; bu[2] = u[2]; btype = side; bi = f; }
      }
    }
    for (int e1 = 0; e1 < Md::NHE; e1++) {
      const int a0 = HE[e1][0], a1 = HE[e1][1];
      float tmp[3] = {HV[a1][0] - HV[a0][0], HV[a1][1] - HV[a0][1], HV[a1][2] - HV[a0][2]};
      float ea[3];
      mulmv3(ea, R1, tmp);
      const float na = sqrtf(dot3(ea, ea));
      for (int e2 = 0; e2 < Md::NHE; e2++) {
        const int b0 = HE[e2][0], b1 = HE[e2][1];
        float tmp2[3] = {HV[b1][0] - HV[b0][0], HV[b1][1] - HV[b0][1], HV[b1][2] - HV[b0][2]};
        float eb[3], u[3];
        mulmv3(eb, R2, tmp2);
        cross3(u, ea, eb);
        const float un = sqrtf(dot3(u, u));
        if (un < 1e-6f * na * sqrtf(dot3(eb, eb))) continue;
        u[0] /= un; u[1] /= un; u[2] /= un;
        if (dot3(u, cc) < 0.0f) { u[0] = -u[0]; u[1] = -u[1]; u[2] = -u[2]; }
        float mx1 = -1e30f, mn2 = 1e30f;
#pragma unroll
        for (int k = 0; k < NH; k++) {
          mx1 = fmaxf(mx1, dot3(u, V1[k]));
          mn2 = fminf(mn2, dot3(u, V2[k]));
        }
        const float sep = mn2 - mx1;
        if (sep > 0.0f) return;
        if (sep > best + 1e-9f) { best = sep; bu[0] = u[0]; bu[1] = u[1]; bu[2] = u[2]; btype = 2; bi = e1; bj = e2; }
      }
    }
    float fr[9];
    make_frame(fr, bu);
    if (btype == 2) {
      float a0[3], a1[3], b0[3], b1[3];
      pick3<NH>(V1, HE[bi][0], a0);
      pick3<NH>(V1, HE[bi][1], a1);
      pick3<NH>(V2, HE[bj][0], b0);
      pick3<NH>(V2, HE[bj][1], b1);
      float d1[3], d2[3], r[3];
      for (int a = 0; a < 3; a++) { d1[a] = a1[a] - a0[a]; d2[a] = b1[a] - b0[a]; r[a] = a0[a] - b0[a]; }
      const float A = dot3(d1, d1), E = dot3(d2, d2), F = dot3(d2, r), C = dot3(d1, r), B = dot3(d1, d2);
      const float den = A * E - B * B;
      float s = den > 1e-15f ? (B * F - C * E) / den : 0.0f;
      s = fminf(fmaxf(s, 0.0f), 1.0f);
      float tt = E > 1e-15f ? (B * s + F) / E : 0.0f;
      if (tt < 0.0f) { tt = 0.0f; s = A > 1e-15f ? -C / A : 0.0f; }
      else if (tt > 1.0f) { tt = 1.0f; s = A > 1e-15f ? (B - C) / A : 0.0f; }
      s = fminf(fmaxf(s, 0.0f), 1.0f);
      float pos[3];
      for (int a = 0; a < 3; a++) pos[a] = 0.5f * (a0[a] + s * d1[a] + b0[a] + tt * d2[a]);
      store_contact(L, slot0, best, pos, fr);
      return;
    }
    const float* Rr = btype == 0 ? R1 : R2;
    const float* pr = btype == 0 ? p1 : p2;
    float fn[3];
    mulmv3(fn, Rr, HN[bi]);
    const float off = Md::hull_face_offset_d()[bi] + dot3(fn, pr);
    float support[NH];
    bool mask[NH];
    float smax = -1e30f;
#pragma unroll
    for (int k = 0; k < NH; k++) {
      const float* v = btype == 0 ? V2[k] : V1[k];
      support[k] = off - dot3(fn, v);
      smax = fmaxf(smax, support[k]);
    }
    const float thr = fmaxf(smax - 1e-3f, 0.0f);
#pragma unroll
    for (int k = 0; k < NH; k++) mask[k] = support[k] > thr;
    int idx[4];
    if (btype == 0) manifold_points<NH>(V2, mask, fn, idx);
    else manifold_points<NH>(V1, mask, fn, idx);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      bool unique = true;
#pragma unroll
      for (int e = 0; e < c; e++) unique = unique && (idx[e] != idx[c]);
      const float dist = unique ? -pick1<NH>(support, idx[c]) : 1.0f;
      float v[3], pos[3];
      if (btype == 0) pick3<NH>(V2, idx[c], v);
      else pick3<NH>(V1, idx[c], v);
      for (int a = 0; a < 3; a++) pos[a] = v[a] - 0.5f * dist * fn[a];
      store_contact(L, slot0 + c, dist, pos, fr);
    }
  }

  static DK void collision(S L) {
#pragma unroll
    for (int p = 0; p < Md::NPAIR; p++) {
      const int s1 = cgeom_slot<Md>(Md::pair_geom1[p]), s2 = cgeom_slot<Md>(Md::pair_geom2[p]);
      if (s1 == 0 && Md::FLOOR_TYPE == 0) collide_plane_hull(L, s2, 4 * p);
      else if (s1 != 0 && s2 != 0) collide_hulls(L, s1, s2, 4 * p);
    }
  }

  // ---------------- constraint rows (mjx make_constraint) ----------------
  static DK void contact_vel(const float* Sp, const float* r, float* v) {
    float t[3];
    cross3(t, Sp, r);
    v[0] = Sp[3] + t[0]; v[1] = Sp[4] + t[1]; v[2] = Sp[5] + t[2];
  }

  // J.x of contact slot for body spatial motions SL/SR -> 4 pyramid edges
  static DK void contact_jx(S L, int p, int slot, const float* SL, const float* SR, float* out4) {
    const int s1 = cgeom_slot<Md>(Md::pair_geom1[p]), s2 = cgeom_slot<Md>(Md::pair_geom2[p]);
    const float mu = Md::pair_friction[p][0];
    const float r[3] = {L[Ly::CR + 3 * slot], L[Ly::CR + 3 * slot + 1], L[Ly::CR + 3 * slot + 2]};
    float v[3] = {0.0f, 0.0f, 0.0f}, t[3];
    if (s2 != 0) { contact_vel(s2 == 1 ? SL : SR, r, t); v[0] += t[0]; v[1] += t[1]; v[2] += t[2]; }
    if (s1 != 0) { contact_vel(s1 == 1 ? SL : SR, r, t); v[0] -= t[0]; v[1] -= t[1]; v[2] -= t[2]; }
    float jr[3];
#pragma unroll
    for (int q = 0; q < 3; q++)
      jr[q] = L[Ly::CFR + 9 * slot + 3 * q] * v[0] + L[Ly::CFR + 9 * slot + 3 * q + 1] * v[1] +
              L[Ly::CFR + 9 * slot + 3 * q + 2] * v[2];
    out4[0] = jr[0] + mu * jr[1];
    out4[1] = jr[0] - mu * jr[1];
    out4[2] = jr[0] + mu * jr[2];
    out4[3] = jr[0] - mu * jr[2];
  }

  static DNI void make_rows(S L) {
    const float dt = Md::timestep;
#pragma unroll
    for (int r = 0; r < NFRIC; r++) {
      const int i = Md::fric_dof[r];
      float k, b, imp;
      kbi(Md::dof_solref[i], Md::dof_solimp[i], 0.0f, dt, k, b, imp);
      const float R = fmaxf(Md::dof_invweight0[i] * (1.0f - imp) / imp, 1e-15f);
      L[Ly::RD + r] = 1.0f / R;
      L[Ly::AREF + r] = -b * L[Ly::QVEL + i];
    }
#pragma unroll
    for (int r = 0; r < NLIM; r++) {
      const int j = Md::lim_jnt[r], i = Md::jnt_dofadr[j];
      const float q = L[Ly::QPOS + Md::jnt_qposadr[j]];
      const float dlo = q - Md::jnt_range[j][0], dhi = Md::jnt_range[j][1] - q;
      const float pos = fminf(dlo, dhi) - Md::jnt_margin[j];
      const float sgn = dlo < dhi ? 1.0f : -1.0f;
      float k, b, imp;
      kbi(Md::jnt_solref[j], Md::jnt_solimp[j], pos, dt, k, b, imp);
      const float R = fmaxf(Md::dof_invweight0[i] * (1.0f - imp) / imp, 1e-15f);
      const bool active = pos < 0.0f;
      L[Ly::RD + Ly::R_LIM + r] = active ? 1.0f / R : 0.0f;
      L[Ly::AREF + Ly::R_LIM + r] = active ? (-b * sgn * L[Ly::QVEL + i] - k * imp * pos) : 0.0f;
      L[Ly::LSGN + r] = sgn;
    }
    float SL[6], SR[6];
#pragma unroll
    for (int k = 0; k < 6; k++) { SL[k] = L[Ly::CVEL + 6 * Md::LFOOT_BODY + k]; SR[k] = L[Ly::CVEL + 6 * Md::RFOOT_BODY + k]; }
#pragma unroll
    for (int p = 0; p < Md::NPAIR; p++) {
      const int s1 = cgeom_slot<Md>(Md::pair_geom1[p]), s2 = cgeom_slot<Md>(Md::pair_geom2[p]);
      const int b1 = Md::cgeom_body[s1], b2 = Md::cgeom_body[s2];
      const float tran = Md::body_invweight0[b1][0] + Md::body_invweight0[b2][0];
      const float mu = Md::pair_friction[p][0];
      const float iw = (tran + mu * mu * tran) * 2.0f * mu * mu / Md::impratio;
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int slot = 4 * p + c;
        const float pos = L[Ly::CDIST + slot] - Md::pair_margin[p];
        const bool active = pos < 0.0f;
        float k, b, imp;
        kbi(Md::pair_solref[p], Md::pair_solimp[p], pos, dt, k, b, imp);
        const float R = fmaxf(iw * (1.0f - imp) / imp, 1e-15f);
        float vel[4];
        contact_jx(L, p, slot, SL, SR, vel);
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const int row = Ly::R_CON + 4 * slot + e;
          L[Ly::RD + row] = active ? 1.0f / R : 0.0f;
          L[Ly::AREF + row] = active ? (-b * vel[e] - k * imp * pos) : 0.0f;
        }
      }
    }
  }

  // spatial motion of body b for joint-space vector at LDS offset X
  static DK void spatial(S L, int b, int X, float* Sp) {
#pragma unroll
    for (int k = 0; k < 6; k++) Sp[k] = 0.0f;
#pragma unroll
    for (int c = 0; c < Md::MAXCHAIN; c++) {
      if (c < Md::chain_len[b]) {
        const int i = Md::chain[b][c];
        const float x = L[X + i];
#pragma unroll
        for (int k = 0; k < 6; k++) Sp[k] += L[Ly::CDOF + 6 * i + k] * x;
      }
    }
  }

  // J.x for all rows -> DST (x at LDS offset X); sub_aref: DST = J.x - aref
  static DNI void jmul(S L, int X, int DST, bool sub_aref) {
#pragma unroll
    for (int r = 0; r < NFRIC; r++) L[DST + r] = L[X + Md::fric_dof[r]];
#pragma unroll
    for (int r = 0; r < NLIM; r++) L[DST + Ly::R_LIM + r] = L[Ly::LSGN + r] * L[X + Md::jnt_dofadr[Md::lim_jnt[r]]];
    float SL[6], SR[6];
    spatial(L, Md::LFOOT_BODY, X, SL);
    spatial(L, Md::RFOOT_BODY, X, SR);
#pragma unroll
    for (int p = 0; p < Md::NPAIR; p++)
#pragma unroll
      for (int c = 0; c < 4; c++) {
        float v[4];
        contact_jx(L, p, 4 * p + c, SL, SR, v);
#pragma unroll
        for (int e = 0; e < 4; e++) L[DST + Ly::R_CON + 4 * (4 * p + c) + e] = v[e];
      }
    if (sub_aref)
      for (int r = 0; r < NROW; r++) L[DST + r] -= L[Ly::AREF + r];
  }

  // constraint cost of all rows for Jaref stored at JA (mjx _update_constraint)
  static DNI float cost_rows(S L) {
    float cost = 0.0f;
#pragma unroll
    for (int r = 0; r < NFRIC; r++) {
      const float D = L[Ly::RD + r], x = L[Ly::JA + r], f = L[Ly::DFRIC + Md::fric_dof[r]];
      const float rf = f / D;
      cost += x <= -rf ? (-f * x - 0.5f * rf * f) : (x >= rf ? (f * x - 0.5f * rf * f) : 0.5f * D * x * x);
    }
    for (int r = Ly::R_LIM; r < NROW; r++) {
      const float D = L[Ly::RD + r], x = L[Ly::JA + r];
      cost += x < 0.0f ? 0.5f * D * x * x : 0.0f;
    }
    return cost;
  }

  // 0.5 (M x - f_smooth).(x - qacc_smooth) with M x at MX
  static DK float gauss(S L, int X, int MX) {
    float g = 0.0f;
#pragma unroll
    for (int i = 0; i < NV; i++) g += 0.5f * (L[MX + i] - L[Ly::FSM + i]) * (L[X + i] - L[Ly::QSM + i]);
    return g;
  }

  static DNI void mul_M(S L, int X, int Y) {
    S Ms{L.p + Ly::M * WG};
    float x[NV], y[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) x[i] = L[X + i];
    Md::mul_sym(Ms, x, y);
#pragma unroll
    for (int i = 0; i < NV; i++) L[Y + i] = y[i];
  }

  struct LsPt { float alpha, cost, d0, d1; };

  static DNI LsPt ls_eval(S L, float q0, float q1, float q2, float alpha) {
#pragma unroll
    for (int r = 0; r < NFRIC; r++) {
      const float D = L[Ly::RD + r], ja = L[Ly::JA + r], v = L[Ly::JV + r], f = L[Ly::DFRIC + Md::fric_dof[r]];
      const float rf = f / D, x = ja + alpha * v;
      if (x <= -rf) { q0 += -0.5f * rf * f - f * ja; q1 += -f * v; }
      else if (x >= rf) { q0 += -0.5f * rf * f + f * ja; q1 += f * v; }
      else { q0 += 0.5f * D * ja * ja; q1 += D * v * ja; q2 += 0.5f * D * v * v; }
    }
    for (int r = Ly::R_LIM; r < NROW; r++) {
      const float D = L[Ly::RD + r], ja = L[Ly::JA + r], v = L[Ly::JV + r];
      const float x = ja + alpha * v;
      if (x < 0.0f) { q0 += 0.5f * D * ja * ja; q1 += D * v * ja; q2 += 0.5f * D * v * v; }
    }
    LsPt p;
    p.alpha = alpha;
    p.cost = alpha * alpha * q2 + alpha * q1 + q0;
    p.d0 = 2.0f * alpha * q2 + q1;
    p.d1 = 2.0f * q2;
    return p;
  }

  // gradient and Newton direction at JA/MA (mjx _update_gradient): SRCH = -H^-1 grad
  static DNI bool newton_direction(S L) {
#pragma unroll
    for (int i = 0; i < NV; i++) L[Ly::GRAD + i] = L[Ly::MA + i] - L[Ly::FSM + i];
#pragma unroll
    for (int k = 0; k < Md::NM; k++) L[Ly::H + k] = L[Ly::M + k];
#pragma unroll
    for (int r = 0; r < NFRIC; r++) {
      const int i = Md::fric_dof[r];
      const float D = L[Ly::RD + r], x = L[Ly::JA + r], f = L[Ly::DFRIC + i], rf = f / D;
      const float force = x <= -rf ? f : (x >= rf ? -f : -D * x);
      L[Ly::GRAD + i] -= force;
      if (x > -rf && x < rf) L[Ly::H + Md::M_adr[i][i]] += D;
    }
#pragma unroll
    for (int r = 0; r < NLIM; r++) {
      const int i = Md::jnt_dofadr[Md::lim_jnt[r]];
      const float D = L[Ly::RD + Ly::R_LIM + r], x = L[Ly::JA + Ly::R_LIM + r];
      if (x < 0.0f) {
        L[Ly::GRAD + i] -= L[Ly::LSGN + r] * (-D * x);
        L[Ly::H + Md::M_adr[i][i]] += D;
      }
    }
    for (int k = 0; k < 21; k++) { L[Ly::KL + k] = 0.0f; L[Ly::KR + k] = 0.0f; }
    for (int k = 0; k < 36; k++) L[Ly::KLR + k] = 0.0f;
    for (int k = 0; k < 6; k++) { L[Ly::FL + k] = 0.0f; L[Ly::FR + k] = 0.0f; }
    bool ff_active = false;
#pragma unroll
    for (int p = 0; p < Md::NPAIR; p++) {
      const int s1 = cgeom_slot<Md>(Md::pair_geom1[p]), s2 = cgeom_slot<Md>(Md::pair_geom2[p]);
      const float mu = Md::pair_friction[p][0];
      const bool ff = (s1 != 0 && s2 != 0);
#pragma unroll 1
      for (int c = 0; c < 4; c++) {
        asm volatile("" ::: "memory");
        const int slot = 4 * p + c;
        const float r[3] = {L[Ly::CR + 3 * slot], L[Ly::CR + 3 * slot + 1], L[Ly::CR + 3 * slot + 2]};
        for (int e = 0; e < 4; e++) {
          const int row = Ly::R_CON + 4 * slot + e;
          const float D = L[Ly::RD + row], x = L[Ly::JA + row];
          if (!(x < 0.0f) || D == 0.0f) continue;
          const int t = 1 + (e >> 1);
          const float sg = (e & 1) ? -mu : mu;
          float u[3], a[6];
#pragma unroll
          for (int q = 0; q < 3; q++) u[q] = L[Ly::CFR + 9 * slot + q] + sg * L[Ly::CFR + 9 * slot + 3 * t + q];
          cross3(a, r, u);
          a[3] = u[0]; a[4] = u[1]; a[5] = u[2];
          const float force = -D * x;
          const int K2 = (s2 == 1) ? Ly::KL : Ly::KR, F2 = (s2 == 1) ? Ly::FL : Ly::FR;
          int o = 0;
#pragma unroll
          for (int q = 0; q < 6; q++)
#pragma unroll
            for (int kk = q; kk < 6; kk++) { L[K2 + o] += D * a[q] * a[kk]; o++; }
#pragma unroll
          for (int q = 0; q < 6; q++) L[F2 + q] += force * a[q];
          if (ff) {
            ff_active = true;
            o = 0;
#pragma unroll
            for (int q = 0; q < 6; q++)
#pragma unroll
              for (int kk = q; kk < 6; kk++) { L[Ly::KL + o] += D * a[q] * a[kk]; o++; }
#pragma unroll
            for (int q = 0; q < 6; q++) {
              L[Ly::FL + q] -= force * a[q];
#pragma unroll
              for (int kk = 0; kk < 6; kk++) L[Ly::KLR + 6 * q + kk] -= D * a[q] * a[kk];
            }
          }
        }
      }
    }
    // project K_b / F_b onto the foot's dof chain
#pragma unroll
    for (int side = 0; side < 2; side++) {
      const int b = side == 0 ? Md::LFOOT_BODY : Md::RFOOT_BODY;
      const int KO = side == 0 ? Ly::KL : Ly::KR, FO = side == 0 ? Ly::FL : Ly::FR;
      float Kf[6][6], F[6];
      int o = 0;
#pragma unroll
      for (int q = 0; q < 6; q++)
#pragma unroll
        for (int kk = q; kk < 6; kk++) { const float v = L[KO + o]; Kf[q][kk] = v; Kf[kk][q] = v; o++; }
#pragma unroll
      for (int q = 0; q < 6; q++) F[q] = L[FO + q];
#pragma unroll
      for (int cj = 0; cj < Md::MAXCHAIN; cj++) {
        if (cj >= Md::chain_len[b]) continue;
        asm volatile("" ::: "memory");
        const int j = Md::chain[b][cj];
        float cdj[6], kc[6];
#pragma unroll
        for (int k = 0; k < 6; k++) cdj[k] = L[Ly::CDOF + 6 * j + k];
        float g = 0.0f;
#pragma unroll
        for (int q = 0; q < 6; q++) {
          float s = 0.0f;
#pragma unroll
          for (int k = 0; k < 6; k++) s += Kf[q][k] * cdj[k];
          kc[q] = s;
          g += cdj[q] * F[q];
        }
        L[Ly::GRAD + j] -= g;
#pragma unroll
        for (int ci = 0; ci < Md::MAXCHAIN; ci++) {
          if (ci < cj || ci >= Md::chain_len[b]) continue;
          const int i = Md::chain[b][ci];
          float s = 0.0f;
#pragma unroll
          for (int k = 0; k < 6; k++) s += L[Ly::CDOF + 6 * i + k] * kc[k];
          L[Ly::H + Md::M_adr[i][j]] += s;
        }
      }
    }
    return ff_active;
  }

  static DNI void factor_H(S L) {
    S Hs{L.p + Ly::H * WG};
    Md::ldl_factor(Hs);
  }
  // DST = sign * H^-1 SRC (H factored in place)
  static DNI void solve_H(S L, int SRC, int DST, float sign) {
    S Hs{L.p + Ly::H * WG};
    float x[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) x[i] = L[SRC + i];
    Md::ldl_solve(Hs, x);
#pragma unroll
    for (int i = 0; i < NV; i++) L[DST + i] = sign * x[i];
  }

  // dense fallback when foot/foot contact rows couple the two leg chains
  static DNI void dense_direction(S L, float* A, int stride) {
    auto At = [&](int i, int j) -> float& { return A[(i * NV + j) * stride]; };
    for (int i = 0; i < NV; i++)
      for (int j = 0; j < NV; j++) At(i, j) = 0.0f;
#pragma unroll
    for (int i = 0; i < NV; i++)
#pragma unroll
      for (int j = 0; j <= i; j++)
        if (Md::M_adr[i][j] >= 0) {
          const float v = L[Ly::H + Md::M_adr[i][j]];
          At(i, j) = v;
          At(j, i) = v;
        }
    constexpr int bl = Md::LFOOT_BODY, br = Md::RFOOT_BODY;
    const int(*CH)[Md::MAXCHAIN] = Md::chain_d();
    for (int cl = 0; cl < Md::chain_len[bl]; cl++) {
      const int i = CH[bl][cl];
      float kc[6];
      for (int k = 0; k < 6; k++) {
        float s = 0.0f;
        for (int q = 0; q < 6; q++) s += L[Ly::CDOF + 6 * i + q] * L[Ly::KLR + 6 * q + k];
        kc[k] = s;
      }
      for (int cr = 0; cr < Md::chain_len[br]; cr++) {
        const int j = CH[br][cr];
        float v = 0.0f;
        for (int k = 0; k < 6; k++) v += kc[k] * L[Ly::CDOF + 6 * j + k];
        At(i, j) += v;
        At(j, i) += v;
      }
    }
    for (int j = 0; j < NV; j++) {
      float s = At(j, j);
      for (int k = 0; k < j; k++) s -= At(j, k) * At(j, k);
      const float d = sqrtf(fmaxf(s, 1e-30f));
      At(j, j) = d;
      for (int i = j + 1; i < NV; i++) {
        float t = At(i, j);
        for (int k = 0; k < j; k++) t -= At(i, k) * At(j, k);
        At(i, j) = t / d;
      }
    }
    for (int i = 0; i < NV; i++) {
      float s = L[Ly::GRAD + i];
      for (int k = 0; k < i; k++) s -= At(i, k) * L[Ly::SRCH + k];
      L[Ly::SRCH + i] = s / At(i, i);
    }
    for (int i = NV - 1; i >= 0; i--) {
      float s = L[Ly::SRCH + i];
      for (int k = i + 1; k < NV; k++) s -= At(k, i) * L[Ly::SRCH + k];
      L[Ly::SRCH + i] = s / At(i, i);
    }
    for (int i = 0; i < NV; i++) L[Ly::SRCH + i] = -L[Ly::SRCH + i];
  }

  // mjx solver.solve with iterations = 1: warmstart choice, Newton direction, zoom line search
  static DNI void solve(S L, float* scratch, int stride) {
    mul_M(L, Ly::WARM, Ly::MA);
    const float gw = gauss(L, Ly::WARM, Ly::MA);
    jmul(L, Ly::WARM, Ly::JA, true);
    const float cw = gw + cost_rows(L);
    jmul(L, Ly::QSM, Ly::JA, true);
    const float cs = cost_rows(L);
    if (cw < cs) {
#pragma unroll
      for (int i = 0; i < NV; i++) L[Ly::QACC + i] = L[Ly::WARM + i];
      jmul(L, Ly::QACC, Ly::JA, true);  // MA already holds M qacc_warmstart
    } else {
#pragma unroll
      for (int i = 0; i < NV; i++) L[Ly::QACC + i] = L[Ly::QSM + i];
      mul_M(L, Ly::QACC, Ly::MA);  // JA already holds J qacc_smooth - aref
    }
    const float g0 = gauss(L, Ly::QACC, Ly::MA);
    const bool ff = newton_direction(L);
    if (ff) {
      dense_direction(L, scratch, stride);
    } else {
      factor_H(L);
      solve_H(L, Ly::GRAD, Ly::SRCH, -1.0f);
    }
    jmul(L, Ly::SRCH, Ly::JV, false);
    mul_M(L, Ly::SRCH, Ly::GRAD);  // GRAD is dead after the direction: reuse for M.search
    float sn = 0.0f, sMa = 0.0f, sf = 0.0f, sMv = 0.0f;
#pragma unroll
    for (int i = 0; i < NV; i++) {
      const float s = L[Ly::SRCH + i];
      sn += s * s;
      sMa += s * L[Ly::MA + i];
      sf += s * L[Ly::FSM + i];
      sMv += s * L[Ly::GRAD + i];
    }
    const float gtol = Md::tolerance * Md::ls_tolerance * sqrtf(sn) * Md::meaninertia * (float)(NV > 1 ? NV : 1);
    const float q0 = g0, q1 = sMa - sf, q2 = 0.5f * sMv;
    LsPt p0 = ls_eval(L, q0, q1, q2, 0.0f);
    LsPt lo = ls_eval(L, q0, q1, q2, p0.alpha - p0.d0 / p0.d1);
    LsPt hi;
    if (lo.d0 < p0.d0) { hi = p0; } else { hi = lo; lo = p0; }
    bool swap = true;
    for (int it = 0; it < Md::ls_iterations; it++) {
      bool done = !swap;
      done = done || ((lo.d0 < 0.0f) && (lo.d0 > -gtol));
      done = done || ((hi.d0 > 0.0f) && (hi.d0 < gtol));
      if (done) break;
      const LsPt lo_next = ls_eval(L, q0, q1, q2, lo.alpha - lo.d0 / lo.d1);
      const LsPt hi_next = ls_eval(L, q0, q1, q2, hi.alpha - hi.d0 / hi.d1);
      const LsPt mid = ls_eval(L, q0, q1, q2, 0.5f * (lo.alpha + hi.alpha));
      const bool s1 = (lo.d0 > 0.0f) || (lo.d0 < lo_next.d0);
      if (s1) lo = lo_next;
      const bool s2 = (mid.d0 < 0.0f) && (lo.d0 < mid.d0);
      if (s2) lo = mid;
      const bool s3 = (hi.d0 < 0.0f) || (hi.d0 > hi_next.d0);
      if (s3) hi = hi_next;
      const bool s4 = (mid.d0 > 0.0f) && (hi.d0 > mid.d0);
      if (s4) hi = mid;
      swap = s1 || s2 || s3 || s4;
    }
    const bool improved = (lo.cost < p0.cost) || (hi.cost < p0.cost);
    const float alpha = lo.cost < hi.cost ? lo.alpha : hi.alpha;
    if (improved) {
#pragma unroll
      for (int i = 0; i < NV; i++) L[Ly::QACC + i] += L[Ly::SRCH + i] * alpha;
    }
  }

  // ---------------- sensors and env-facing outputs (pre-integration) ----------------
  static DNI void sensors(S L) {
    float com[3] = {L[Ly::COM], L[Ly::COM + 1], L[Ly::COM + 2]};
    float cacc1[6];
#pragma unroll
    for (int k = 0; k < 6; k++) cacc1[k] = (k >= 3) ? -Md::gravity[k - 3] : 0.0f;
#pragma unroll
    for (int i = 0; i < 6; i++) {
      const float v = L[Ly::QVEL + i], a = L[Ly::QACC + i];
#pragma unroll
      for (int k = 0; k < 6; k++) {
        const float cdd = i >= 3 ? L[Ly::CDD1 + 6 * (i - 3) + k] : 0.0f;
        cacc1[k] += cdd * v + L[Ly::CDOF + 6 * i + k] * a;
      }
    }
#pragma unroll
    for (int s = 0; s < Md::NSENSOR; s++) {
      SCHED_FENCE();
      const int typ = Md::sensor_type[s], site = Md::sensor_objid[s], adr = Md::sensor_adr[s];
      const int b = Md::site_bodyid[site];
      float R[9], sp[3], sR[9], t[3];
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = L[Ly::XMAT + 9 * b + k];
      mulmv3(t, R, Md::site_pos[site]);
#pragma unroll
      for (int k = 0; k < 3; k++) sp[k] = L[Ly::XPOS + 3 * b + k] + t[k];
      mulmm3(sR, R, Md::site_mat[site]);
      const float off[3] = {sp[0] - com[0], sp[1] - com[1], sp[2] - com[2]};
      float ang[3] = {L[Ly::CVEL + 6 * b], L[Ly::CVEL + 6 * b + 1], L[Ly::CVEL + 6 * b + 2]}, lin[3];
      cross3(t, ang, off);
#pragma unroll
      for (int k = 0; k < 3; k++) lin[k] = L[Ly::CVEL + 6 * b + 3 + k] + t[k];
      float o[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (typ == 0) mulmtv3(o, sR, ang);
      else if (typ == 1) mulmtv3(o, sR, lin);
      else if (typ == 2) {
        float acc[3];
        cross3(t, cacc1, off);
#pragma unroll
        for (int k = 0; k < 3; k++) acc[k] = cacc1[3 + k] + t[k];
        cross3(t, ang, lin);
#pragma unroll
        for (int k = 0; k < 3; k++) acc[k] += t[k];
        mulmtv3(o, sR, acc);
      } else if (typ == 3) { o[0] = sR[2]; o[1] = sR[5]; o[2] = sR[8]; }
      else if (typ == 4) { o[0] = sR[0]; o[1] = sR[3]; o[2] = sR[6]; }
      else if (typ == 5) { o[0] = lin[0]; o[1] = lin[1]; o[2] = lin[2]; }
      else if (typ == 6) { o[0] = ang[0]; o[1] = ang[1]; o[2] = ang[2]; }
      else if (typ == 7) { o[0] = sp[0]; o[1] = sp[1]; o[2] = sp[2]; }
      else if (typ == 8) {
        float bq[4] = {L[Ly::XQ + 4 * b], L[Ly::XQ + 4 * b + 1], L[Ly::XQ + 4 * b + 2], L[Ly::XQ + 4 * b + 3]};
        qmul(o, bq, Md::site_quat[site]);
        qnormalize(o);
      }
      const int dim = typ == 8 ? 4 : 3;
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (k < dim) L[Ly::SENS + adr + k] = o[k];
      if (site == Md::IMU_SITE) { L[Ly::IMUR] = sR[6]; L[Ly::IMUR + 1] = sR[7]; L[Ly::IMUR + 2] = sR[8]; }
      if (site == Md::LFOOT_SITE) L[Ly::FOOTZ] = sp[2];
      if (site == Md::RFOOT_SITE) L[Ly::FOOTZ + 1] = sp[2];
    }
#pragma unroll
    for (int p = 0; p < Md::NPAIR; p++) {
      const int s1 = cgeom_slot<Md>(Md::pair_geom1[p]), s2 = cgeom_slot<Md>(Md::pair_geom2[p]);
      if (s1 != 0) continue;
      float mn = 1e4f;
#pragma unroll
      for (int c = 0; c < 4; c++) mn = fminf(mn, L[Ly::CDIST + 4 * p + c]);
      L[Ly::OCON + s2 - 1] = mn < 0.0f ? 1.0f : 0.0f;
    }
  }

  // debug record: qacc, qacc_smooth, qvel (pre-integration), qfrc_smooth, actuator_force,
  // sensordata, con_dist, con_pos, M
  static DNI void write_aux(S L, float* aux, int stride) {
    int o = 0;
    for (int i = 0; i < NV; i++) aux[(o++) * stride] = L[Ly::QACC + i];
    for (int i = 0; i < NV; i++) aux[(o++) * stride] = L[Ly::QSM + i];
    for (int i = 0; i < NV; i++) aux[(o++) * stride] = L[Ly::QVEL + i];
    for (int i = 0; i < NV; i++) aux[(o++) * stride] = L[Ly::FSM + i];
    for (int a = 0; a < NU; a++) aux[(o++) * stride] = L[Ly::AF + a];
    for (int k = 0; k < Md::NSENSORDATA; k++) aux[(o++) * stride] = L[Ly::SENS + k];
    for (int s = 0; s < NCON; s++) aux[(o++) * stride] = L[Ly::CDIST + s];
    for (int s = 0; s < NCON; s++)
      for (int a = 0; a < 3; a++) aux[(o++) * stride] = L[Ly::CR + 3 * s + a] + L[Ly::COM + a];
    for (int k = 0; k < Md::NM; k++) aux[(o++) * stride] = L[Ly::M + k];
#ifdef DUCK_AUX_LDS
    // debug builds: the whole env slice (Lay fields + the team's chain/spatial scratch)
    for (int k = 0; k < Ly::TOTAL + 12 * Md::MAXCHAIN + 24; k++) aux[(o++) * stride] = L[k];
#endif
  }

  // ---------------- semi-implicit Euler (eulerdamp disabled) ----------------
  static DNI void euler(S L) {
    const float dt = Md::timestep;
#pragma unroll
    for (int i = 0; i < NV; i++) L[Ly::QVEL + i] += dt * L[Ly::QACC + i];
#pragma unroll
    for (int k = 0; k < 3; k++) L[Ly::QPOS + k] += dt * L[Ly::QVEL + k];
    const float v[3] = {L[Ly::QVEL + 3], L[Ly::QVEL + 4], L[Ly::QVEL + 5]};
    const float nvv = sqrtf(dot3(v, v));
    float ax[3] = {1.0f, 0.0f, 0.0f};
    if (nvv > 1e-15f) { ax[0] = v[0] / nvv; ax[1] = v[1] / nvv; ax[2] = v[2] / nvv; }
    float s, c;
    sincosf(0.5f * dt * nvv, &s, &c);
    const float qr[4] = {c, ax[0] * s, ax[1] * s, ax[2] * s};
    float q[4] = {L[Ly::QPOS + 3], L[Ly::QPOS + 4], L[Ly::QPOS + 5], L[Ly::QPOS + 6]};
    qmul(q, q, qr);
    qnormalize(q);
#pragma unroll
    for (int k = 0; k < 4; k++) L[Ly::QPOS + 3 + k] = q[k];
#pragma unroll
    for (int j = 1; j < Md::NJ; j++) L[Ly::QPOS + Md::jnt_qposadr[j]] += dt * L[Ly::QVEL + Md::jnt_dofadr[j]];
  }

  // one substep: forward (+ outputs when want_out) and optional integration
  static DK void step(S L, bool integrate, bool want_out, float* aux, int aux_stride, float* scratch, int sstride) {
    STAGE_T0();
    kinematics(L);
    STAGE_MARK(0);
    com_pos(L);
    STAGE_MARK(1);
    rne(L);
    STAGE_MARK(2);
    crb(L);
    STAGE_MARK(3);
    smooth(L);
    factor_H(L);
    solve_H(L, Ly::FSM, Ly::QSM, 1.0f);
    STAGE_MARK(4);
    collision(L);
    STAGE_MARK(5);
    make_rows(L);
    STAGE_MARK(6);
    solve(L, scratch, sstride);
    STAGE_MARK(7);
    if (want_out) {
      sensors(L);
      if (aux) write_aux(L, aux, aux_stride);
    }
#pragma unroll
    for (int i = 0; i < NV; i++) L[Ly::WARM + i] = L[Ly::QACC + i];
    if (integrate) euler(L);
    STAGE_MARK(8);
  }
};

template <class Md>
constexpr int aux_size() {
  return 4 * Md::NV + Md::NU + Md::NSENSORDATA + 4 * Lay<Md>::NCON + Md::NM
#ifdef DUCK_AUX_LDS
         + Lay<Md>::TOTAL + 12 * Md::MAXCHAIN + 24
#endif
      ;
}
