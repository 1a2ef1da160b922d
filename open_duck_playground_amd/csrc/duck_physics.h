// duck_physics.h — per-env LDS layout and shared physics helpers of the MI355X Open Duck kernels.
//
// The fused mjx.step itself (kinematics -> com/cinert/cdof -> RNE -> CRB -> actuation/passive ->
// smooth acceleration -> collision -> constraint rows -> MJX Newton -> sensors -> Euler) is the
// 16-lane team implementation in duck_team.h. This header holds what it builds on: the per-env LDS
// slice layout (Lay), the impedance law (kbi), the plane/convex manifold helpers, and a few per-env
// helpers (Phys). The round-1 single-lane debug build (one env per lane, -DDUCK_TEAM=0) is retired.
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
#if defined(DUCK_STAGE_PROF) || defined(DUCK_WAVE_PROF) || defined(DUCK_LAT_PROF)
#define DUCK_ANY_PROF 1
#endif
#ifdef DUCK_ANY_PROF
#define DUCK_NSTAGE 60
static __device__ unsigned long long g_stage_cycles[DUCK_NSTAGE + 3 * 1024];
// the stage counters themselves are kept per workgroup slot (summed by the host): one shared
// counter per stage made every workgroup's atomics contend at one L2 channel, which slowed whole
// XCDs by up to 30 % in profiled runs
static __device__ unsigned long long g_stage_wg[DUCK_NSTAGE * 256];
#define STAGE_ADD(k, v) atomicAdd(&g_stage_wg[(k) * 256 + (blockIdx.x & 255)], (v))
#endif
#ifdef DUCK_STAGE_PROF
// g_stage_cycles: [0, DUCK_NSTAGE) stage counters; then per wave of the first 1024: clock64 cycles,
// wall-clock (s_memrealtime, 100 MHz) start, wall-clock end; [DUCK_NSTAGE, DUCK_NSTAGE + 1024) cycles of each of the first 1024 waves
// of the last step_kernel launch (wave = 4 * workgroup + wave-in-workgroup), for the launch tail
#define STAGE_T0() unsigned long long _t0 = wall_clock64(), _c0 = clock64()
#define STAGE_RESET() (_c0 = clock64())
#define STAGE_MARK(k)                                                             \
  do {                                                                            \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                            \
    const unsigned long long _c1 = clock64();                                     \
    if (threadIdx.x == 0) STAGE_ADD(k, _c1 - _c0);                                \
    _c0 = _c1;                                                                    \
    (void)_t0;                                                                    \
  } while (0)
#elif defined(DUCK_LAT_PROF)
// latency-kernel builds (tools/lat_prof.py): each stage's cycles summed over the launch in workgroup 0
// (lane 0 of the wave that runs it; in the latency kernel every stage runs on one wave) into
// g_stage_cycles[DUCK_NSTAGE + 64 + k]; the waits between stages are outside every stage
#define STAGE_T0() unsigned long long _c0 = clock64()
#define STAGE_RESET() (_c0 = clock64())
#define STAGE_MARK(k)                                                                  \
  do {                                                                                 \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                 \
    const unsigned long long _c1 = clock64();                                          \
    if (blockIdx.x == 0 && ((int)threadIdx.x & 63) == 0) g_stage_cycles[DUCK_NSTAGE + 64 + (k)] += _c1 - _c0; \
    _c0 = _c1;                                                                         \
  } while (0)
#elif defined(DUCK_ASM_MARKS)
// static instruction counts per stage (tools/isa_stage_hist.py on hipcc -S output): a comment
// at each stage boundary, no code
#define STAGE_T0() \
  do {             \
  } while (0)
#define STAGE_MARK(k) asm volatile("; STAGE_MARK " #k ::: "memory")
#define STAGE_RESET() \
  do {                \
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
  // M, then one word kept at zero (crb writes it with M): the register column
  // loads of M read it for the entries outside the tree pattern (codegen mcolz table)
  static constexpr int M = CDD1 + 18, MZERO = M + Md::NM, H = MZERO + 1;
  // H: scratch in front of the constraint rows, dead outside the stage that uses it together with
  // the rows (the Newton Hessian itself is assembled in registers, never stored). Its users, each
  // from H on: the tree passes' scratch (rne: 12 NB + 6 NV), the hull/hull SAT's edge tables (6 per
  // hull edge and face), the height-field survivor queue (16 entries of 28 per env slice + 16-B
  // alignment), the staged privileged observation row (env code, 86 + 9 NU). H is sized so that
  // H + rows covers the largest of them: the rows alone cover most, so H is short (the backlash
  // scenes' slices then leave LDS for the model blob: TLay::TAB_LDS).
  static constexpr int SCR_TREE = 12 * NB + 6 * NV, SCR_SAT = 6 * (Md::NHE + Md::NHF);
  static constexpr int SCR_HF = Md::FLOOR_TYPE == 1 ? 3 + 28 * 16 : 0, SCR_OBS = 86 + 9 * NU;
  static constexpr int cmax(int a, int b) { return a > b ? a : b; }
  static constexpr int SCR_NEED = cmax(cmax(SCR_TREE, SCR_SAT), cmax(SCR_HF, SCR_OBS));
  static constexpr int NROWS = NROW;
  static constexpr int HSZ = ((cmax(SCR_NEED - 4 * NROWS - Md::NLIM, 0) + 3) / 4) * 4;
  // RNE accumulators live in the H + row storage (dead until smooth()/make_rows())
  static constexpr int CACC = H, CFRC = CACC + 6 * NB;
  static_assert(12 * NB <= HSZ + 4 * NROW, "RNE scratch must fit in H + rows");
  static constexpr int JA = H + HSZ, JV = JA + NROWS, RD = JV + NROWS, AREF = RD + NROWS;
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

// Per-env helpers shared with the team kernels (duck_team.h): nominal per-env model values, collision
// geom frames, contact records, contact point velocity, the debug aux record.
template <class Md, int WG>
struct Phys {
  using Ly = Lay<Md>;
  using S = Slice<WG>;
  static constexpr int NV = Md::NV, NB = Md::NB, NQ = Md::NQ, NU = Md::NU;
  static constexpr int NCON = Ly::NCON;

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

  // ---------------- constraint rows (mjx make_constraint) ----------------
  static DK void contact_vel(const float* Sp, const float* r, float* v) {
    float t[3];
    cross3(t, Sp, r);
    v[0] = Sp[3] + t[0]; v[1] = Sp[4] + t[1]; v[2] = Sp[5] + t[2];
  }

  // debug record: qacc, qacc_smooth, qvel (pre-integration), qfrc_smooth, actuator_force,
  // sensordata, con_dist, con_pos, con_normal, M
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
    for (int s = 0; s < NCON; s++)
      for (int a = 0; a < 3; a++) aux[(o++) * stride] = L[Ly::CFR + 9 * s + a];  // contact normal
    for (int k = 0; k < Md::NM; k++) aux[(o++) * stride] = L[Ly::M + k];
#ifdef DUCK_AUX_LDS
    // debug builds: the whole env slice (Lay fields + the team's chain/spatial scratch)
    for (int k = 0; k < Ly::TOTAL + 12 * Md::MAXCHAIN + 24; k++) aux[(o++) * stride] = L[k];
#endif
  }
};

template <class Md>
constexpr int aux_size() {
  return 4 * Md::NV + Md::NU + Md::NSENSORDATA + 7 * Lay<Md>::NCON + Md::NM
#ifdef DUCK_AUX_LDS
         + Lay<Md>::TOTAL + 12 * Md::MAXCHAIN + 24
#endif
      ;
}
