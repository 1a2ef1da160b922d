/* duck_oracle.c — CPU (fp64) restatement of the Open Duck Joystick hot path.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline). See duck_oracle.h for the
 * scope and DESIGN.md for what is pinned and what is not. Every block cites the
 * reference file:line it restates; physics blocks name the upstream MuJoCo/MJX stage.
 */
#include "duck_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define MINVAL 1e-15
#define PI 3.14159265358979323846
#define MINIMP 0.0001
#define MAXIMP 0.9999
#define MAXEFC 128
#define NV DUCK_MAXV
#define DUCK_HULL_SAT_TIE 1e-5 /* m; = codegen.HULL_SAT_TIE */

struct oracle_model {
  int nq, nv, nu, nbody, njnt, ngeom, nsite, nsensor, nsensordata, npair;
  double timestep, gravity[3], impratio, tolerance, ls_tolerance, meaninertia;
  int iterations, ls_iterations, eulerdamp;
  int body_parentid[DUCK_MAXBODY], body_rootid[DUCK_MAXBODY], body_weldid[DUCK_MAXBODY],
      body_jntnum[DUCK_MAXBODY], body_jntadr[DUCK_MAXBODY], body_dofnum[DUCK_MAXBODY], body_dofadr[DUCK_MAXBODY];
  double body_pos[DUCK_MAXBODY][3], body_quat[DUCK_MAXBODY][4], body_ipos[DUCK_MAXBODY][3],
      body_iquat[DUCK_MAXBODY][4], body_mass[DUCK_MAXBODY], body_inertia[DUCK_MAXBODY][3],
      body_invweight0[DUCK_MAXBODY][2];
  int jnt_type[DUCK_MAXJNT], jnt_qposadr[DUCK_MAXJNT], jnt_dofadr[DUCK_MAXJNT], jnt_bodyid[DUCK_MAXJNT],
      jnt_limited[DUCK_MAXJNT];
  double jnt_pos[DUCK_MAXJNT][3], jnt_axis[DUCK_MAXJNT][3], jnt_range[DUCK_MAXJNT][2], jnt_margin[DUCK_MAXJNT],
      jnt_solref[DUCK_MAXJNT][2], jnt_solimp[DUCK_MAXJNT][5];
  int dof_bodyid[NV], dof_jntid[NV], dof_parentid[NV];
  double dof_armature[NV], dof_damping[NV], dof_frictionloss[NV], dof_invweight0[NV], dof_solref[NV][2],
      dof_solimp[NV][5];
  int dof_has_friction[NV]; /* row selection from the nominal model (MJX: static) */
  int geom_type[DUCK_MAXGEOM], geom_bodyid[DUCK_MAXGEOM], geom_dataid[DUCK_MAXGEOM];
  double geom_pos[DUCK_MAXGEOM][3], geom_quat[DUCK_MAXGEOM][4], geom_rbound[DUCK_MAXGEOM], geom_size[DUCK_MAXGEOM][3];
  int pair_geom1[DUCK_MAXPAIR], pair_geom2[DUCK_MAXPAIR], pair_condim[DUCK_MAXPAIR];
  double pair_friction[DUCK_MAXPAIR][5], pair_solref[DUCK_MAXPAIR][2], pair_solimp[DUCK_MAXPAIR][5],
      pair_margin[DUCK_MAXPAIR];
  int hull_nvert, hull_nface, hull_nedge;
  double hull_vert[DUCK_MAXHULLV][3], hull_face_normal[DUCK_MAXHULLF][3], hull_face_offset[DUCK_MAXHULLF];
  int hull_edge[DUCK_MAXHULLE][2];
  int hull_edge_face[DUCK_MAXHULLE][2]; /* the two faces whose planes hold the edge */
  int hull_face_nv[DUCK_MAXHULLF], hull_face_vert[DUCK_MAXHULLF][DUCK_MAXHULLV]; /* face polygons (CCW) */
  double hull_center[3], hull_radius;
  int hfield_nrow, hfield_ncol;
  double hfield_size[4];
  double* hfield_data;
  int site_bodyid[DUCK_MAXSITE];
  double site_pos[DUCK_MAXSITE][3], site_quat[DUCK_MAXSITE][4];
  int actuator_trnid[DUCK_MAXU], actuator_ctrllimited[DUCK_MAXU], actuator_forcelimited[DUCK_MAXU];
  double actuator_kp[DUCK_MAXU], actuator_kv[DUCK_MAXU], actuator_gear[DUCK_MAXU], actuator_ctrlrange[DUCK_MAXU][2],
      actuator_forcerange[DUCK_MAXU][2];
  int sensor_type[DUCK_MAXSENSOR], sensor_objid[DUCK_MAXSENSOR], sensor_adr[DUCK_MAXSENSOR],
      sensor_dim[DUCK_MAXSENSOR];
  double qpos0[DUCK_MAXQ];
};

/* ------------------------------------------------------------------------------------ */
/* model                                                                                */
/* ------------------------------------------------------------------------------------ */

#define CP(dst, src, n) memcpy((dst), (src), sizeof(*(src)) * (size_t)(n))

oracle_model* oracle_model_create(const duck_model_desc* s) {
  if (s->nbody > DUCK_MAXBODY || s->nv > DUCK_MAXV || s->nq > DUCK_MAXQ || s->nu > DUCK_MAXU ||
      s->njnt > DUCK_MAXJNT || s->ngeom > DUCK_MAXGEOM || s->npair > DUCK_MAXPAIR ||
      s->hull_nvert > DUCK_MAXHULLV || s->hull_nface > DUCK_MAXHULLF || s->hull_nedge > DUCK_MAXHULLE ||
      s->nsite > DUCK_MAXSITE || s->nsensor > DUCK_MAXSENSOR || s->nsensordata > DUCK_MAXSENSORDATA ||
      /* every constraint row fits the fixed-capacity Jacobian: friction <= nv, limits <= njnt, 4
       * pyramid rows per contact slot */
      s->nv + s->njnt + 4 * DUCK_CON_PER_PAIR * s->npair > MAXEFC)
    return NULL;
  oracle_model* m = (oracle_model*)calloc(1, sizeof(oracle_model));
  m->nq = s->nq; m->nv = s->nv; m->nu = s->nu; m->nbody = s->nbody; m->njnt = s->njnt; m->ngeom = s->ngeom;
  m->nsite = s->nsite; m->nsensor = s->nsensor; m->nsensordata = s->nsensordata; m->npair = s->npair;
  m->timestep = s->timestep; CP(m->gravity, s->gravity, 3); m->impratio = s->impratio;
  m->tolerance = s->tolerance; m->ls_tolerance = s->ls_tolerance; m->meaninertia = s->meaninertia;
  m->iterations = s->iterations; m->ls_iterations = s->ls_iterations; m->eulerdamp = s->eulerdamp;
  int nb = s->nbody;
  for (int i = 0; i < nb; i++) {
    m->body_parentid[i] = s->body_parentid[i]; m->body_rootid[i] = s->body_rootid[i];
    m->body_weldid[i] = s->body_weldid[i]; m->body_jntnum[i] = s->body_jntnum[i];
    m->body_jntadr[i] = s->body_jntadr[i]; m->body_dofnum[i] = s->body_dofnum[i];
    m->body_dofadr[i] = s->body_dofadr[i]; m->body_mass[i] = s->body_mass[i];
    CP(m->body_pos[i], s->body_pos + 3 * i, 3); CP(m->body_quat[i], s->body_quat + 4 * i, 4);
    CP(m->body_ipos[i], s->body_ipos + 3 * i, 3); CP(m->body_iquat[i], s->body_iquat + 4 * i, 4);
    CP(m->body_inertia[i], s->body_inertia + 3 * i, 3); CP(m->body_invweight0[i], s->body_invweight0 + 2 * i, 2);
  }
  for (int j = 0; j < s->njnt; j++) {
    m->jnt_type[j] = s->jnt_type[j]; m->jnt_qposadr[j] = s->jnt_qposadr[j]; m->jnt_dofadr[j] = s->jnt_dofadr[j];
    m->jnt_bodyid[j] = s->jnt_bodyid[j]; m->jnt_limited[j] = s->jnt_limited[j]; m->jnt_margin[j] = s->jnt_margin[j];
    CP(m->jnt_pos[j], s->jnt_pos + 3 * j, 3); CP(m->jnt_axis[j], s->jnt_axis + 3 * j, 3);
    CP(m->jnt_range[j], s->jnt_range + 2 * j, 2); CP(m->jnt_solref[j], s->jnt_solref + 2 * j, 2);
    CP(m->jnt_solimp[j], s->jnt_solimp + 5 * j, 5);
  }
  for (int i = 0; i < s->nv; i++) {
    m->dof_bodyid[i] = s->dof_bodyid[i]; m->dof_jntid[i] = s->dof_jntid[i]; m->dof_parentid[i] = s->dof_parentid[i];
    m->dof_armature[i] = s->dof_armature[i]; m->dof_damping[i] = s->dof_damping[i];
    m->dof_frictionloss[i] = s->dof_frictionloss[i]; m->dof_invweight0[i] = s->dof_invweight0[i];
    m->dof_has_friction[i] = s->dof_frictionloss[i] > 0;
    CP(m->dof_solref[i], s->dof_solref + 2 * i, 2); CP(m->dof_solimp[i], s->dof_solimp + 5 * i, 5);
  }
  for (int g = 0; g < s->ngeom; g++) {
    m->geom_type[g] = s->geom_type[g]; m->geom_bodyid[g] = s->geom_bodyid[g]; m->geom_dataid[g] = s->geom_dataid[g];
    m->geom_rbound[g] = s->geom_rbound[g];
    CP(m->geom_pos[g], s->geom_pos + 3 * g, 3); CP(m->geom_quat[g], s->geom_quat + 4 * g, 4);
    CP(m->geom_size[g], s->geom_size + 3 * g, 3);
  }
  for (int p = 0; p < s->npair; p++) {
    m->pair_geom1[p] = s->pair_geom1[p]; m->pair_geom2[p] = s->pair_geom2[p]; m->pair_condim[p] = s->pair_condim[p];
    CP(m->pair_friction[p], s->pair_friction + 5 * p, 5); CP(m->pair_solref[p], s->pair_solref + 2 * p, 2);
    CP(m->pair_solimp[p], s->pair_solimp + 5 * p, 5); m->pair_margin[p] = s->pair_margin[p];
  }
  m->hull_nvert = s->hull_nvert; m->hull_nface = s->hull_nface; m->hull_nedge = s->hull_nedge;
  double c[3] = {0, 0, 0};
  for (int k = 0; k < s->hull_nvert; k++) {
    CP(m->hull_vert[k], s->hull_vert + 3 * k, 3);
    for (int a = 0; a < 3; a++) c[a] += m->hull_vert[k][a] / s->hull_nvert;
  }
  double r = 0;
  for (int k = 0; k < s->hull_nvert; k++) {
    double dx = m->hull_vert[k][0] - c[0], dy = m->hull_vert[k][1] - c[1], dz = m->hull_vert[k][2] - c[2];
    double rr = sqrt(dx * dx + dy * dy + dz * dz);
    if (rr > r) r = rr;
  }
  CP(m->hull_center, c, 3); m->hull_radius = r;
  for (int f = 0; f < s->hull_nface; f++) {
    CP(m->hull_face_normal[f], s->hull_face_normal + 3 * f, 3);
    m->hull_face_offset[f] = s->hull_face_offset[f];
  }
  for (int e = 0; e < s->hull_nedge; e++) { m->hull_edge[e][0] = s->hull_edge[2 * e]; m->hull_edge[e][1] = s->hull_edge[2 * e + 1]; }
  /* edge -> adjacent faces: both endpoints on the face plane (vertices of other faces are
   * >= 2.7e-6 m off it for the Open Duck foot hull; codegen.hull_edge_faces builds the same
   * table from the polygons) */
  for (int e = 0; e < s->hull_nedge; e++) {
    int n = 0;
    for (int f = 0; f < s->hull_nface && n <= 2; f++) {
      const double *fnm = m->hull_face_normal[f], *va = m->hull_vert[m->hull_edge[e][0]],
                   *vb = m->hull_vert[m->hull_edge[e][1]];
      double da = fnm[0] * va[0] + fnm[1] * va[1] + fnm[2] * va[2] - m->hull_face_offset[f];
      double db = fnm[0] * vb[0] + fnm[1] * vb[1] + fnm[2] * vb[2] - m->hull_face_offset[f];
      if (fabs(da) < 1e-7 && fabs(db) < 1e-7) {
        if (n < 2) m->hull_edge_face[e][n] = f;
        n++;
      }
    }
    if (n != 2) { free(m); return NULL; }
  }
  /* face polygons: the vertices on the face plane, counter-clockwise about the outward normal,
   * ordered as mjcf.convex_hull orders them (angle from the lowest-index vertex about the
   * centroid, atan2 ascending), so that codegen's hull_face_vert table and this agree */
  for (int f = 0; f < s->hull_nface; f++) {
    const double* fnm = m->hull_face_normal[f];
    int nfv = 0, vid[DUCK_MAXHULLV];
    double cf[3] = {0, 0, 0};
    for (int k = 0; k < s->hull_nvert; k++) {
      const double* v = m->hull_vert[k];
      if (fabs(fnm[0] * v[0] + fnm[1] * v[1] + fnm[2] * v[2] - m->hull_face_offset[f]) < 1e-7) {
        vid[nfv++] = k;
        for (int a = 0; a < 3; a++) cf[a] += v[a];
      }
    }
    if (nfv < 3) { free(m); return NULL; }
    for (int a = 0; a < 3; a++) cf[a] /= nfv;
    double u[3], w[3], ang[DUCK_MAXHULLV];
    for (int a = 0; a < 3; a++) u[a] = m->hull_vert[vid[0]][a] - cf[a];
    const double un = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    for (int a = 0; a < 3; a++) u[a] /= un;
    w[0] = fnm[1] * u[2] - fnm[2] * u[1]; w[1] = fnm[2] * u[0] - fnm[0] * u[2]; w[2] = fnm[0] * u[1] - fnm[1] * u[0];
    for (int i = 0; i < nfv; i++) {
      const double* v = m->hull_vert[vid[i]];
      const double d[3] = {v[0] - cf[0], v[1] - cf[1], v[2] - cf[2]};
      ang[i] = atan2(d[0] * w[0] + d[1] * w[1] + d[2] * w[2], d[0] * u[0] + d[1] * u[1] + d[2] * u[2]);
    }
    for (int i = 1; i < nfv; i++) /* insertion sort by angle (stable) */
      for (int j = i; j > 0 && ang[j - 1] > ang[j]; j--) {
        const double ta = ang[j]; ang[j] = ang[j - 1]; ang[j - 1] = ta;
        const int tv = vid[j]; vid[j] = vid[j - 1]; vid[j - 1] = tv;
      }
    m->hull_face_nv[f] = nfv;
    for (int i = 0; i < nfv; i++) m->hull_face_vert[f][i] = vid[i];
  }
  m->hfield_nrow = s->hfield_nrow; m->hfield_ncol = s->hfield_ncol; CP(m->hfield_size, s->hfield_size, 4);
  if (s->hfield_nrow > 0) {
    m->hfield_data = (double*)malloc(sizeof(double) * (size_t)s->hfield_nrow * s->hfield_ncol);
    CP(m->hfield_data, s->hfield_data, (size_t)s->hfield_nrow * s->hfield_ncol);
  }
  for (int i = 0; i < s->nsite; i++) {
    m->site_bodyid[i] = s->site_bodyid[i];
    CP(m->site_pos[i], s->site_pos + 3 * i, 3); CP(m->site_quat[i], s->site_quat + 4 * i, 4);
  }
  for (int a = 0; a < s->nu; a++) {
    m->actuator_trnid[a] = s->actuator_trnid[a]; m->actuator_ctrllimited[a] = s->actuator_ctrllimited[a];
    m->actuator_forcelimited[a] = s->actuator_forcelimited[a]; m->actuator_kp[a] = s->actuator_kp[a];
    m->actuator_kv[a] = s->actuator_kv[a]; m->actuator_gear[a] = s->actuator_gear[a];
    CP(m->actuator_ctrlrange[a], s->actuator_ctrlrange + 2 * a, 2);
    CP(m->actuator_forcerange[a], s->actuator_forcerange + 2 * a, 2);
  }
  for (int i = 0; i < s->nsensor; i++) {
    m->sensor_type[i] = s->sensor_type[i]; m->sensor_objid[i] = s->sensor_objid[i];
    m->sensor_adr[i] = s->sensor_adr[i]; m->sensor_dim[i] = s->sensor_dim[i];
  }
  CP(m->qpos0, s->qpos0, s->nq);
  return m;
}

void oracle_model_destroy(oracle_model* m) {
  if (!m) return;
  free(m->hfield_data);
  free(m);
}

/* ------------------------------------------------------------------------------------ */
/* small math                                                                           */
/* ------------------------------------------------------------------------------------ */

static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void cross3(double* r, const double* a, const double* b) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  r[0] = t[0]; r[1] = t[1]; r[2] = t[2];
}
static double norm3(const double* a) { return sqrt(dot3(a, a)); }
static void mulmv3(double* r, const double* M, const double* v) {
  double t[3] = {M[0] * v[0] + M[1] * v[1] + M[2] * v[2], M[3] * v[0] + M[4] * v[1] + M[5] * v[2],
                 M[6] * v[0] + M[7] * v[1] + M[8] * v[2]};
  r[0] = t[0]; r[1] = t[1]; r[2] = t[2];
}
static void mulmtv3(double* r, const double* M, const double* v) {
  double t[3] = {M[0] * v[0] + M[3] * v[1] + M[6] * v[2], M[1] * v[0] + M[4] * v[1] + M[7] * v[2],
                 M[2] * v[0] + M[5] * v[1] + M[8] * v[2]};
  r[0] = t[0]; r[1] = t[1]; r[2] = t[2];
}
static void mulmm3(double* r, const double* A, const double* B) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
  memcpy(r, t, sizeof(t));
}
static void quat_mul(double* r, const double* a, const double* b) {
  double t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                 a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                 a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                 a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  memcpy(r, t, sizeof(t));
}
static void quat_normalize(double* q) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  for (int i = 0; i < 4; i++) q[i] /= n;
}
static void quat2mat(double* R, const double* q) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}
static void axis_angle_quat(double* q, const double* axis, double angle) {
  double s = sin(0.5 * angle);
  q[0] = cos(0.5 * angle); q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}

/* spatial algebra in MuJoCo's com-based convention: motion/force = [angular; linear] */
static void mul_inert_vec(double* r, const double* I, const double* v) {
  r[0] = I[0] * v[0] + I[3] * v[1] + I[4] * v[2] - I[8] * v[4] + I[7] * v[5];
  r[1] = I[3] * v[0] + I[1] * v[1] + I[5] * v[2] + I[8] * v[3] - I[6] * v[5];
  r[2] = I[4] * v[0] + I[5] * v[1] + I[2] * v[2] - I[7] * v[3] + I[6] * v[4];
  r[3] = I[8] * v[1] - I[7] * v[2] + I[9] * v[3];
  r[4] = I[6] * v[2] - I[8] * v[0] + I[9] * v[4];
  r[5] = I[7] * v[0] - I[6] * v[1] + I[9] * v[5];
}
static void cross_motion(double* r, const double* v, const double* u) {
  r[0] = -v[2] * u[1] + v[1] * u[2];
  r[1] = v[2] * u[0] - v[0] * u[2];
  r[2] = -v[1] * u[0] + v[0] * u[1];
  r[3] = -v[2] * u[4] + v[1] * u[5] - v[5] * u[1] + v[4] * u[2];
  r[4] = v[2] * u[3] - v[0] * u[5] + v[5] * u[0] - v[3] * u[2];
  r[5] = -v[1] * u[3] + v[0] * u[4] - v[4] * u[0] + v[3] * u[1];
}
static void cross_force(double* r, const double* v, const double* f) {
  r[0] = -v[2] * f[1] + v[1] * f[2] - v[5] * f[4] + v[4] * f[5];
  r[1] = v[2] * f[0] - v[0] * f[2] + v[5] * f[3] - v[3] * f[5];
  r[2] = -v[1] * f[0] + v[0] * f[1] - v[4] * f[3] + v[3] * f[4];
  r[3] = -v[2] * f[4] + v[1] * f[5];
  r[4] = v[2] * f[3] - v[0] * f[5];
  r[5] = -v[1] * f[3] + v[0] * f[4];
}
static double dot6(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

/* dense Cholesky (lower), in place; returns 0 on failure */
static int cholesky(double* A, int n) {
  for (int j = 0; j < n; j++) {
    double s = A[j * NV + j];
    for (int k = 0; k < j; k++) s -= A[j * NV + k] * A[j * NV + k];
    if (s <= MINVAL) return 0;
    double d = sqrt(s);
    A[j * NV + j] = d;
    for (int i = j + 1; i < n; i++) {
      double t = A[i * NV + j];
      for (int k = 0; k < j; k++) t -= A[i * NV + k] * A[j * NV + k];
      A[i * NV + j] = t / d;
    }
  }
  return 1;
}
static void chol_solve(const double* L, int n, double* x) {
  for (int i = 0; i < n; i++) {
    double s = x[i];
    for (int k = 0; k < i; k++) s -= L[i * NV + k] * x[k];
    x[i] = s / L[i * NV + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = x[i];
    for (int k = i + 1; k < n; k++) s -= L[k * NV + i] * x[k];
    x[i] = s / L[i * NV + i];
  }
}

/* ------------------------------------------------------------------------------------ */
/* forward-pass scratch                                                                 */
/* ------------------------------------------------------------------------------------ */

typedef struct fwd_ws {
  double xanchor[DUCK_MAXJNT][3], xaxis[DUCK_MAXJNT][3];
  double subtree_com[DUCK_MAXBODY][3];
  double cinert[DUCK_MAXBODY][10], crb[DUCK_MAXBODY][10];
  double cdof[NV][6], cdof_dot[NV][6], cvel[DUCK_MAXBODY][6];
  double site_xquat[DUCK_MAXSITE][4];
  /* constraint rows */
  int nefc;
  double J[MAXEFC][NV], D[MAXEFC], R[MAXEFC], aref[MAXEFC], frictionloss[MAXEFC];
  int ineq[MAXEFC]; /* 1: inequality (limit/contact), 0: friction */
} fwd_ws;

/* mj_kinematics (smooth.kinematics): body/site/geom frames from qpos.
 * Hinge rotation angle is qpos - qpos0 (MuJoCo semantics; DR jitters qpos0, randomize.py:78-86). */
static void kinematics(const oracle_model* m, oracle_data* d, fwd_ws* w) {
  d->xpos[0][0] = d->xpos[0][1] = d->xpos[0][2] = 0;
  d->xquat[0][0] = 1; d->xquat[0][1] = d->xquat[0][2] = d->xquat[0][3] = 0;
  quat2mat(d->xmat[0], d->xquat[0]);
  memcpy(d->xipos[0], d->xpos[0], sizeof(d->xpos[0]));
  memcpy(d->ximat[0], d->xmat[0], sizeof(d->xmat[0]));
  for (int i = 1; i < m->nbody; i++) {
    int p = m->body_parentid[i], ja = m->body_jntadr[i], jn = m->body_jntnum[i];
    if (jn > 0 && m->jnt_type[ja] == DUCK_JNT_FREE) {
      int a = m->jnt_qposadr[ja];
      memcpy(d->xpos[i], d->qpos + a, 3 * sizeof(double));
      memcpy(d->xquat[i], d->qpos + a + 3, 4 * sizeof(double));
      quat_normalize(d->xquat[i]);
      memcpy(w->xanchor[ja], d->xpos[i], 3 * sizeof(double));
      w->xaxis[ja][0] = 0; w->xaxis[ja][1] = 0; w->xaxis[ja][2] = 1;
    } else {
      double t[3], q[4], R[9];
      mulmv3(t, d->xmat[p], m->body_pos[i]);
      for (int k = 0; k < 3; k++) d->xpos[i][k] = d->xpos[p][k] + t[k];
      quat_mul(q, d->xquat[p], m->body_quat[i]);
      for (int j = ja; j < ja + jn; j++) {
        quat2mat(R, q);
        mulmv3(t, R, m->jnt_pos[j]);
        for (int k = 0; k < 3; k++) w->xanchor[j][k] = t[k] + d->xpos[i][k];
        mulmv3(w->xaxis[j], R, m->jnt_axis[j]);
        int a = m->jnt_qposadr[j];
        if (m->jnt_type[j] == DUCK_JNT_HINGE) {
          double ql[4];
          axis_angle_quat(ql, m->jnt_axis[j], d->qpos[a] - m->qpos0[a]);
          quat_mul(q, q, ql);
          quat2mat(R, q);
          mulmv3(t, R, m->jnt_pos[j]);
          for (int k = 0; k < 3; k++) d->xpos[i][k] = w->xanchor[j][k] - t[k];
        } else if (m->jnt_type[j] == DUCK_JNT_SLIDE) {
          for (int k = 0; k < 3; k++) d->xpos[i][k] += w->xaxis[j][k] * (d->qpos[a] - m->qpos0[a]);
        }
      }
      memcpy(d->xquat[i], q, sizeof(q));
      quat_normalize(d->xquat[i]);
    }
    quat2mat(d->xmat[i], d->xquat[i]);
    double t[3], Ri[9];
    mulmv3(t, d->xmat[i], m->body_ipos[i]);
    for (int k = 0; k < 3; k++) d->xipos[i][k] = d->xpos[i][k] + t[k];
    quat2mat(Ri, m->body_iquat[i]);
    mulmm3(d->ximat[i], d->xmat[i], Ri);
  }
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_bodyid[s];
    double t[3], Rs[9];
    mulmv3(t, d->xmat[b], m->site_pos[s]);
    for (int k = 0; k < 3; k++) d->site_xpos[s][k] = d->xpos[b][k] + t[k];
    quat_mul(w->site_xquat[s], d->xquat[b], m->site_quat[s]);
    quat_normalize(w->site_xquat[s]);
    quat2mat(Rs, m->site_quat[s]);
    mulmm3(d->site_xmat[s], d->xmat[b], Rs);
  }
  for (int g = 0; g < m->ngeom; g++) {
    int b = m->geom_bodyid[g];
    double t[3], Rg[9];
    mulmv3(t, d->xmat[b], m->geom_pos[g]);
    for (int k = 0; k < 3; k++) d->geom_xpos[g][k] = d->xpos[b][k] + t[k];
    quat2mat(Rg, m->geom_quat[g]);
    mulmm3(d->geom_xmat[g], d->xmat[b], Rg);
  }
}

/* mj_comPos (smooth.com_pos): subtree coms, com-based inertias, motion dofs */
static void com_pos(const oracle_model* m, oracle_data* d, fwd_ws* w) {
  double msum[DUCK_MAXBODY], acc[DUCK_MAXBODY][3];
  for (int i = 0; i < m->nbody; i++) {
    msum[i] = m->body_mass[i];
    for (int k = 0; k < 3; k++) acc[i][k] = m->body_mass[i] * d->xipos[i][k];
  }
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    msum[p] += msum[i];
    for (int k = 0; k < 3; k++) acc[p][k] += acc[i][k];
  }
  for (int i = 0; i < m->nbody; i++)
    for (int k = 0; k < 3; k++) w->subtree_com[i][k] = fabs(msum[i]) > MINVAL ? acc[i][k] / msum[i] : d->xipos[i][k];
  for (int i = 1; i < m->nbody; i++) {
    const double* c = w->subtree_com[m->body_rootid[i]];
    double dif[3] = {d->xipos[i][0] - c[0], d->xipos[i][1] - c[1], d->xipos[i][2] - c[2]};
    const double* R = d->ximat[i];
    const double* I = m->body_inertia[i];
    double mass = m->body_mass[i];
    double rot[9];
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++)
        rot[3 * a + b] = R[3 * a] * I[0] * R[3 * b] + R[3 * a + 1] * I[1] * R[3 * b + 1] + R[3 * a + 2] * I[2] * R[3 * b + 2];
    double dd = dot3(dif, dif);
    double* ci = w->cinert[i];
    ci[0] = rot[0] + mass * (dd - dif[0] * dif[0]);
    ci[1] = rot[4] + mass * (dd - dif[1] * dif[1]);
    ci[2] = rot[8] + mass * (dd - dif[2] * dif[2]);
    ci[3] = rot[1] - mass * dif[0] * dif[1];
    ci[4] = rot[2] - mass * dif[0] * dif[2];
    ci[5] = rot[5] - mass * dif[1] * dif[2];
    ci[6] = mass * dif[0]; ci[7] = mass * dif[1]; ci[8] = mass * dif[2];
    ci[9] = mass;
  }
  for (int j = 0; j < m->njnt; j++) {
    int b = m->jnt_bodyid[j], da = m->jnt_dofadr[j];
    const double* c = w->subtree_com[m->body_rootid[b]];
    double off[3] = {c[0] - w->xanchor[j][0], c[1] - w->xanchor[j][1], c[2] - w->xanchor[j][2]};
    if (m->jnt_type[j] == DUCK_JNT_FREE) {
      for (int k = 0; k < 3; k++) {
        memset(w->cdof[da + k], 0, 6 * sizeof(double));
        w->cdof[da + k][3 + k] = 1;
      }
      for (int k = 0; k < 3; k++) {
        double ax[3] = {d->xmat[b][k], d->xmat[b][3 + k], d->xmat[b][6 + k]};
        memcpy(w->cdof[da + 3 + k], ax, sizeof(ax));
        cross3(w->cdof[da + 3 + k] + 3, ax, off);
      }
    } else if (m->jnt_type[j] == DUCK_JNT_HINGE) {
      memcpy(w->cdof[da], w->xaxis[j], 3 * sizeof(double));
      cross3(w->cdof[da] + 3, w->xaxis[j], off);
    } else { /* slide */
      memset(w->cdof[da], 0, 3 * sizeof(double));
      memcpy(w->cdof[da] + 3, w->xaxis[j], 3 * sizeof(double));
    }
  }
}

/* mj_crb (smooth.crb): composite inertias and joint-space mass matrix */
static void crb(const oracle_model* m, oracle_data* d, fwd_ws* w) {
  memcpy(w->crb, w->cinert, sizeof(w->crb));
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    if (p > 0)
      for (int k = 0; k < 10; k++) w->crb[p][k] += w->crb[i][k];
  }
  memset(d->qM, 0, sizeof(d->qM));
  for (int i = 0; i < m->nv; i++) {
    double buf[6];
    mul_inert_vec(buf, w->crb[m->dof_bodyid[i]], w->cdof[i]);
    for (int j = i; j >= 0; j = m->dof_parentid[j]) {
      double v = dot6(w->cdof[j], buf);
      d->qM[i][j] = v;
      d->qM[j][i] = v;
    }
    d->qM[i][i] += m->dof_armature[i];
  }
}

/* mj_comVel (smooth.com_vel) */
static void com_vel(const oracle_model* m, const oracle_data* d, fwd_ws* w) {
  memset(w->cvel[0], 0, 6 * sizeof(double));
  for (int i = 1; i < m->nbody; i++) {
    double cv[6];
    memcpy(cv, w->cvel[m->body_parentid[i]], sizeof(cv));
    int da = m->body_dofadr[i], dn = m->body_dofnum[i];
    int j = 0;
    while (j < dn) {
      int dof = da + j;
      int jt = m->jnt_type[m->dof_jntid[dof]];
      if (jt == DUCK_JNT_FREE) {
        for (int k = 0; k < 3; k++) memset(w->cdof_dot[dof + k], 0, 6 * sizeof(double));
        for (int k = 0; k < 3; k++)
          for (int c = 0; c < 6; c++) cv[c] += w->cdof[dof + k][c] * d->qvel[dof + k];
        for (int k = 3; k < 6; k++) cross_motion(w->cdof_dot[dof + k], cv, w->cdof[dof + k]);
        for (int k = 3; k < 6; k++)
          for (int c = 0; c < 6; c++) cv[c] += w->cdof[dof + k][c] * d->qvel[dof + k];
        j += 6;
      } else {
        cross_motion(w->cdof_dot[dof], cv, w->cdof[dof]);
        for (int c = 0; c < 6; c++) cv[c] += w->cdof[dof][c] * d->qvel[dof];
        j += 1;
      }
    }
    memcpy(w->cvel[i], cv, sizeof(cv));
  }
}

/* mj_rne with flg_acc = 0 (smooth.rne): Coriolis/centrifugal + gravity bias forces */
static void rne_bias(const oracle_model* m, oracle_data* d, const fwd_ws* w) {
  double cacc[DUCK_MAXBODY][6], cfrc[DUCK_MAXBODY][6];
  memset(cacc[0], 0, 6 * sizeof(double));
  for (int k = 0; k < 3; k++) cacc[0][3 + k] = -m->gravity[k];
  for (int i = 1; i < m->nbody; i++) {
    int p = m->body_parentid[i];
    memcpy(cacc[i], cacc[p], 6 * sizeof(double));
    for (int j = 0; j < m->body_dofnum[i]; j++) {
      int dof = m->body_dofadr[i] + j;
      for (int c = 0; c < 6; c++) cacc[i][c] += w->cdof_dot[dof][c] * d->qvel[dof];
    }
    double t1[6], t2[6];
    mul_inert_vec(cfrc[i], w->cinert[i], cacc[i]);
    mul_inert_vec(t1, w->cinert[i], w->cvel[i]);
    cross_force(t2, w->cvel[i], t1);
    for (int c = 0; c < 6; c++) cfrc[i][c] += t2[c];
  }
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    if (p > 0)
      for (int c = 0; c < 6; c++) cfrc[p][c] += cfrc[i][c];
  }
  for (int i = 0; i < m->nv; i++) d->qfrc_bias[i] = dot6(w->cdof[i], cfrc[m->dof_bodyid[i]]);
}

/* ------------------------------------------------------------------------------------ */
/* collision (MJX collision_driver semantics, fixed 4 slots per pair)                   */
/* ------------------------------------------------------------------------------------ */

/* argmax with a tie band: first index whose value is within tol of the maximum */
static int argmax_tol(const double* v, int n, double tol) {
  if (n <= 0) return 0;
  double mx = v[0];
  for (int i = 1; i < n; i++)
    if (v[i] > mx) mx = v[i];
  for (int i = 0; i < n; i++)
    if (v[i] >= mx - tol) return i;
  return 0;
}
#define MANIFOLD_TOL 2e-8

/* mjx collision_convex._manifold_points: 4 points of approximately maximal area; the first is
 * point a (mjx: the first masked point; the height field's prism contacts start from the deepest) */
#define MANIFOLD_MAXN 128
static void manifold_points_from(const double (*poly)[3], const int* mask, int n, const double* nrm, int a, int idx[4]) {
  if (n > MANIFOLD_MAXN) abort(); /* fixed-capacity scratch */
  double dm[MANIFOLD_MAXN] = {0}, s[2 * MANIFOLD_MAXN];
  for (int k = 0; k < n; k++) dm[k] = mask[k] ? 0.0 : -1e6;
  for (int k = 0; k < n; k++) {
    double dx = poly[a][0] - poly[k][0], dy = poly[a][1] - poly[k][1], dz = poly[a][2] - poly[k][2];
    s[k] = dx * dx + dy * dy + dz * dz + dm[k];
  }
  int b = argmax_tol(s, n, MANIFOLD_TOL);
  double ab[3], amb[3] = {poly[a][0] - poly[b][0], poly[a][1] - poly[b][1], poly[a][2] - poly[b][2]};
  cross3(ab, nrm, amb);
  for (int k = 0; k < n; k++) {
    double ap[3] = {poly[a][0] - poly[k][0], poly[a][1] - poly[k][1], poly[a][2] - poly[k][2]};
    s[k] = fabs(dot3(ap, ab)) + dm[k];
  }
  int c = argmax_tol(s, n, MANIFOLD_TOL);
  double ac[3], bc[3];
  double amc[3] = {poly[a][0] - poly[c][0], poly[a][1] - poly[c][1], poly[a][2] - poly[c][2]};
  double bmc[3] = {poly[b][0] - poly[c][0], poly[b][1] - poly[c][1], poly[b][2] - poly[c][2]};
  cross3(ac, nrm, amc);
  cross3(bc, nrm, bmc);
  for (int k = 0; k < n; k++) {
    double bp[3] = {poly[b][0] - poly[k][0], poly[b][1] - poly[k][1], poly[b][2] - poly[k][2]};
    double ap[3] = {poly[a][0] - poly[k][0], poly[a][1] - poly[k][1], poly[a][2] - poly[k][2]};
    s[k] = fabs(dot3(bp, bc)) + dm[k];
    s[n + k] = fabs(dot3(ap, ac)) + dm[k];
  }
  int dd = argmax_tol(s, 2 * n, MANIFOLD_TOL) % n;
  idx[0] = a; idx[1] = b; idx[2] = c; idx[3] = dd;
}
static void manifold_points(const double (*poly)[3], const int* mask, int n, const double* nrm, int idx[4]) {
  if (n > MANIFOLD_MAXN) abort();
  double dm[MANIFOLD_MAXN] = {0};
  for (int k = 0; k < n; k++) dm[k] = mask[k] ? 0.0 : -1e6;
  manifold_points_from(poly, mask, n, nrm, argmax_tol(dm, n, 0.0), idx);
}

/* mjx math.make_frame: rows (normal, t1, t2) */
static void make_frame(double* fr, const double* nin) {
  double n[3] = {nin[0], nin[1], nin[2]};
  double nn = norm3(n);
  if (nn > MINVAL) { n[0] /= nn; n[1] /= nn; n[2] /= nn; }
  double b[3];
  if (-0.5 < n[1] && n[1] < 0.5) { b[0] = 0; b[1] = 1; b[2] = 0; } else { b[0] = 0; b[1] = 0; b[2] = 1; }
  double nb = dot3(n, b);
  for (int k = 0; k < 3; k++) b[k] -= n[k] * nb;
  double bn = norm3(b);
  if (bn > MINVAL) { b[0] /= bn; b[1] /= bn; b[2] /= bn; }
  double c[3];
  cross3(c, n, b);
  memcpy(fr, n, 3 * sizeof(double)); memcpy(fr + 3, b, 3 * sizeof(double)); memcpy(fr + 6, c, 3 * sizeof(double));
}

static void set_inactive(oracle_data* d, int slot, int g1, int g2) {
  d->con_dist[slot] = 1.0;
  d->con_geom1[slot] = g1; d->con_geom2[slot] = g2;
  memset(d->con_pos[slot], 0, 3 * sizeof(double));
  double n[3] = {0, 0, 1};
  make_frame(d->con_frame[slot], n);
}

/* plane (geom g1) vs convex hull (geom g2): mjx collision_convex plane_convex */
static void collide_plane_convex(const oracle_model* m, oracle_data* d, int g1, int g2, int slot0) {
  const double* pp = d->geom_xpos[g1];
  const double* PR = d->geom_xmat[g1];
  const double* cp = d->geom_xpos[g2];
  const double* CR = d->geom_xmat[g2];
  double n[3] = {PR[2], PR[5], PR[8]};
  double dif[3] = {pp[0] - cp[0], pp[1] - cp[1], pp[2] - cp[2]};
  double plane_local[3], n_local[3];
  mulmtv3(plane_local, CR, dif);
  mulmtv3(n_local, CR, n);
  int nv = m->hull_nvert;
  double support[DUCK_MAXHULLV];
  double smax = -1e30;
  for (int k = 0; k < nv; k++) {
    double t[3] = {plane_local[0] - m->hull_vert[k][0], plane_local[1] - m->hull_vert[k][1],
                   plane_local[2] - m->hull_vert[k][2]};
    support[k] = dot3(t, n_local);
    if (support[k] > smax) smax = support[k];
  }
  double thr = smax - 1e-3 > 0 ? smax - 1e-3 : 0;
  int mask[DUCK_MAXHULLV];
  for (int k = 0; k < nv; k++) mask[k] = support[k] > thr;
  int idx[4];
  manifold_points((const double(*)[3])m->hull_vert, mask, nv, n_local, idx);
  double fr[9];
  make_frame(fr, n);
  for (int c = 0; c < 4; c++) {
    int k = idx[c], unique = 1;
    for (int e = 0; e < c; e++)
      if (idx[e] == k) unique = 0;
    double dist = unique ? -support[k] : 1.0;
    double vw[3];
    mulmv3(vw, CR, m->hull_vert[k]);
    int s = slot0 + c;
    for (int a = 0; a < 3; a++) d->con_pos[s][a] = cp[a] + vw[a] - 0.5 * dist * n[a];
    d->con_dist[s] = dist;
    memcpy(d->con_frame[s], fr, sizeof(fr));
    d->con_geom1[s] = g1; d->con_geom2[s] = g2;
  }
}

/* ------------------------------------------------------------------------------------ */
/* height field vs convex hull: MuJoCo's prism decomposition                             */
/* ------------------------------------------------------------------------------------ */
/* MuJoCo mjc_ConvexHField (engine_collision_convex.c), which MJX's hfield collision follows:
 *  - the hull's bounding box in the height field's frame (its extreme vertices along +-x, +-y,
 *    +-z) is tested against the field's box [-sx, sx] x [-sy, sy] x [-size[3], size[2]];
 *  - the sub-grid: vertex columns cmin = floor((xmin + sx) / (2 sx) (ncol - 1)), cmax = ceil(..)
 *    clamped to [0, ncol - 1]; rows rmin / rmax likewise;
 *  - each row r in [rmin, rmax) is walked as a triangle strip over the vertices (c, r), (c, r + 1),
 *    c = cmin .. cmax (addVert): every three consecutive vertices are the top of a prism whose
 *    bottom is at z = -size[3]; cell (c, r) thus holds the triangles
 *    A = {(c, r), (c, r + 1), (c + 1, r)} and B = {(c, r + 1), (c + 1, r), (c + 1, r + 1)}
 *    (the cell's (c, r + 1)-(c + 1, r) diagonal);
 *  - the prism height test: a prism whose three top vertices are all below the hull's lowest
 *    point is skipped;
 *  - every other prism is collided with the hull as a convex-convex pair, one contact per prism.
 * Restated with an exact penetration depth in place of libccd's MPR estimate: the minimum over
 * the faces of the Minkowski difference P - H of its support function (separating-axis test over
 * the prism's 5 face normals, the hull's face normals and the edge pairs whose Gauss-map arcs
 * cross -- Gregorius, GDC 2013), and MJX's fixed DUCK_CON_PER_PAIR slots per pair, filled from the
 * prism contacts by MJX's _manifold_points starting at the deepest (within HF_DEPTH_TIE). Declared choices (DESIGN.md
 * §5 item 6): equal overlaps resolve to the first axis in the order prism top, sides, bottom, hull
 * faces, top-edge pairs, vertical-edge pairs, bottom-edge pairs; the contact point of a prism
 * is the penetration-weighted centroid of the vertices of each shape inside the other, or, when no
 * vertex is inside (crossing edges), the midpoint of the two shapes' support features (the centroid
 * of each shape's vertices within HF_WITNESS_BAND of its support plane along the normal, weighted 1
 * at the plane to 0 at the band edge; the prism's top vertices only). */
#define HF_WITNESS_BAND 1e-3 /* m; = TPhys HF_WITNESS_BAND */
#define HF_POINT_BAND 1e-4   /* m; test aid only (oracle_set_hf_band_scale): round 4's "point band", see below */
#define HF_DEPTH_TIE 1e-6    /* m; = TPhys HF_DEPTH_TIE: prisms sharing a grid vertex or edge often tie exactly */
#define HF_MAXPRISM 128      /* prisms under one hull (the sub-grid of a 0.11 m foot: <= 18) */

/* test aid: how often each class of separating axis gave a prism's penetration (oracle_hfield_axis_wins) */
static long long hf_axis_wins[14];
void oracle_hfield_axis_wins(long long out[14], int reset) {
  for (int i = 0; i < 14; i++) { out[i] = hf_axis_wins[i]; if (reset) hf_axis_wins[i] = 0; }
}


/* test aid (oracle_set_hf_tie_last): a prism's overlaps within this band of the minimum resolve to the
 * LAST such axis of the priority order (0, default: the first, the declared rule). The band is the
 * kernel's fp32 error bound on an overlap (hull coordinates ~0.3 m from the mesh origin, ~20
 * operations: a few 1e-7 m): two axes that close are tied at the kernel's precision, and its fp32
 * overlaps may order them the other way (teacher forcing's "sat_tie" rule). */
static _Thread_local double g_hf_tie_last;
void oracle_set_hf_tie_last(double band) { g_hf_tie_last = band; }
/* test aid (oracle_set_hf_tie_first): the FIRST axis of the priority order whose overlap is within this
 * band of the minimum (0, default: the minimum itself). The mirror case of tie_last: the fp64 minimum is
 * a later axis by less than the band, the kernel's fp32 overlaps put an earlier one at or below it. */
static _Thread_local double g_hf_tie_first;
void oracle_set_hf_tie_first(double band) { g_hf_tie_first = band; }

/* test aid (oracle_set_hf_band_scale): with s > 0 a prism contact whose total penetration weight W
 * is below s * HF_POINT_BAND moves towards the support midpoint (pos = C / band + (1 - W / band) mid),
 * round 4's "point band" for onset prisms. Default 0: the declared rule (the plain weighted centroid),
 * which the kernel computes; the band made fp32 and fp64 disagree 2-3x as often
 * and now serves as a contact-generation-only injected defect (teacher_forcing.DEFECTS) and for
 * tools/hfield_deviation.py. Process-wide, not thread-local: the batched entry points run envs on
 * OpenMP workers, which must all see it. */
static double g_hf_band_scale = 0.0;
void oracle_set_hf_band_scale(double s) { g_hf_band_scale = s; }
double oracle_get_hf_band_scale(void) { return g_hf_band_scale; }

/* test aids: injected contact-generation defects for the teacher-forcing classifier's teeth
 * (teacher_forcing.DEFECTS; the kernel keeps the declared rules): which = 0 the point band scale
 * (above), 1 a scale of HF_WITNESS_BAND, 2 a scale of HF_DEPTH_TIE, 3 the rank of the prism contact
 * the 4-slot manifold starts from (0: the deepest, the declared rule; 1: the second deepest).
 * Process-wide, like the band scale. */
static double g_hf_witness_scale = 1.0, g_hf_depth_tie_scale = 1.0;
static int g_hf_manifold_start = 0;
void oracle_set_hf_defect(int which, double v) {
  if (which == 0) g_hf_band_scale = v;
  else if (which == 1) g_hf_witness_scale = v;
  else if (which == 2) g_hf_depth_tie_scale = v;
  else if (which == 3) g_hf_manifold_start = (int)v;
}
double oracle_get_hf_defect(int which) {
  return which == 0 ? g_hf_band_scale
                    : (which == 1 ? g_hf_witness_scale : (which == 2 ? g_hf_depth_tie_scale : (double)g_hf_manifold_start));
}

/* the hull in the local frame (the height field's axes, origin at the hull's frame) */
typedef struct {
  int nv, nf, ne;
  double V[DUCK_MAXHULLV][3], FN[DUCK_MAXHULLF][3];
} hf_hull;

/* support values over a point set */
static double pts_min(const double* u, const double (*P)[3], int n) {
  double v = 1e300;
  for (int i = 0; i < n; i++) v = fmin(v, dot3(u, P[i]));
  return v;
}
static double pts_max(const double* u, const double (*P)[3], int n) {
  double v = -1e300;
  for (int i = 0; i < n; i++) v = fmax(v, dot3(u, P[i]));
  return v;
}

/* the prism's outward face normals: top nt (z > 0), side k through top edge T_k -> T_{k+1} */
static void prism_normals(const double T[3][3], double nt[3], double s[3][3]) {
  double e0[3], e1[3];
  for (int a = 0; a < 3; a++) { e0[a] = T[1][a] - T[0][a]; e1[a] = T[2][a] - T[0][a]; }
  cross3(nt, e0, e1);
  const double nn = norm3(nt), sg = nt[2] < 0 ? -1.0 : 1.0;
  for (int a = 0; a < 3; a++) nt[a] *= sg / nn;
  for (int k = 0; k < 3; k++) {
    const double* p = T[k];
    const double* q = T[(k + 1) % 3];
    const double* o = T[(k + 2) % 3];
    double sx = q[1] - p[1], sy = -(q[0] - p[0]);
    const double l = sqrt(sx * sx + sy * sy);
    sx /= l; sy /= l;
    if (sx * (o[0] - p[0]) + sy * (o[1] - p[1]) > 0) { sx = -sx; sy = -sy; }
    s[k][0] = sx; s[k][1] = sy; s[k][2] = 0.0;
  }
}

/* Gregorius' Minkowski-face test: do the Gauss-map arcs (A, B) of one polytope's edge and
 * (C, D) of the other's negated edge cross? */
static int minkowski_face(const double* A, const double* B, const double* C, const double* D) {
  double BxA[3], DxC[3];
  cross3(BxA, B, A);
  cross3(DxC, D, C);
  const double CBA = dot3(C, BxA), DBA = dot3(D, BxA), ADC = dot3(A, DxC), BDC = dot3(B, DxC);
  return CBA * DBA < 0 && ADC * BDC < 0 && CBA * BDC > 0;
}

/* one prism (top vertices T, bottom at z = base, local frame) against the hull: exact
 * penetration depth, contact normal u (pushes the hull out of the prism) and point. Returns 0
 * when the shapes do not overlap. */
static int hf_prism_contact(const oracle_model* m, const hf_hull* H, const double T[3][3], double base, double* depth,
                            double u_out[3], double pos[3]) {
  double P[6][3], nt[3], s[3][3];
  for (int k = 0; k < 3; k++) {
    memcpy(P[k], T[k], sizeof(double) * 3);
    P[k + 3][0] = T[k][0]; P[k + 3][1] = T[k][1]; P[k + 3][2] = base;
  }
  prism_normals(T, nt, s);
  /* candidate axes in priority order */
  enum { NAX = 5 + DUCK_MAXHULLF + 9 * DUCK_MAXHULLE };
  double ax[NAX][3], ov[NAX];
  int kind_of_axis[NAX];
  int na = 0;
  memcpy(ax[na++], nt, sizeof(nt));
  for (int k = 0; k < 3; k++) memcpy(ax[na++], s[k], sizeof(double) * 3);
  ax[na][0] = 0; ax[na][1] = 0; ax[na][2] = -1; na++;
  for (int f = 0; f < H->nf; f++)
    for (int a = 0; a < 3; a++) ax[na + f][a] = -H->FN[f][a];
  na += H->nf;
  /* edge pairs, in the order top edges (hull edge e, prism top edge k), vertical edges (e, k),
   * bottom edges (e, k): prism top edge k (T_k, T_k+1; faces nt, s_k), vertical edge k (at
   * vertex k; faces s_k-1, s_k), bottom edge k (faces -z, s_k) */
  const double mz[3] = {0, 0, -1};
  for (int kind = 0; kind < 3; kind++)
    for (int e = 0; e < H->ne; e++) {
      const int v0 = m->hull_edge[e][0], v1 = m->hull_edge[e][1];
      const double *nA = H->FN[m->hull_edge_face[e][0]], *nB = H->FN[m->hull_edge_face[e][1]];
      const double C[3] = {-nA[0], -nA[1], -nA[2]}, D[3] = {-nB[0], -nB[1], -nB[2]};
      double eh[3];
      for (int a = 0; a < 3; a++) eh[a] = H->V[v1][a] - H->V[v0][a];
      for (int k = 0; k < 3; k++) {
        const double *fa, *fb;
        double ep[3];
        if (kind == 0) {
          fa = nt; fb = s[k];
          for (int a = 0; a < 3; a++) ep[a] = T[(k + 1) % 3][a] - T[k][a];
        } else if (kind == 1) {
          fa = s[(k + 2) % 3]; fb = s[k];
          ep[0] = 0; ep[1] = 0; ep[2] = 1;
        } else {
          fa = mz; fb = s[k];
          for (int a = 0; a < 2; a++) ep[a] = T[(k + 1) % 3][a] - T[k][a];
          ep[2] = 0;
        }
        if (!minkowski_face(fa, fb, C, D)) continue;
        double u[3];
        cross3(u, eh, ep);
        const double un = norm3(u);
        if (un < 1e-6 * norm3(eh) * norm3(ep)) continue;
        const double sg = (dot3(u, fa) + dot3(u, fb)) < 0 ? -1.0 : 1.0;
        for (int a = 0; a < 3; a++) ax[na][a] = sg * u[a] / un;
        kind_of_axis[na] = kind;
        na++;
      }
    }
  double mn = 1e300;
  for (int i = 0; i < na; i++) {
    ov[i] = pts_max(ax[i], (const double(*)[3])P, 6) - pts_min(ax[i], (const double(*)[3])H->V, H->nv);
    mn = fmin(mn, ov[i]);
  }
  if (!(mn > 0)) {
    /* separated: which class of axis separates, when the prism's own faces do not (kernel screen) */
    int cheap = 1;
    for (int i = 0; i < 5; i++) cheap &= ov[i] > 0;
    if (cheap) {
      int w = 0;
      while (ov[w] > mn) w++;
      int cls = w < 5 + H->nf ? 3 : 4 + kind_of_axis[w];
#ifdef _OPENMP
#pragma omp atomic
#endif
      hf_axis_wins[7 + cls]++;
    }
    return 0;
  }
  int w = 0;
  while (w < na - 1 && ov[w] > mn + g_hf_tie_first) w++; /* (g_hf_tie_first: test aid, 0 by default) */
  if (g_hf_tie_last > 0) /* test aid: the last axis within the tie band instead of the first */
    for (int i = 0; i < na; i++)
      if (ov[i] <= mn + g_hf_tie_last) w = i;
  {
    /* which class of axis won (hf_axis_wins: prism top, sides, bottom, hull faces, top-edge,
     * vertical-edge, bottom-edge pairs) */
    int cls = w == 0 ? 0 : (w < 4 ? 1 : (w == 4 ? 2 : (w < 5 + H->nf ? 3 : 4)));
    if (cls == 4) cls = 4 + kind_of_axis[w];
#ifdef _OPENMP
#pragma omp atomic
#endif
    hf_axis_wins[cls]++;
  }
  const double* u = ax[w];
  /* the contact point: the centroid of the vertices of each shape inside the other (hull vertices
   * inside the prism, prism top vertices inside the hull), each weighted by its penetration (distance
   * to the nearest face of the other shape); the midpoint of the two shapes' support features along u
   * when no vertex is inside (crossing edges). (Test aid: with the band scale > 0, a weight W below
   * the band blends towards that midpoint, C / band + (1 - W / band) mid.) */
  double wsum = 0, c[3] = {0, 0, 0};
  const double ptop = dot3(nt, T[0]);
  for (int k = 0; k < H->nv; k++) {
    const double* v = H->V[k];
    double pen = fmin(ptop - dot3(nt, v), v[2] - base);
    for (int j = 0; j < 3; j++) pen = fmin(pen, s[j][0] * (T[j][0] - v[0]) + s[j][1] * (T[j][1] - v[1]));
    if (pen > 0) { wsum += pen; for (int a = 0; a < 3; a++) c[a] += pen * v[a]; }
  }
  for (int j = 0; j < 3; j++) {
    double pen = 1e300;
    for (int f = 0; f < H->nf; f++) pen = fmin(pen, m->hull_face_offset[f] - dot3(H->FN[f], T[j]));
    if (pen > 0) { wsum += pen; for (int a = 0; a < 3; a++) c[a] += pen * T[j][a]; }
  }
  const double pband = HF_POINT_BAND * g_hf_band_scale;
  if (wsum > 0 && wsum >= pband) {
    for (int a = 0; a < 3; a++) pos[a] = c[a] / wsum;
  } else {
    const double hmin = pts_min(u, (const double(*)[3])H->V, H->nv), pmax = pts_max(u, T, 3);
    double wh = 0, wp = 0, ch[3] = {0, 0, 0}, cp[3] = {0, 0, 0};
    for (int k = 0; k < H->nv; k++) {
      const double wk = fmax(0.0, 1.0 - (dot3(u, H->V[k]) - hmin) / (HF_WITNESS_BAND * g_hf_witness_scale));
      wh += wk;
      for (int a = 0; a < 3; a++) ch[a] += wk * H->V[k][a];
    }
    for (int k = 0; k < 3; k++) {
      const double wk = fmax(0.0, 1.0 - (pmax - dot3(u, T[k])) / (HF_WITNESS_BAND * g_hf_witness_scale));
      wp += wk;
      for (int a = 0; a < 3; a++) cp[a] += wk * T[k][a];
    }
    /* (wsum == 0 when the band is off: the midpoint alone) */
    const double f = pband > 0 ? 1.0 - wsum / pband : 1.0;
    for (int a = 0; a < 3; a++) pos[a] = (pband > 0 ? c[a] / pband : 0.0) + f * 0.5 * (ch[a] / wh + cp[a] / wp);
  }
  memcpy(u_out, u, sizeof(double) * 3);
  *depth = mn;
  return 1;
}

/* the hull in the height field's local frame; its bounding box in the hfield frame; the
 * sub-grid. Returns 0 when the box misses the field. */
typedef struct {
  double R[9], t[3];  /* hull frame -> hfield frame: x_hf = R v + t */
  double zmin;
  int cmin, cmax, rmin, rmax;
} hf_frame;

static int hf_setup(const oracle_model* m, const oracle_data* d, int g_hf, int g_cvx, hf_hull* H, hf_frame* F) {
  const double *hp = d->geom_xpos[g_hf], *HR = d->geom_xmat[g_hf], *cp = d->geom_xpos[g_cvx], *CR = d->geom_xmat[g_cvx];
  for (int a = 0; a < 3; a++)
    for (int b = 0; b < 3; b++) F->R[3 * a + b] = HR[a] * CR[b] + HR[3 + a] * CR[3 + b] + HR[6 + a] * CR[6 + b];
  const double off[3] = {cp[0] - hp[0], cp[1] - hp[1], cp[2] - hp[2]};
  mulmtv3(F->t, HR, off);
  H->nv = m->hull_nvert; H->nf = m->hull_nface; H->ne = m->hull_nedge;
  double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
  for (int k = 0; k < H->nv; k++) {
    mulmv3(H->V[k], F->R, m->hull_vert[k]);
    for (int a = 0; a < 3; a++) {
      lo[a] = fmin(lo[a], H->V[k][a] + F->t[a]);
      hi[a] = fmax(hi[a], H->V[k][a] + F->t[a]);
    }
  }
  for (int f = 0; f < H->nf; f++) mulmv3(H->FN[f], F->R, m->hull_face_normal[f]);
  const double *sz = m->hfield_size;
  const int nr = m->hfield_nrow, nc = m->hfield_ncol;
  F->zmin = lo[2];
  if (hi[0] < -sz[0] || lo[0] > sz[0] || hi[1] < -sz[1] || lo[1] > sz[1] || lo[2] > sz[2] || hi[2] < -sz[3])
    return 0;
  F->cmin = (int)floor((lo[0] + sz[0]) / (2 * sz[0]) * (nc - 1));
  F->cmax = (int)ceil((hi[0] + sz[0]) / (2 * sz[0]) * (nc - 1));
  F->rmin = (int)floor((lo[1] + sz[1]) / (2 * sz[1]) * (nr - 1));
  F->rmax = (int)ceil((hi[1] + sz[1]) / (2 * sz[1]) * (nr - 1));
  F->cmin = F->cmin < 0 ? 0 : F->cmin;
  F->cmax = F->cmax > nc - 1 ? nc - 1 : F->cmax;
  F->rmin = F->rmin < 0 ? 0 : F->rmin;
  F->rmax = F->rmax > nr - 1 ? nr - 1 : F->rmax;
  return 1;
}

/* top vertices of strip prism (r, c, tri) in the local frame; returns 0 when the prism height
 * test skips it */
static int hf_prism_top(const oracle_model* m, const hf_frame* F, int r, int c, int tri, double T[3][3]) {
  static const int cc[2][3][2] = {{{0, 0}, {0, 1}, {1, 0}}, {{0, 1}, {1, 0}, {1, 1}}}; /* (dc, dr) */
  const double* sz = m->hfield_size;
  const int nr = m->hfield_nrow, nc = m->hfield_ncol;
  int below = 0;
  for (int k = 0; k < 3; k++) {
    const int ci = c + cc[tri][k][0], ri = r + cc[tri][k][1];
    const double x = sz[0] * (2.0 * ci / (nc - 1) - 1.0), y = sz[1] * (2.0 * ri / (nr - 1) - 1.0);
    const double z = sz[2] * m->hfield_data[ri * nc + ci];
    below += z < F->zmin;
    T[k][0] = x - F->t[0]; T[k][1] = y - F->t[1]; T[k][2] = z - F->t[2];
  }
  return below < 3;
}

/* height field (g1) vs convex hull (g2): the DUCK_CON_PER_PAIR deepest prism contacts */
/* every penetrating prism's contact (depth, normal, point; the hull frame F.t-relative field axes), in
 * strip order; returns their number (0 when the hull misses the field) */
static int hf_contacts(const oracle_model* m, const oracle_data* d, int g1, int g2, hf_frame* F,
                       double dep[HF_MAXPRISM], double nrm[HF_MAXPRISM][3], double pt[HF_MAXPRISM][3]) {
  hf_hull H;
  if (!hf_setup(m, d, g1, g2, &H, F)) return 0;
  int n = 0;
  const double base = -m->hfield_size[3] - F->t[2];
  for (int r = F->rmin; r < F->rmax; r++)
    for (int c = F->cmin; c < F->cmax; c++)
      for (int tri = 0; tri < 2; tri++) {
        double T[3][3];
        if (!hf_prism_top(m, F, r, c, tri, T)) continue;
        if (n >= HF_MAXPRISM) abort(); /* the fixed-capacity list: never reached by a foot-sized hull */
        if (hf_prism_contact(m, &H, (const double(*)[3])T, base, &dep[n], nrm[n], pt[n])) n++;
      }
  return n;
}

/* test aid: the prism contacts of height field g_hf vs hull g_cvx before the manifold selection (the
 * candidates the 4 slots are chosen from), world frame: depth[i] > 0, unit normal (pushes the hull
 * out), point. Returns their number (at most max). d must hold the kinematics (oracle_forward). */
int oracle_hfield_contacts(const oracle_model* m, const oracle_data* d, int g_hf, int g_cvx, int max, double* depth,
                           double* normal, double* point) {
  if (!m->hfield_data) return 0;
  hf_frame F;
  double dep[HF_MAXPRISM], nrm[HF_MAXPRISM][3], pt[HF_MAXPRISM][3];
  const int n = hf_contacts(m, d, g_hf, g_cvx, &F, dep, nrm, pt);
  const double *hp = d->geom_xpos[g_hf], *HR = d->geom_xmat[g_hf];
  int k = 0;
  for (int i = 0; i < n && k < max; i++, k++) {
    double pl[3];
    for (int q = 0; q < 3; q++) pl[q] = pt[i][q] + F.t[q];
    mulmv3(point + 3 * k, HR, pl);
    for (int q = 0; q < 3; q++) point[3 * k + q] += hp[q];
    mulmv3(normal + 3 * k, HR, nrm[i]);
    depth[k] = dep[i];
  }
  return k;
}

/* the 4 slots' prism contacts (indices into the candidates, strip order): mjx's _manifold_points over
 * their points, from the deepest (the first in strip order within HF_DEPTH_TIE of the deepest: prisms
 * that share a grid vertex or edge often reach the same depth through it), areas taken in the plane of
 * its normal. Frame-free (differences and cross products only). */
static void hf_select(const double* dep, const double (*pt)[3], const double (*nrm)[3], int n, int idx[4]) {
  double dmax = dep[0];
  for (int i = 1; i < n; i++) dmax = fmax(dmax, dep[i]);
  int a = 0;
  while (dep[a] < dmax - HF_DEPTH_TIE * g_hf_depth_tie_scale) a++;
  if (g_hf_manifold_start == 1 && n > 1) { /* test aid (injected defect): the second deepest */
    int b = a == 0 ? 1 : 0;
    for (int i = 0; i < n; i++)
      if (i != a && dep[i] > dep[b]) b = i;
    a = b;
  }
  int mask[HF_MAXPRISM];
  for (int i = 0; i < n; i++) mask[i] = 1;
  manifold_points_from(pt, mask, n, nrm[a], a, idx);
}

/* test aid: hf_select over caller-given candidates (n <= 128; depth [n], point [n][3], normal [n][3],
 * any one frame): the teacher-forcing selection rules replay the oracle's own choice under fp32 noise */
int oracle_hfield_select(const double* depth, const double* point, const double* normal, int n, int idx[4]) {
  if (n < 1 || n > HF_MAXPRISM) return -1;
  hf_select(depth, (const double(*)[3])point, (const double(*)[3])normal, n, idx);
  return 0;
}

static void collide_hfield_convex(const oracle_model* m, oracle_data* d, int g1, int g2, int slot0) {
  for (int c = 0; c < DUCK_CON_PER_PAIR; c++) set_inactive(d, slot0 + c, g1, g2);
  hf_frame F;
  double dep[HF_MAXPRISM], nrm[HF_MAXPRISM][3], pt[HF_MAXPRISM][3];
  const int n = hf_contacts(m, d, g1, g2, &F, dep, nrm, pt);
  if (n == 0) return;
  /* 4 of the prism contacts (hf_select); repeats stay inactive (plane_convex's rule) */
  int idx[4];
  hf_select(dep, (const double(*)[3])pt, (const double(*)[3])nrm, n, idx);
  const double *hp = d->geom_xpos[g1], *HR = d->geom_xmat[g1];
  for (int s = 0; s < DUCK_CON_PER_PAIR; s++) {
    const int b = idx[s];
    int unique = 1;
    for (int e = 0; e < s; e++)
      if (idx[e] == b) unique = 0;
    double pl[3], nw[3];
    for (int q = 0; q < 3; q++) pl[q] = pt[b][q] + F.t[q];
    mulmv3(d->con_pos[slot0 + s], HR, pl);
    for (int q = 0; q < 3; q++) d->con_pos[slot0 + s][q] += hp[q];
    mulmv3(nw, HR, nrm[b]);
    make_frame(d->con_frame[slot0 + s], nw);
    d->con_dist[slot0 + s] = unique ? -dep[b] : 1.0;
  }
}

/* Brute-force reference for the prism decomposition (tools/hfield_deviation.py, tests): the same
 * sub-grid, strip and height test, and for every prism the separating-axis minimum over ALL
 * axes -- the 5 prism faces, every hull face, every hull edge x prism edge direction, no
 * Minkowski-face filter and no tie rule -- with its unit normal (pushes the hull out, world
 * frame), the deepest hull vertex along it (world) and the prism's strip index. Returns the
 * number of penetrating prisms written (at most max). */
int oracle_hfield_prisms(const oracle_model* m, const oracle_data* d, int g_hf, int g_cvx, int max, double* depth,
                         double* normal, double* point, int* index) {
  if (!m->hfield_data) return 0;
  hf_hull H;
  hf_frame F;
  if (!hf_setup(m, d, g_hf, g_cvx, &H, &F)) return 0;
  const double *hp = d->geom_xpos[g_hf], *HR = d->geom_xmat[g_hf];
  const double base = -m->hfield_size[3] - F.t[2];
  int n = 0, idx = 0;
  for (int r = F.rmin; r < F.rmax; r++)
    for (int c = F.cmin; c < F.cmax; c++)
      for (int tri = 0; tri < 2; tri++, idx++) {
        double T[3][3], P[6][3], nt[3], s[3][3];
        if (!hf_prism_top(m, &F, r, c, tri, T)) continue;
        for (int k = 0; k < 3; k++) {
          memcpy(P[k], T[k], sizeof(double) * 3);
          P[k + 3][0] = T[k][0]; P[k + 3][1] = T[k][1]; P[k + 3][2] = base;
        }
        prism_normals((const double(*)[3])T, nt, s);
        double pe[9][3];
        for (int k = 0; k < 3; k++) {
          for (int a = 0; a < 3; a++) pe[k][a] = T[(k + 1) % 3][a] - T[k][a];
          pe[3 + k][0] = 0; pe[3 + k][1] = 0; pe[3 + k][2] = 1;
          pe[6 + k][0] = pe[k][0]; pe[6 + k][1] = pe[k][1]; pe[6 + k][2] = 0;
        }
        double best = 1e300, bu[3] = {0, 0, 1};
        int sep = 0;
        const int naxes = 5 + H.nf + 9 * H.ne;
        for (int i = 0; i < naxes && !sep; i++) {
          double u[3];
          if (i == 0) memcpy(u, nt, sizeof(u));
          else if (i < 4) memcpy(u, s[i - 1], sizeof(u));
          else if (i == 4) { u[0] = 0; u[1] = 0; u[2] = -1; }
          else if (i < 5 + H.nf) for (int a = 0; a < 3; a++) u[a] = -H.FN[i - 5][a];
          else {
            const int q = i - 5 - H.nf, e = q / 9, k = q % 9;
            double eh[3];
            for (int a = 0; a < 3; a++) eh[a] = H.V[m->hull_edge[e][1]][a] - H.V[m->hull_edge[e][0]][a];
            cross3(u, eh, pe[k]);
            const double un = norm3(u);
            if (un < 1e-9 * norm3(eh) * norm3(pe[k])) continue;
            for (int a = 0; a < 3; a++) u[a] /= un;
          }
          /* both directions of an edge axis; faces are outward already */
          for (int sgn = 0; sgn < (i >= 5 + H.nf ? 2 : 1); sgn++) {
            if (sgn) for (int a = 0; a < 3; a++) u[a] = -u[a];
            const double o = pts_max(u, (const double(*)[3])P, 6) - pts_min(u, (const double(*)[3])H.V, H.nv);
            if (o <= 0) { sep = 1; break; }
            if (o < best) { best = o; memcpy(bu, u, sizeof(bu)); }
          }
        }
        if (sep) continue;
        if (n >= max) return n;
        int kd = 0;
        for (int k = 1; k < H.nv; k++)
          if (dot3(H.V[k], bu) < dot3(H.V[kd], bu)) kd = k;
        depth[n] = best;
        mulmv3(normal + 3 * n, HR, bu);
        double pl[3];
        for (int a = 0; a < 3; a++) pl[a] = H.V[kd][a] + F.t[a];
        mulmv3(point + 3 * n, HR, pl);
        for (int a = 0; a < 3; a++) point[3 * n + a] += hp[a];
        index[n] = idx;
        n++;
      }
  return n;
}

/* convex hull (g1) vs convex hull (g2): separating-axis test over face normals and edge
 * pairs; on overlap, mjx's clipped 4-point manifold on the reference face, or one edge-edge
 * point (mjx collision_convex: SAT over the Gauss map, then _clip + _manifold_points). */
static void collide_convex_convex(const oracle_model* m, oracle_data* d, int g1, int g2, int slot0) {
  for (int c = 0; c < 4; c++) set_inactive(d, slot0 + c, g1, g2);
  const double *p1 = d->geom_xpos[g1], *R1 = d->geom_xmat[g1], *p2 = d->geom_xpos[g2], *R2 = d->geom_xmat[g2];
  double c1[3], c2[3], t[3];
  mulmv3(t, R1, m->hull_center);
  for (int a = 0; a < 3; a++) c1[a] = p1[a] + t[a];
  mulmv3(t, R2, m->hull_center);
  for (int a = 0; a < 3; a++) c2[a] = p2[a] + t[a];
  double cc[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
  if (norm3(cc) > 2 * m->hull_radius) return;
  int nv = m->hull_nvert;
  double V1[DUCK_MAXHULLV][3], V2[DUCK_MAXHULLV][3];
  for (int k = 0; k < nv; k++) {
    mulmv3(t, R1, m->hull_vert[k]);
    for (int a = 0; a < 3; a++) V1[k][a] = p1[a] + t[a];
    mulmv3(t, R2, m->hull_vert[k]);
    for (int a = 0; a < 3; a++) V2[k][a] = p2[a] + t[a];
  }
  /* best axis: max separation; type 0 = face of 1, 1 = face of 2, 2 = edge pair. Near-equal
   * axes (parallel faces of the two feet, an edge axis equal to a face normal) differ only by
   * rounding, so the choice among them uses a tolerance the fp32 kernel resolves the same way:
   * the lowest-index face within DUCK_HULL_SAT_TIE of the best face; an edge pair only when it
   * beats that face by more than the tolerance (codegen.HULL_SAT_TIE, TPhys::collide_hulls_team). */
  const int nf = m->hull_nface;
  double FN[2 * DUCK_MAXHULLF][3], fsep[2 * DUCK_MAXHULLF], ftop = -1e30;
  for (int a = 0; a < 2 * nf; a++) {
    const int side = a / nf, f = a - side * nf;
    mulmv3(FN[a], side == 0 ? R1 : R2, m->hull_face_normal[f]);
    if (side == 1) { FN[a][0] = -FN[a][0]; FN[a][1] = -FN[a][1]; FN[a][2] = -FN[a][2]; }
    double mx1 = -1e30, mn2 = 1e30;
    for (int k = 0; k < nv; k++) {
      double a1 = dot3(FN[a], V1[k]), a2 = dot3(FN[a], V2[k]);
      if (a1 > mx1) mx1 = a1;
      if (a2 < mn2) mn2 = a2;
    }
    fsep[a] = mn2 - mx1;
    if (fsep[a] > 0) return;
    if (fsep[a] > ftop) ftop = fsep[a];
  }
  int fbest = 0;
  while (fsep[fbest] < ftop - DUCK_HULL_SAT_TIE) fbest++;
  double best = fsep[fbest], bu[3];
  memcpy(bu, FN[fbest], sizeof(bu));
  int btype = fbest / nf, bi = fbest - btype * nf, bj = -1;
  /* edge pairs: only those whose Gauss-map arcs cross (arc of edge e1 between its two face
   * normals on hull 1, arc of e2 on -hull 2: a face of the Minkowski difference; Gregorius,
   * "The Separating Axis Test between Convex Polyhedra", GDC 2013). The others are never the
   * deepest axis but can tie with it, and their closest points clamp to a segment end. */
  double emax = -1e30, eu[3] = {0, 0, 1};
  int ei = -1, ej = -1;
  for (int e1 = 0; e1 < m->hull_nedge; e1++) {
    double ea[3], eb[3], tmp[3], BxA[3];
    for (int a = 0; a < 3; a++) tmp[a] = m->hull_vert[m->hull_edge[e1][1]][a] - m->hull_vert[m->hull_edge[e1][0]][a];
    mulmv3(ea, R1, tmp);
    const double *A = FN[m->hull_edge_face[e1][0]], *B = FN[m->hull_edge_face[e1][1]];
    cross3(BxA, B, A);
    for (int e2 = 0; e2 < m->hull_nedge; e2++) {
      const double *C = FN[nf + m->hull_edge_face[e2][0]], *D = FN[nf + m->hull_edge_face[e2][1]];
      double DxC[3];
      cross3(DxC, D, C);
      const double CBA = dot3(C, BxA), DBA = dot3(D, BxA), ADC = dot3(A, DxC), BDC = dot3(B, DxC);
      if (!(CBA * DBA < 0 && ADC * BDC < 0 && CBA * BDC > 0)) continue;
      for (int a = 0; a < 3; a++) tmp[a] = m->hull_vert[m->hull_edge[e2][1]][a] - m->hull_vert[m->hull_edge[e2][0]][a];
      mulmv3(eb, R2, tmp);
      double u[3];
      cross3(u, ea, eb);
      double un = norm3(u);
      if (un < 1e-6 * norm3(ea) * norm3(eb)) continue;
      for (int a = 0; a < 3; a++) u[a] /= un;
      if (dot3(u, cc) < 0) { u[0] = -u[0]; u[1] = -u[1]; u[2] = -u[2]; }
      double mx1 = -1e30, mn2 = 1e30;
      for (int k = 0; k < nv; k++) {
        double a1 = dot3(u, V1[k]), a2 = dot3(u, V2[k]);
        if (a1 > mx1) mx1 = a1;
        if (a2 < mn2) mn2 = a2;
      }
      double sep = mn2 - mx1;
      if (sep > 0) return;
      if (sep > emax) { emax = sep; memcpy(eu, u, sizeof(u)); ei = e1; ej = e2; }
    }
  }
  if (ei >= 0 && emax > best + DUCK_HULL_SAT_TIE) { best = emax; memcpy(bu, eu, sizeof(bu)); btype = 2; bi = ei; bj = ej; }
  double fr[9];
  make_frame(fr, bu);
  if (btype == 2) {
    /* closest points of the two edge segments */
    const double *a0 = V1[m->hull_edge[bi][0]], *a1 = V1[m->hull_edge[bi][1]];
    const double *b0 = V2[m->hull_edge[bj][0]], *b1 = V2[m->hull_edge[bj][1]];
    double d1[3], d2[3], r[3];
    for (int a = 0; a < 3; a++) { d1[a] = a1[a] - a0[a]; d2[a] = b1[a] - b0[a]; r[a] = a0[a] - b0[a]; }
    double A = dot3(d1, d1), E = dot3(d2, d2), F = dot3(d2, r), C = dot3(d1, r), B = dot3(d1, d2);
    double den = A * E - B * B, s = 0, tt = 0;
    if (den > MINVAL) s = (B * F - C * E) / den;
    s = s < 0 ? 0 : (s > 1 ? 1 : s);
    tt = E > MINVAL ? (B * s + F) / E : 0;
    if (tt < 0) { tt = 0; s = A > MINVAL ? -C / A : 0; } else if (tt > 1) { tt = 1; s = A > MINVAL ? (B - C) / A : 0; }
    s = s < 0 ? 0 : (s > 1 ? 1 : s);
    for (int a = 0; a < 3; a++) d->con_pos[slot0][a] = 0.5 * (a0[a] + s * d1[a] + b0[a] + tt * d2[a]);
    d->con_dist[slot0] = best;
    memcpy(d->con_frame[slot0], fr, sizeof(fr));
    return;
  }
  /* face contact, mjx's clipped manifold: the incident face (the other hull's face most
   * anti-parallel to the reference face's normal; the first among equal ones) clipped by the
   * reference face's side planes (Sutherland-Hodgman, planes in the reference polygon's order),
   * the clipped points below the reference plane, 4 of them by _manifold_points. Each contact
   * sits midway between its point and the reference plane. */
  const int inc_hull = btype == 0 ? 1 : 0;
  double (*Vi)[3] = inc_hull == 1 ? V2 : V1;
  double (*Vr)[3] = inc_hull == 1 ? V1 : V2;
  const double* Rr = btype == 0 ? R1 : R2;
  const double* Ri = btype == 0 ? R2 : R1;
  const double* pr = btype == 0 ? p1 : p2;
  double fn[3], off;
  mulmv3(fn, Rr, m->hull_face_normal[bi]);
  off = m->hull_face_offset[bi] + dot3(fn, pr);  /* world plane: fn . x = off (fn outward of ref hull) */
  int finc = 0;
  double dmin = 1e300;
  for (int f = 0; f < nf; f++) {
    double ni[3];
    mulmv3(ni, Ri, m->hull_face_normal[f]);
    const double dd = dot3(ni, fn);
    if (dd < dmin) { dmin = dd; finc = f; }
  }
  enum { CLIPMAX = 2 * DUCK_MAXHULLV };
  double poly[CLIPMAX][3], tmpp[CLIPMAX][3];
  int np = m->hull_face_nv[finc];
  for (int i = 0; i < np; i++) memcpy(poly[i], Vi[m->hull_face_vert[finc][i]], sizeof(double) * 3);
  const int nr = m->hull_face_nv[bi];
  for (int i = 0; i < nr && np > 0; i++) {
    const double *a = Vr[m->hull_face_vert[bi][i]], *b = Vr[m->hull_face_vert[bi][(i + 1) % nr]];
    double ab[3], sd[3];
    for (int q = 0; q < 3; q++) ab[q] = b[q] - a[q];
    cross3(sd, ab, fn); /* outward side normal of the reference polygon's edge a -> b */
    int nt = 0;
    for (int j = 0; j < np; j++) {
      const double *P = poly[j], *Q = poly[(j + 1) % np];
      const double dp = sd[0] * (P[0] - a[0]) + sd[1] * (P[1] - a[1]) + sd[2] * (P[2] - a[2]);
      const double dq = sd[0] * (Q[0] - a[0]) + sd[1] * (Q[1] - a[1]) + sd[2] * (Q[2] - a[2]);
      if (dp <= 0) memcpy(tmpp[nt++], P, sizeof(double) * 3);
      if ((dp <= 0) != (dq <= 0)) {
        const double tt = dp / (dp - dq);
        for (int q = 0; q < 3; q++) tmpp[nt][q] = P[q] + tt * (Q[q] - P[q]);
        nt++;
      }
      if (nt > CLIPMAX - 2) abort(); /* fixed capacity: a convex clip never grows past np + nr */
    }
    np = nt;
    memcpy(poly, tmpp, sizeof(double) * 3 * (size_t)nt);
  }
  double depth[CLIPMAX];
  int mask[CLIPMAX], idx[4], any = 0;
  for (int k = 0; k < np; k++) {
    depth[k] = off - dot3(fn, poly[k]);
    mask[k] = depth[k] > 0;
    any |= mask[k];
  }
  if (!any) return;
  manifold_points((const double(*)[3])poly, mask, np, fn, idx);
  for (int c = 0; c < 4; c++) {
    int k = idx[c], unique = 1;
    for (int e = 0; e < c; e++)
      if (idx[e] == k) unique = 0;
    double dist = unique ? -depth[k] : 1.0;
    int s = slot0 + c;
    for (int a = 0; a < 3; a++) d->con_pos[s][a] = poly[k][a] - 0.5 * dist * fn[a];
    d->con_dist[s] = dist;
    memcpy(d->con_frame[s], fr, sizeof(fr));
  }
}

/* test aid (oracle_set_con_override): after collision, every slot s takes dist buf[7s], pos
 * buf[7s+1..3] and the frame of normal buf[7s+4..6] (a contact set computed elsewhere, e.g. the
 * kernel's), so that the rest of the substep can be compared from identical contacts; NULL = off */
static _Thread_local const double* g_con_override;
void oracle_set_con_override(const double* buf) { g_con_override = buf; }

static void collision(const oracle_model* m, oracle_data* d) {
  d->ncon = m->npair * DUCK_CON_PER_PAIR;
  for (int p = 0; p < m->npair; p++) {
    int g1 = m->pair_geom1[p], g2 = m->pair_geom2[p], t1 = m->geom_type[g1], t2 = m->geom_type[g2];
    int s0 = p * DUCK_CON_PER_PAIR;
    if (t1 == DUCK_GEOM_PLANE && t2 == DUCK_GEOM_MESH) collide_plane_convex(m, d, g1, g2, s0);
    else if (t1 == DUCK_GEOM_HFIELD && t2 == DUCK_GEOM_MESH && m->hfield_data) collide_hfield_convex(m, d, g1, g2, s0);
    else if (t1 == DUCK_GEOM_MESH && t2 == DUCK_GEOM_MESH) collide_convex_convex(m, d, g1, g2, s0);
    else
      for (int c = 0; c < 4; c++) set_inactive(d, s0 + c, g1, g2);
  }
}

/* ------------------------------------------------------------------------------------ */
/* constraints (mjx constraint.make_constraint semantics)                               */
/* ------------------------------------------------------------------------------------ */

static void kbi(const oracle_model* m, const double* solref, const double* solimp, double pos, double* k,
                double* b, double* imp) {
  double timeconst = solref[0], dampratio = solref[1];
  if (timeconst < 2 * m->timestep) timeconst = 2 * m->timestep; /* refsafe */
  double dmin = fmin(fmax(solimp[0], MINIMP), MAXIMP), dmax = fmin(fmax(solimp[1], MINIMP), MAXIMP);
  double width = fmax(MINVAL, solimp[2]), mid = fmin(fmax(solimp[3], MINIMP), MAXIMP), power = fmax(1.0, solimp[4]);
  *k = 1.0 / (dmax * dmax * timeconst * timeconst * dampratio * dampratio);
  *b = 2.0 / (dmax * timeconst);
  if (solref[0] <= 0) *k = -solref[0] / (dmax * dmax);
  if (solref[1] <= 0) *b = -solref[1] / dmax;
  double x = fabs(pos) / width;
  double ya = (1.0 / pow(mid, power - 1)) * pow(x, power);
  double yb = 1 - (1.0 / pow(1 - mid, power - 1)) * pow(1 - x, power);
  double y = x < mid ? ya : yb;
  double im = dmin + y * (dmax - dmin);
  im = fmin(fmax(im, dmin), dmax);
  if (x > 1.0) im = dmax;
  *imp = im;
}

static void add_row(const oracle_model* m, oracle_data* d, fwd_ws* w, const double* J, double pos,
                    double invweight, const double* solref, const double* solimp, double frictionloss, int ineq) {
  int r = w->nefc++;
  if (r >= MAXEFC) abort(); /* fixed-capacity rows (oracle_model_create bounds nefc) */
  memcpy(w->J[r], J, sizeof(double) * NV);
  double k, b, imp;
  kbi(m, solref, solimp, pos, &k, &b, &imp);
  double R = fmax(invweight * (1 - imp) / imp, MINVAL);
  double vel = 0;
  for (int i = 0; i < m->nv; i++) vel += J[i] * d->qvel[i];
  w->R[r] = R;
  w->D[r] = 1.0 / R;
  w->aref[r] = -b * vel - k * imp * pos;
  w->frictionloss[r] = frictionloss;
  w->ineq[r] = ineq;
}

/* translational jacobian of a world point attached to body b (mj_jac, via cdof) */
static void jac_point(const oracle_model* m, const fwd_ws* w, int b, const double* p, double (*Jp)[NV]) {
  for (int a = 0; a < 3; a++) memset(Jp[a], 0, sizeof(double) * NV);
  if (m->body_weldid[b] == 0) return;
  int wb = m->body_weldid[b];
  const double* c = w->subtree_com[m->body_rootid[b]];
  double off[3] = {p[0] - c[0], p[1] - c[1], p[2] - c[2]};
  for (int dof = m->body_dofadr[wb] + m->body_dofnum[wb] - 1; dof >= 0; dof = m->dof_parentid[dof]) {
    double t[3];
    cross3(t, w->cdof[dof], off);
    for (int a = 0; a < 3; a++) Jp[a][dof] = w->cdof[dof][3 + a] + t[a];
  }
}

static void make_constraint(const oracle_model* m, oracle_data* d, fwd_ws* w) {
  w->nefc = 0;
  double J[NV];
  /* dof friction loss rows (mjx _instantiate_friction) */
  for (int i = 0; i < m->nv; i++) {
    if (!m->dof_has_friction[i]) continue;
    memset(J, 0, sizeof(J));
    J[i] = 1;
    add_row(m, d, w, J, 0.0, m->dof_invweight0[i], m->dof_solref[i], m->dof_solimp[i], m->dof_frictionloss[i], 0);
  }
  /* joint limits (mjx _instantiate_limit_slide_hinge): one row per joint, closer side */
  for (int j = 0; j < m->njnt; j++) {
    if (!m->jnt_limited[j] || (m->jnt_type[j] != DUCK_JNT_HINGE && m->jnt_type[j] != DUCK_JNT_SLIDE)) continue;
    double q = d->qpos[m->jnt_qposadr[j]];
    double dlo = q - m->jnt_range[j][0], dhi = m->jnt_range[j][1] - q;
    double pos = (dlo < dhi ? dlo : dhi) - m->jnt_margin[j];
    if (!(pos < 0)) continue;
    int dof = m->jnt_dofadr[j];
    memset(J, 0, sizeof(J));
    J[dof] = dlo < dhi ? 1.0 : -1.0;
    add_row(m, d, w, J, pos, m->dof_invweight0[dof], m->jnt_solref[j], m->jnt_solimp[j], 0.0, 1);
  }
  /* contacts, pyramidal cone (mjx _instantiate_contact) */
  for (int p = 0; p < m->npair; p++) {
    int g1 = m->pair_geom1[p], g2 = m->pair_geom2[p];
    int b1 = m->geom_bodyid[g1], b2 = m->geom_bodyid[g2];
    double tran = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
    const double* fri = m->pair_friction[p];
    int dim = m->pair_condim[p];
    for (int c = 0; c < DUCK_CON_PER_PAIR; c++) {
      int s = p * DUCK_CON_PER_PAIR + c;
      double pos = d->con_dist[s] - m->pair_margin[p];
      if (!(pos < 0)) continue;
      double J1[3][NV], J2[3][NV], Jd[3][NV];
      jac_point(m, w, b1, d->con_pos[s], J1);
      jac_point(m, w, b2, d->con_pos[s], J2);
      for (int a = 0; a < 3; a++)
        for (int i = 0; i < NV; i++) Jd[a][i] = J2[a][i] - J1[a][i];
      const double* fr = d->con_frame[s];
      double Jf[3][NV];
      for (int r = 0; r < 3; r++)
        for (int i = 0; i < NV; i++) Jf[r][i] = fr[3 * r] * Jd[0][i] + fr[3 * r + 1] * Jd[1][i] + fr[3 * r + 2] * Jd[2][i];
      for (int t = 0; t < dim - 1; t++) {
        double mu = fri[t];
        double iw = (tran + mu * mu * tran) * 2 * fri[0] * fri[0] / m->impratio;
        for (int sgn = 0; sgn < 2; sgn++) {
          for (int i = 0; i < NV; i++) J[i] = Jf[0][i] + (sgn == 0 ? mu : -mu) * Jf[1 + t][i];
          add_row(m, d, w, J, pos, iw, m->pair_solref[p], m->pair_solimp[p], 0.0, 1);
        }
      }
    }
  }
  d->nefc = w->nefc;
}

/* ------------------------------------------------------------------------------------ */
/* Newton solver (mjx solver.solve, iterations = opt.iterations, zoom line search)      */
/* ------------------------------------------------------------------------------------ */

typedef struct sctx {
  double qacc[NV], Ma[NV], Jaref[MAXEFC], efc_force[MAXEFC], qfrc_constraint[NV];
  double grad[NV], Mgrad[NV], search[NV];
  double cost, gauss, prev_cost;
} sctx;

static void mulM(const oracle_model* m, const oracle_data* d, const double* x, double* y) {
  for (int i = 0; i < m->nv; i++) {
    double s = 0;
    for (int j = 0; j < m->nv; j++) s += d->qM[i][j] * x[j];
    y[i] = s;
  }
}

/* _update_constraint: forces and cost at ctx.qacc */
static void update_constraint(const oracle_model* m, const oracle_data* d, const fwd_ws* w, sctx* c) {
  double cost = 0;
  for (int r = 0; r < w->nefc; r++) {
    double x = c->Jaref[r], D = w->D[r];
    if (w->ineq[r]) {
      if (x < 0) { c->efc_force[r] = -D * x; cost += 0.5 * D * x * x; } else c->efc_force[r] = 0;
    } else {
      double f = w->frictionloss[r], rf = w->R[r] * f;
      if (x <= -rf) { c->efc_force[r] = f; cost += -f * x - 0.5 * rf * f; }
      else if (x >= rf) { c->efc_force[r] = -f; cost += f * x - 0.5 * rf * f; }
      else { c->efc_force[r] = -D * x; cost += 0.5 * D * x * x; }
    }
  }
  double gauss = 0;
  for (int i = 0; i < m->nv; i++) gauss += 0.5 * (c->Ma[i] - d->qfrc_smooth[i]) * (c->qacc[i] - d->qacc_smooth[i]);
  for (int i = 0; i < m->nv; i++) {
    double s = 0;
    for (int r = 0; r < w->nefc; r++) s += w->J[r][i] * c->efc_force[r];
    c->qfrc_constraint[i] = s;
  }
  c->prev_cost = c->cost;
  c->gauss = gauss;
  c->cost = gauss + cost;
}

/* test aid (oracle_set_hdump): buf[0] = nefc, buf[1..NV*NV] the first Newton Hessian (row stride NV) of
 * the next solve, then per row (Jaref, |J||qacc| + |aref|, friction band R*f or 0) at that point */
static _Thread_local double* g_hdump;
static _Thread_local int g_hdump_done;
void oracle_set_hdump(double* buf) { g_hdump = buf; g_hdump_done = 0; }

/* _update_gradient (Newton): grad and H^-1 grad with H = M + J' diag(D*active) J */
static void update_gradient(const oracle_model* m, const oracle_data* d, const fwd_ws* w, sctx* c) {
  int nv = m->nv;
  for (int i = 0; i < nv; i++) c->grad[i] = c->Ma[i] - d->qfrc_smooth[i] - c->qfrc_constraint[i];
  double H[NV * NV];
  for (int i = 0; i < nv; i++)
    for (int j = 0; j < nv; j++) H[i * NV + j] = d->qM[i][j];
  for (int r = 0; r < w->nefc; r++) {
    double x = c->Jaref[r];
    int active;
    if (w->ineq[r]) active = x < 0;
    else { double rf = w->R[r] * w->frictionloss[r]; active = (x > -rf) && (x < rf); }
    if (!active) continue;
    for (int i = 0; i < nv; i++) {
      if (w->J[r][i] == 0) continue;
      double a = w->D[r] * w->J[r][i];
      for (int j = 0; j < nv; j++) H[i * NV + j] += a * w->J[r][j];
    }
  }
  if (g_hdump && !g_hdump_done) { /* test aid: the first Newton Hessian and the rows' margins at its point */
    g_hdump_done = 1;
    g_hdump[0] = w->nefc;
    memcpy(g_hdump + 1, H, sizeof(double) * NV * NV);
    for (int r = 0; r < w->nefc; r++) {
      double sc = fabs(w->aref[r]);
      for (int i = 0; i < nv; i++) sc += fabs(w->J[r][i] * c->qacc[i]);
      g_hdump[1 + NV * NV + 3 * r] = c->Jaref[r];
      g_hdump[2 + NV * NV + 3 * r] = sc;
      g_hdump[3 + NV * NV + 3 * r] = w->ineq[r] ? 0 : w->R[r] * w->frictionloss[r];
    }
  }
  cholesky(H, nv);
  memcpy(c->Mgrad, c->grad, sizeof(double) * nv);
  chol_solve(H, nv, c->Mgrad);
}

typedef struct lspt { double alpha, cost, d0, d1; } lspt;

static lspt ls_eval(const oracle_model* m, const fwd_ws* w, const sctx* c, const double* jv, const double qg[3],
                    double alpha) {
  double q0 = qg[0], q1 = qg[1], q2 = qg[2];
  for (int r = 0; r < w->nefc; r++) {
    double x = c->Jaref[r] + alpha * jv[r], D = w->D[r], ja = c->Jaref[r], v = jv[r];
    if (w->ineq[r]) {
      if (x < 0) { q0 += 0.5 * D * ja * ja; q1 += D * v * ja; q2 += 0.5 * D * v * v; }
    } else {
      double f = w->frictionloss[r], rf = w->R[r] * f;
      if (x <= -rf) { q0 += -0.5 * rf * f - f * ja; q1 += -f * v; }
      else if (x >= rf) { q0 += -0.5 * rf * f + f * ja; q1 += f * v; }
      else { q0 += 0.5 * D * ja * ja; q1 += D * v * ja; q2 += 0.5 * D * v * v; }
    }
  }
  lspt p;
  p.alpha = alpha;
  p.cost = alpha * alpha * q2 + alpha * q1 + q0;
  p.d0 = 2 * alpha * q2 + q1;
  p.d1 = 2 * q2;
  return p;
}

/* test aid (oracle_set_ls_floor): the HIP kernel's declared fp32 line-search stop,
 * a bracket end whose slope is below floor x the starting slope; 0 (default) = MJX's rule alone */
static _Thread_local double g_ls_floor;
void oracle_set_ls_floor(double floor) { g_ls_floor = floor; }
/* test aid (oracle_set_force_start): 1 start the Newton solve from qacc_warmstart, 2 from qacc_smooth,
 * 0 (default) the lower-cost one (mjx solver._init); for explaining a near-tie of the two costs */
static _Thread_local int g_force_start;
void oracle_set_force_start(int mode) { g_force_start = mode; }
static _Thread_local double g_start_costs[2];
void oracle_last_start_costs(double out[2]) { out[0] = g_start_costs[0]; out[1] = g_start_costs[1]; }

/* test aid (oracle_ls_trace, tools/ls_divergence.py): the iteration counts of this thread's line searches
 * since the last reset, in call order (the first 4096 kept) */
static _Thread_local int g_ls_hist[4096];
static _Thread_local int g_ls_n;
int oracle_ls_trace(int* out, int cap, int reset) {
  const int n = g_ls_n < cap ? g_ls_n : cap;
  if (out) memcpy(out, g_ls_hist, sizeof(int) * (size_t)(n < 4096 ? n : 4096));
  const int tot = g_ls_n;
  if (reset) g_ls_n = 0;
  return tot;
}

static void linesearch(const oracle_model* m, const oracle_data* d, const fwd_ws* w, sctx* c) {
  int nv = m->nv;
  double snorm = 0;
  for (int i = 0; i < nv; i++) snorm += c->search[i] * c->search[i];
  snorm = sqrt(snorm);
  double smag = snorm * m->meaninertia * (nv > 1 ? nv : 1);
  double gtol = m->tolerance * m->ls_tolerance * smag;
  double mv[NV], jv[MAXEFC];
  mulM(m, d, c->search, mv);
  for (int r = 0; r < w->nefc; r++) {
    double s = 0;
    for (int i = 0; i < nv; i++) s += w->J[r][i] * c->search[i];
    jv[r] = s;
  }
  double qg[3];
  double sMa = 0, sf = 0, sMv = 0;
  for (int i = 0; i < nv; i++) { sMa += c->search[i] * c->Ma[i]; sf += c->search[i] * d->qfrc_smooth[i]; sMv += c->search[i] * mv[i]; }
  qg[0] = c->gauss; qg[1] = sMa - sf; qg[2] = 0.5 * sMv;

  lspt p0 = ls_eval(m, w, c, jv, qg, 0.0);
  lspt lo = ls_eval(m, w, c, jv, qg, p0.alpha - p0.d0 / p0.d1);
  lspt hi;
  if (lo.d0 < p0.d0) { hi = p0; } else { hi = lo; lo = p0; }
  if (g_ls_floor > 0 && g_ls_floor * fabs(p0.d0) > gtol) gtol = g_ls_floor * fabs(p0.d0);
  int swap = 1, iter = 0;
  for (;;) {
    int done = iter >= m->ls_iterations;
    done |= !swap;
    done |= (lo.d0 < 0) && (lo.d0 > -gtol);
    done |= (hi.d0 > 0) && (hi.d0 < gtol);
    if (done) break;
    lspt lo_next = ls_eval(m, w, c, jv, qg, lo.alpha - lo.d0 / lo.d1);
    lspt hi_next = ls_eval(m, w, c, jv, qg, hi.alpha - hi.d0 / hi.d1);
    lspt mid = ls_eval(m, w, c, jv, qg, 0.5 * (lo.alpha + hi.alpha));
    int s1 = (lo.d0 > 0) || (lo.d0 < lo_next.d0);
    if (s1) lo = lo_next;
    int s2 = (mid.d0 < 0) && (lo.d0 < mid.d0);
    if (s2) lo = mid;
    int s3 = (hi.d0 < 0) || (hi.d0 > hi_next.d0);
    if (s3) hi = hi_next;
    int s4 = (mid.d0 > 0) && (hi.d0 > mid.d0);
    if (s4) hi = mid;
    swap = s1 || s2 || s3 || s4;
    iter++;
  }
  if (g_ls_n < 4096) g_ls_hist[g_ls_n] = iter;
  g_ls_n++;
  int improved = (lo.cost < p0.cost) || (hi.cost < p0.cost);
  double alpha = lo.cost < hi.cost ? lo.alpha : hi.alpha;
  if (improved) {
    for (int i = 0; i < nv; i++) { c->qacc[i] += c->search[i] * alpha; c->Ma[i] += mv[i] * alpha; }
    for (int r = 0; r < w->nefc; r++) c->Jaref[r] += jv[r] * alpha;
  }
}

static void ctx_init(const oracle_model* m, const oracle_data* d, const fwd_ws* w, sctx* c, const double* qacc) {
  memcpy(c->qacc, qacc, sizeof(double) * m->nv);
  mulM(m, d, c->qacc, c->Ma);
  for (int r = 0; r < w->nefc; r++) {
    double s = 0;
    for (int i = 0; i < m->nv; i++) s += w->J[r][i] * c->qacc[i];
    c->Jaref[r] = s - w->aref[r];
  }
  c->cost = 0;
  update_constraint(m, d, w, c);
}

static void solve(const oracle_model* m, oracle_data* d, const fwd_ws* w) {
  int nv = m->nv;
  if (w->nefc == 0) {
    memcpy(d->qacc, d->qacc_smooth, sizeof(double) * nv);
    memset(d->qfrc_constraint, 0, sizeof(double) * nv);
    memcpy(d->qacc_warmstart, d->qacc, sizeof(double) * nv);
    return;
  }
  sctx warm, smth, *c;
  ctx_init(m, d, w, &warm, d->qacc_warmstart);
  ctx_init(m, d, w, &smth, d->qacc_smooth);
  g_start_costs[0] = warm.cost;
  g_start_costs[1] = smth.cost;
  c = warm.cost < smth.cost ? &warm : &smth;
  if (g_force_start) c = g_force_start == 1 ? &warm : &smth; /* test aid */
  update_gradient(m, d, w, c);
  for (int i = 0; i < nv; i++) c->search[i] = -c->Mgrad[i];
  int it = 0;
  for (;;) {
    linesearch(m, d, w, c);
    update_constraint(m, d, w, c);
    it++;
    if (it >= m->iterations) break;
    update_gradient(m, d, w, c);
    double scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
    double improvement = scale * (c->prev_cost - c->cost);
    double gn = 0;
    for (int i = 0; i < nv; i++) gn += c->grad[i] * c->grad[i];
    double gradient = scale * sqrt(gn);
    if (improvement < m->tolerance || gradient < m->tolerance) break;
    for (int i = 0; i < nv; i++) c->search[i] = -c->Mgrad[i];
  }
  d->solver_niter = it;
  memcpy(d->qacc, c->qacc, sizeof(double) * nv);
  memcpy(d->qfrc_constraint, c->qfrc_constraint, sizeof(double) * nv);
  memcpy(d->efc_force, c->efc_force, sizeof(double) * w->nefc);
  memcpy(d->qacc_warmstart, d->qacc, sizeof(double) * nv);
}

/* ------------------------------------------------------------------------------------ */
/* sensors                                                                              */
/* ------------------------------------------------------------------------------------ */

static void site_vel(const oracle_model* m, const oracle_data* d, const fwd_ws* w, int s, double* ang, double* lin) {
  int b = m->site_bodyid[s];
  const double* cv = w->cvel[b];
  const double* c = w->subtree_com[m->body_rootid[b]];
  double off[3] = {d->site_xpos[s][0] - c[0], d->site_xpos[s][1] - c[1], d->site_xpos[s][2] - c[2]};
  double t[3];
  cross3(t, cv, off);
  for (int a = 0; a < 3; a++) { ang[a] = cv[a]; lin[a] = cv[3 + a] + t[a]; }
}

static void sensors(const oracle_model* m, oracle_data* d, const fwd_ws* w, int stage_acc) {
  double cacc[DUCK_MAXBODY][6];
  if (stage_acc) { /* mj_rnePostConstraint: com-based accelerations incl. -gravity */
    memset(cacc[0], 0, 6 * sizeof(double));
    for (int k = 0; k < 3; k++) cacc[0][3 + k] = -m->gravity[k];
    for (int i = 1; i < m->nbody; i++) {
      memcpy(cacc[i], cacc[m->body_parentid[i]], 6 * sizeof(double));
      for (int j = 0; j < m->body_dofnum[i]; j++) {
        int dof = m->body_dofadr[i] + j;
        for (int c = 0; c < 6; c++) cacc[i][c] += w->cdof_dot[dof][c] * d->qvel[dof] + w->cdof[dof][c] * d->qacc[dof];
      }
    }
  }
  for (int i = 0; i < m->nsensor; i++) {
    int s = m->sensor_objid[i], adr = m->sensor_adr[i], typ = m->sensor_type[i];
    double* out = d->sensordata + adr;
    const double* R = d->site_xmat[s];
    double ang[3], lin[3];
    if (typ == DUCK_SENS_ACCELEROMETER) {
      if (!stage_acc) continue;
      int b = m->site_bodyid[s];
      const double* c = w->subtree_com[m->body_rootid[b]];
      double off[3] = {d->site_xpos[s][0] - c[0], d->site_xpos[s][1] - c[1], d->site_xpos[s][2] - c[2]};
      double t[3], acc[3];
      cross3(t, cacc[b], off);
      for (int a = 0; a < 3; a++) acc[a] = cacc[b][3 + a] + t[a];
      site_vel(m, d, w, s, ang, lin);
      cross3(t, ang, lin);
      for (int a = 0; a < 3; a++) acc[a] += t[a];
      mulmtv3(out, R, acc);
      continue;
    }
    if (stage_acc) continue;
    switch (typ) {
      case DUCK_SENS_GYRO: site_vel(m, d, w, s, ang, lin); mulmtv3(out, R, ang); break;
      case DUCK_SENS_VELOCIMETER: site_vel(m, d, w, s, ang, lin); mulmtv3(out, R, lin); break;
      case DUCK_SENS_FRAMEZAXIS: out[0] = R[2]; out[1] = R[5]; out[2] = R[8]; break;
      case DUCK_SENS_FRAMEXAXIS: out[0] = R[0]; out[1] = R[3]; out[2] = R[6]; break;
      case DUCK_SENS_FRAMELINVEL: site_vel(m, d, w, s, ang, lin); memcpy(out, lin, sizeof(lin)); break;
      case DUCK_SENS_FRAMEANGVEL: site_vel(m, d, w, s, ang, lin); memcpy(out, ang, sizeof(ang)); break;
      case DUCK_SENS_FRAMEPOS: memcpy(out, d->site_xpos[s], 3 * sizeof(double)); break;
      case DUCK_SENS_FRAMEQUAT: memcpy(out, w->site_xquat[s], 4 * sizeof(double)); break;
      default: break;
    }
  }
}

/* ------------------------------------------------------------------------------------ */
/* forward / step                                                                       */
/* ------------------------------------------------------------------------------------ */

static void forward_ws(const oracle_model* m, oracle_data* d, fwd_ws* w) {
  int nv = m->nv;
  kinematics(m, d, w);
  com_pos(m, d, w);
  crb(m, d, w);
  collision(m, d);
  if (g_con_override)
    for (int c = 0; c < d->ncon; c++) {
      const double* o = g_con_override + 7 * c;
      d->con_dist[c] = o[0];
      memcpy(d->con_pos[c], o + 1, 3 * sizeof(double));
      make_frame(d->con_frame[c], o + 4);
    }
  make_constraint(m, d, w);
  com_vel(m, d, w);
  sensors(m, d, w, 0);
  /* passive: explicit joint damping (springs are zero in these models) */
  for (int i = 0; i < nv; i++) d->qfrc_passive[i] = -m->dof_damping[i] * d->qvel[i];
  rne_bias(m, d, w);
  /* actuation: <position> servos (mjx forward.fwd_actuation) */
  memset(d->qfrc_actuator, 0, sizeof(double) * nv);
  for (int a = 0; a < m->nu; a++) {
    int j = m->actuator_trnid[a];
    double ctrl = d->ctrl[a];
    if (m->actuator_ctrllimited[a]) ctrl = fmin(fmax(ctrl, m->actuator_ctrlrange[a][0]), m->actuator_ctrlrange[a][1]);
    double gear = m->actuator_gear[a];
    double len = gear * d->qpos[m->jnt_qposadr[j]], vel = gear * d->qvel[m->jnt_dofadr[j]];
    double f = m->actuator_kp[a] * ctrl - m->actuator_kp[a] * len - m->actuator_kv[a] * vel;
    if (m->actuator_forcelimited[a]) f = fmin(fmax(f, m->actuator_forcerange[a][0]), m->actuator_forcerange[a][1]);
    d->actuator_force[a] = f;
    d->qfrc_actuator[m->jnt_dofadr[j]] += gear * f;
  }
  /* smooth acceleration */
  for (int i = 0; i < nv; i++) d->qfrc_smooth[i] = d->qfrc_passive[i] - d->qfrc_bias[i] + d->qfrc_actuator[i];
  double L[NV * NV];
  for (int i = 0; i < nv; i++)
    for (int j = 0; j < nv; j++) L[i * NV + j] = d->qM[i][j];
  cholesky(L, nv);
  memcpy(d->qacc_smooth, d->qfrc_smooth, sizeof(double) * nv);
  chol_solve(L, nv, d->qacc_smooth);
  solve(m, d, w);
  sensors(m, d, w, 1);
}

void oracle_forward(const oracle_model* m, oracle_data* d) {
  fwd_ws w;
  forward_ws(m, d, &w);
}

/* mj_Euler with eulerdamp disabled (integrator.euler -> _advance), semi-implicit */
static void euler(const oracle_model* m, oracle_data* d) {
  double dt = m->timestep;
  for (int i = 0; i < m->nv; i++) d->qvel[i] += dt * d->qacc[i];
  for (int j = 0; j < m->njnt; j++) {
    int qa = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
    if (m->jnt_type[j] == DUCK_JNT_FREE) {
      for (int k = 0; k < 3; k++) d->qpos[qa + k] += dt * d->qvel[da + k];
      double* q = d->qpos + qa + 3;
      double v[3] = {d->qvel[da + 3], d->qvel[da + 4], d->qvel[da + 5]};
      double nv = norm3(v), axis[3] = {1, 0, 0};
      if (nv > MINVAL) { axis[0] = v[0] / nv; axis[1] = v[1] / nv; axis[2] = v[2] / nv; }
      double qr[4];
      axis_angle_quat(qr, axis, dt * nv);
      quat_mul(q, q, qr);
      quat_normalize(q);
    } else {
      d->qpos[qa] += dt * d->qvel[da];
    }
  }
}

void oracle_step(const oracle_model* m, oracle_data* d, int nsubstep) {
  for (int s = 0; s < nsubstep; s++) {
    oracle_forward(m, d);
    euler(m, d);
  }
}

/* ------------------------------------------------------------------------------------ */
/* RNG: threefry2x32 with 20 rounds                                                     */
/* ------------------------------------------------------------------------------------ */

static uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

void oracle_threefry2x32(const uint32_t key[2], const uint32_t ctr[2], uint32_t out[2]) {
  static const int R[8] = {13, 15, 26, 6, 17, 29, 16, 24};
  uint32_t ks[3] = {key[0], key[1], 0x1BD11BDAu ^ key[0] ^ key[1]};
  uint32_t x0 = ctr[0] + ks[0], x1 = ctr[1] + ks[1];
  for (int r = 0; r < 20; r++) {
    x0 += x1;
    x1 = rotl32(x1, R[r % 8]);
    x1 ^= x0;
    if (r % 4 == 3) {
      uint32_t s = (uint32_t)(r / 4 + 1);
      x0 += ks[s % 3];
      x1 += ks[(s + 1) % 3] + s;
    }
  }
  out[0] = x0; out[1] = x1;
}

typedef struct rng_t { uint32_t key[2]; uint32_t ctr; } rng_t;

/* slot k of counter ctr -> uniform in [0,1) with 23 random bits (exact in fp32) */
static double rng_u(const rng_t* r, int slot) {
  uint32_t c[2] = {r->ctr, (uint32_t)(slot >> 1)}, o[2];
  oracle_threefry2x32(r->key, c, o);
  return (double)(o[slot & 1] >> 9) * (1.0 / 8388608.0);
}
static double rng_uniform(const rng_t* r, int slot, double lo, double hi) {
  return (double)(float)(lo + (hi - lo) * rng_u(r, slot));
}
static int rng_randint(const rng_t* r, int slot, int lo, int hi) {
  int k = (int)floor(rng_u(r, slot) * (hi - lo));
  if (k > hi - lo - 1) k = hi - lo - 1;
  return lo + k;
}
static void derive_key(uint64_t seed, int64_t env_id, uint32_t tag, uint32_t out[2]) {
  uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t c[2] = {(uint32_t)env_id, tag ^ (uint32_t)((uint64_t)env_id >> 32)};
  oracle_threefry2x32(k, c, out);
}

/* per-step slot map (documented in DESIGN.md) */
enum {
  SLOT_ACTION_DELAY = 0, SLOT_PUSH_THETA = 1, SLOT_PUSH_MAG = 2, SLOT_GYRO = 3, SLOT_ACCEL = 6,
  SLOT_GRAVITY = 9, SLOT_IMU_IDX = 12, SLOT_QPOS = 13, SLOT_QVEL = 29, SLOT_CMD = 45
};
/* reset slot map */
enum { RSLOT_DXY = 0, RSLOT_YAW = 2, RSLOT_QSCALE = 3, RSLOT_QVEL = 19, RSLOT_CMD = 25, RSLOT_PUSH = 33, RSLOT_OBS = 64 };
#define KEY_TAG_ENV 0x5EEDu
#define KEY_TAG_DR 0xD0D0u

/* ------------------------------------------------------------------------------------ */
/* domain randomisation (randomize.py:26-146)                                            */
/* ------------------------------------------------------------------------------------ */

void oracle_dr_sample(const oracle_model* m, uint64_t seed, int64_t env_id, double* dr) {
  duck_dr_layout L = duck_dr_layout_make(m->nbody, m->nu);
  rng_t r;
  derive_key(seed, env_id, KEY_TAG_DR, r.key);
  r.ctr = 0;
  int slot = 0;
  dr[L.floor_friction] = rng_uniform(&r, slot++, 0.5, 1.0);
  for (int a = 0; a < m->nu; a++) dr[L.frictionloss + a] = rng_uniform(&r, slot++, 0.9, 1.1);
  for (int a = 0; a < m->nu; a++) dr[L.armature + a] = rng_uniform(&r, slot++, 1.0, 1.05);
  for (int k = 0; k < 3; k++) dr[L.base_ipos + k] = rng_uniform(&r, slot++, -0.05, 0.05);
  for (int b = 0; b < m->nbody; b++) dr[L.body_mass + b] = rng_uniform(&r, slot++, 0.9, 1.1);
  double dmass = rng_uniform(&r, slot++, -0.1, 0.1);
  for (int a = 0; a < m->nu; a++) dr[L.qpos0 + a] = rng_uniform(&r, slot++, -0.03, 0.03);
  for (int a = 0; a < m->nu; a++) dr[L.kp + a] = rng_uniform(&r, slot++, 0.9, 1.1);
  /* convert factors to absolute values of the randomised model */
  for (int a = 0; a < m->nu; a++) {
    int dof = m->jnt_dofadr[m->actuator_trnid[a]];
    int qa = m->jnt_qposadr[m->actuator_trnid[a]];
    dr[L.frictionloss + a] *= m->dof_frictionloss[dof];
    dr[L.armature + a] *= m->dof_armature[dof];
    dr[L.qpos0 + a] += m->qpos0[qa];
    dr[L.kp + a] *= m->actuator_kp[a];
  }
  for (int k = 0; k < 3; k++) dr[L.base_ipos + k] += m->body_ipos[1][k];
  for (int b = 0; b < m->nbody; b++) dr[L.body_mass + b] *= m->body_mass[b];
  dr[L.body_mass + 1] += dmass;
}

oracle_model* oracle_model_randomized(const oracle_model* m, const double* dr) {
  duck_dr_layout L = duck_dr_layout_make(m->nbody, m->nu);
  oracle_model* r = (oracle_model*)malloc(sizeof(oracle_model));
  memcpy(r, m, sizeof(oracle_model));
  if (m->hfield_data) {
    r->hfield_data = (double*)malloc(sizeof(double) * (size_t)m->hfield_nrow * m->hfield_ncol);
    memcpy(r->hfield_data, m->hfield_data, sizeof(double) * (size_t)m->hfield_nrow * m->hfield_ncol);
  }
  for (int k = 0; k < 3; k++) r->body_ipos[1][k] = dr[L.base_ipos + k];
  for (int b = 0; b < m->nbody; b++) r->body_mass[b] = dr[L.body_mass + b];
  for (int a = 0; a < m->nu; a++) {
    int j = m->actuator_trnid[a];
    r->dof_frictionloss[m->jnt_dofadr[j]] = dr[L.frictionloss + a];
    r->dof_armature[m->jnt_dofadr[j]] = dr[L.armature + a];
    r->qpos0[m->jnt_qposadr[j]] = dr[L.qpos0 + a];
    r->actuator_kp[a] = dr[L.kp + a];
  }
  return r;
}

/* ------------------------------------------------------------------------------------ */
/* env: reference motion, rewards, obs, reset, step                                     */
/* ------------------------------------------------------------------------------------ */

static int nearest(const float* grid, int n, double v) {
  int best = 0;
  double bd = fabs((double)grid[0] - v);
  for (int i = 1; i < n; i++) {
    double dd = fabs((double)grid[i] - v);
    if (dd < bd) { bd = dd; best = i; }
  }
  return best;
}

/* PolyReferenceMotion.get_reference_motion (poly_reference_motion.py:148-168) */
void oracle_reference_motion(const duck_refmotion* ref, double dx, double dy, double dth, int i, double out[40]) {
  dx = fmin(fmax(dx, ref->dx_range[0]), ref->dx_range[1]);
  dy = fmin(fmax(dy, ref->dy_range[0]), ref->dy_range[1]);
  dth = fmin(fmax(dth, ref->dtheta_range[0]), ref->dtheta_range[1]);
  int ix = nearest(ref->dxs, ref->n_dx, dx), iy = nearest(ref->dys, ref->n_dy, dy),
      it = nearest(ref->dthetas, ref->n_dtheta, dth);
  int nb = ref->nb_steps_in_period;
  double t = (double)(((i % nb) + nb) % nb) / nb;
  t = fmin(fmax(t, 0.0), 1.0);
  const double* c = ref->coeffs + ((size_t)((ix * ref->n_dy + iy) * ref->n_dtheta + it)) * ref->n_dim * ref->n_coef;
  for (int d = 0; d < ref->n_dim && d < 40; d++) {
    /* np.polyval on the flipped (descending) coefficients = Horner from the top power */
    double acc = 0;
    for (int k = ref->n_coef - 1; k >= 0; k--) acc = acc * t + c[d * ref->n_coef + k];
    out[d] = acc;
  }
}

static double nan_to_num(double x) {
  if (isnan(x)) return 0.0;
  if (isinf(x)) return x > 0 ? 3.4028234663852886e38 : -3.4028234663852886e38;
  return x;
}

/* custom_rewards.reward_imitation (custom_rewards.py:4-148), use_imitation_reward = True */
double oracle_reward_imitation(const double base_qpos[7], const double base_qvel[6], const double* jq,
                               const double* jqd, const double contacts[2], const double* ref,
                               const double cmd[7], int nu) {
  (void)base_qpos;
  double cmd_norm = sqrt(cmd[0] * cmd[0] + cmd[1] * cmd[1] + cmd[2] * cmd[2]);
  double lxy = 0, ax = 0;
  for (int k = 0; k < 2; k++) lxy += (base_qvel[k] - ref[34 + k]) * (base_qvel[k] - ref[34 + k]);
  double lin_xy = exp(-8.0 * lxy);
  double lin_z = exp(-8.0 * (base_qvel[2] - ref[36]) * (base_qvel[2] - ref[36]));
  for (int k = 0; k < 2; k++) ax += (base_qvel[3 + k] - ref[37 + k]) * (base_qvel[3 + k] - ref[37 + k]);
  double ang_xy = exp(-2.0 * ax) * 0.5;
  double ang_z = exp(-2.0 * (base_qvel[5] - ref[39]) * (base_qvel[5] - ref[39])) * 0.5;
  /* legs only: ref dims [0:5] + [11:16] vs joints [0:5] + [9:14] */
  double jp = 0, jv = 0;
  for (int k = 0; k < 5; k++) {
    jp += (jq[k] - ref[k]) * (jq[k] - ref[k]);
    jp += (jq[nu - 5 + k] - ref[11 + k]) * (jq[nu - 5 + k] - ref[11 + k]);
    jv += (jqd[k] - ref[16 + k]) * (jqd[k] - ref[16 + k]);
    jv += (jqd[nu - 5 + k] - ref[27 + k]) * (jqd[nu - 5 + k] - ref[27 + k]);
  }
  double joint_pos = -jp * 15.0, joint_vel = -jv * 1e-3;
  double contact = 0;
  for (int k = 0; k < 2; k++) contact += (contacts[k] == (ref[32 + k] > 0.5 ? 1.0 : 0.0)) ? 1.0 : 0.0;
  double r = lin_xy + lin_z + ang_xy + ang_z + joint_pos + joint_vel + contact;
  r *= cmd_norm > 0.01 ? 1.0 : 0.0;
  return nan_to_num(r);
}

/* common/rewards.py terms used by joystick.py:634-667 (unscaled):
 * out = {tracking_lin_vel, tracking_ang_vel, torques, action_rate, stand_still} */
void oracle_rewards(const double cmd[7], const double lv[3], const double gyro[3], const double* af,
                    const double* action, const double* last_act, const double* jq, const double* jqd,
                    const double* q0, int nu, double sigma, double out[5]) {
  double ex = (cmd[0] - lv[0]) * (cmd[0] - lv[0]);
  double ey = fmax(fabs(lv[1] - cmd[1]) - 0.1, 0.0);
  out[0] = nan_to_num(exp(-(ex + ey * ey) / sigma));
  out[1] = nan_to_num(exp(-((cmd[2] - gyro[2]) * (cmd[2] - gyro[2])) / sigma));
  double t = 0, a = 0, pc = 0, vc = 0;
  for (int k = 0; k < nu; k++) {
    t += af[k] * af[k];
    a += (action[k] - last_act[k]) * (action[k] - last_act[k]);
    pc += fabs(jq[k] - q0[k]);
    vc += fabs(jqd[k]);
  }
  out[2] = nan_to_num(t);
  out[3] = nan_to_num(a);
  double cn = sqrt(cmd[0] * cmd[0] + cmd[1] * cmd[1] + cmd[2] * cmd[2]);
  out[4] = nan_to_num(pc + vc) * (cn < 0.01 ? 1.0 : 0.0);
}

/* Standing reward terms, unscaled (standing.py:584-606 via common/rewards.py):
 * out = {orientation (:45-46), torques, action_rate, alive, stand_still(ignore_head=True) (:93-117),
 *        head_pos (:131-147)} */
void oracle_standing_rewards(const double cmd[7], const double up[3], const double* af, const double* action,
                             const double* last_act, const double* jq, const double* jqd, const double* q0, int nu,
                             double out[6]) {
  double t = 0, a = 0, pc = 0, vc = 0, hp = 0;
  for (int k = 0; k < nu; k++) {
    t += af[k] * af[k];
    a += (action[k] - last_act[k]) * (action[k] - last_act[k]);
  }
  for (int k = 0; k < 5; k++) { /* legs: qpos[:5] and qpos[9:] */
    pc += fabs(jq[k] - q0[k]);
    vc += fabs(jqd[k]);
  }
  for (int k = nu - 5; k < nu; k++) {
    pc += fabs(jq[k] - q0[k]);
    vc += fabs(jqd[k]);
  }
  for (int k = 0; k < 4; k++) hp += (jq[5 + k] - cmd[3 + k]) * (jq[5 + k] - cmd[3 + k]);
  double cn = sqrt(cmd[0] * cmd[0] + cmd[1] * cmd[1] + cmd[2] * cmd[2]);
  out[0] = nan_to_num(up[0] * up[0] + up[1] * up[1]);
  out[1] = nan_to_num(t);
  out[2] = nan_to_num(a);
  out[3] = 1.0;
  out[4] = nan_to_num(pc + vc) * (cn < 0.01 ? 1.0 : 0.0);
  out[5] = nan_to_num(hp) * (cn > 0.01 ? 1.0 : 0.0);
}

/* Joystick.sample_command (joystick.py:671-725) */
static void sample_command(const duck_env_config* cfg, const rng_t* r, int slot, double cmd[7]) {
  double f = cfg->head_range_factor;
  cmd[0] = rng_uniform(r, slot + 0, cfg->lin_vel_x[0], cfg->lin_vel_x[1]);
  cmd[1] = rng_uniform(r, slot + 1, cfg->lin_vel_y[0], cfg->lin_vel_y[1]);
  cmd[2] = rng_uniform(r, slot + 2, cfg->ang_vel_yaw[0], cfg->ang_vel_yaw[1]);
  cmd[3] = rng_uniform(r, slot + 3, cfg->neck_pitch_range[0] * f, cfg->neck_pitch_range[1] * f);
  cmd[4] = rng_uniform(r, slot + 4, cfg->head_pitch_range[0] * f, cfg->head_pitch_range[1] * f);
  cmd[5] = rng_uniform(r, slot + 5, cfg->head_yaw_range[0] * f, cfg->head_yaw_range[1] * f);
  cmd[6] = rng_uniform(r, slot + 6, cfg->head_roll_range[0] * f, cfg->head_roll_range[1] * f);
  if (rng_u(r, slot + 7) < 0.1)
    for (int k = 0; k < 7; k++) cmd[k] = 0;
}

/* mujoco_playground collision.geoms_colliding on the fixed contact slots */
static double geoms_colliding(const oracle_data* d, int g1, int g2) {
  double best = 1e4;
  int found = 0;
  for (int s = 0; s < d->ncon; s++) {
    int a = d->con_geom1[s], b = d->con_geom2[s];
    if ((a == g1 && b == g2) || (a == g2 && b == g1)) {
      found = 1;
      if (d->con_dist[s] < best) best = d->con_dist[s];
    }
  }
  return (found && best < 0) ? 1.0 : 0.0;
}

/* Joystick._get_obs (joystick.py:487-620). fstate/istate = this env, stride 1. */
static void get_obs(const oracle_model* m, const duck_env_config* cfg, const duck_layout* L, const oracle_data* d,
                    double* fs, const rng_t* r, int slot_base, const double contact[2], double* obs, double* priv) {
  int nu = m->nu;
  const double* sd = d->sensordata;
  double gyro[3], acc[3], grav[3], jangle[DUCK_MAXU], jvel[DUCK_MAXU];
  const double* R = d->site_xmat[cfg->imu_site];
  for (int k = 0; k < 3; k++) {
    gyro[k] = sd[cfg->sens_gyro + k];
    acc[k] = sd[cfg->sens_accelerometer + k];
    grav[k] = -R[6 + k]; /* site_xmat.T @ [0,0,-1] */
  }
  double ngyro[3], nacc[3], ngrav[3];
  for (int k = 0; k < 3; k++) {
    ngyro[k] = gyro[k] + (2 * rng_u(r, slot_base + SLOT_GYRO + k) - 1) * cfg->noise_level * cfg->noise_gyro;
    nacc[k] = acc[k] + (2 * rng_u(r, slot_base + SLOT_ACCEL + k) - 1) * cfg->noise_level * cfg->noise_accelerometer;
    ngrav[k] = grav[k] + (2 * rng_u(r, slot_base + SLOT_GRAVITY + k) - 1) * cfg->noise_level * cfg->noise_gravity;
  }
  /* IMU delay history (joystick.py:521-530); the delayed sample is never emitted */
  double* ih = fs + L->imu_history;
  for (int k = 8; k >= 3; k--) ih[k] = ih[k - 3];
  for (int k = 0; k < 3; k++) ih[k] = ngrav[k];
  for (int a = 0; a < nu; a++) {
    jangle[a] = d->qpos[cfg->actuator_qposadr[a]];
    if (cfg->backlash_qposadr[a] >= 0) jangle[a] += d->qpos[cfg->backlash_qposadr[a]];
    jvel[a] = d->qvel[cfg->actuator_qveladr[a]];
  }
  int o = 0;
  for (int k = 0; k < 3; k++) obs[o++] = ngyro[k];
  for (int k = 0; k < 3; k++) obs[o++] = nacc[k];
  for (int k = 0; k < 7; k++) obs[o++] = fs[L->command + k];
  for (int a = 0; a < nu; a++)
    obs[o++] = jangle[a] + (2 * rng_u(r, slot_base + SLOT_QPOS + a) - 1) * cfg->noise_level * cfg->qpos_noise_scale[a] -
               cfg->default_actuator[a];
  for (int a = 0; a < nu; a++)
    obs[o++] = (jvel[a] + (2 * rng_u(r, slot_base + SLOT_QVEL + a) - 1) * cfg->noise_level * cfg->noise_joint_vel) *
               cfg->dof_vel_scale;
  for (int a = 0; a < nu; a++) obs[o++] = fs[L->last_act + a];
  for (int a = 0; a < nu; a++) obs[o++] = fs[L->last_last_act + a];
  for (int a = 0; a < nu; a++) obs[o++] = fs[L->last_last_last_act + a];
  int joystick = L->task == DUCK_TASK_JOYSTICK; /* standing.py:532-548 has no targets, no phase */
  if (joystick)
    for (int a = 0; a < nu; a++) obs[o++] = fs[L->motor_targets + a];
  obs[o++] = contact[0];
  obs[o++] = contact[1];
  if (joystick) {
    obs[o++] = fs[L->imitation_phase];
    obs[o++] = fs[L->imitation_phase + 1];
  }
  /* privileged */
  int p = 0;
  for (int k = 0; k < o; k++) priv[p++] = obs[k];
  for (int k = 0; k < 3; k++) priv[p++] = gyro[k];
  for (int k = 0; k < 3; k++) priv[p++] = acc[k];
  for (int k = 0; k < 3; k++) priv[p++] = grav[k];
  for (int k = 0; k < 3; k++) priv[p++] = sd[cfg->sens_local_linvel + k];
  for (int k = 0; k < 3; k++) priv[p++] = sd[cfg->sens_global_angvel + k];
  for (int a = 0; a < nu; a++) priv[p++] = jangle[a] - cfg->default_actuator[a];
  for (int a = 0; a < nu; a++) priv[p++] = jvel[a];
  priv[p++] = d->qpos[2];
  for (int a = 0; a < nu; a++) priv[p++] = d->actuator_force[a];
  priv[p++] = contact[0];
  priv[p++] = contact[1];
  for (int k = 0; k < 3; k++) priv[p++] = sd[cfg->sens_left_foot_linvel + k];
  for (int k = 0; k < 3; k++) priv[p++] = sd[cfg->sens_right_foot_linvel + k];
  priv[p++] = fs[L->feet_air_time];
  priv[p++] = fs[L->feet_air_time + 1];
  if (L->imitation)
    for (int k = 0; k < 40; k++) priv[p++] = fs[L->ref_motion + k];
  if (joystick) {
    priv[p++] = 0; /* imitation_i, filled by caller */
    priv[p++] = fs[L->imitation_phase];
    priv[p++] = fs[L->imitation_phase + 1];
  }
}

static void load_data(const duck_layout* L, const double* fs, oracle_data* d) {
  memset(d, 0, sizeof(*d));
  memcpy(d->qpos, fs + L->qpos, sizeof(double) * L->nq);
  memcpy(d->qvel, fs + L->qvel, sizeof(double) * L->nv);
  memcpy(d->qacc_warmstart, fs + L->qacc_warmstart, sizeof(double) * L->nv);
  memcpy(d->ctrl, fs + L->ctrl, sizeof(double) * L->nu);
}
static void store_data(const duck_layout* L, const oracle_data* d, double* fs) {
  memcpy(fs + L->qpos, d->qpos, sizeof(double) * L->nq);
  memcpy(fs + L->qvel, d->qvel, sizeof(double) * L->nv);
  memcpy(fs + L->qacc_warmstart, d->qacc_warmstart, sizeof(double) * L->nv);
  memcpy(fs + L->ctrl, d->ctrl, sizeof(double) * L->nu);
}

/* Joystick.reset (joystick.py:206-321); Standing.reset (standing.py:200-321) differs in the
 * base velocity range and the initial motor targets */
int oracle_env_reset(const oracle_model* m, const duck_env_config* cfg, const duck_refmotion* ref, uint64_t seed,
                     int64_t env_id, double* fs, int32_t* is, double* obs, double* priv) {
  duck_layout L = duck_layout_make(m->nq, m->nv, m->nu, cfg->use_imitation, cfg->task);
  int nu = m->nu;
  memset(fs, 0, sizeof(double) * L.nfloat);
  memset(is, 0, sizeof(int32_t) * L.nint);
  rng_t r;
  derive_key(seed, env_id, KEY_TAG_ENV, r.key);
  r.ctr = 0;
  oracle_data d;
  memset(&d, 0, sizeof(d));
  for (int i = 0; i < m->nq; i++) d.qpos[i] = cfg->init_qpos[i];
  d.qpos[0] += rng_uniform(&r, RSLOT_DXY + 0, -0.05, 0.05);
  d.qpos[1] += rng_uniform(&r, RSLOT_DXY + 1, -0.05, 0.05);
  double yaw = rng_uniform(&r, RSLOT_YAW, -3.14, 3.14);
  double zax[3] = {0, 0, 1}, qy[4];
  axis_angle_quat(qy, zax, yaw);
  quat_mul(d.qpos + 3, d.qpos + 3, qy);
  for (int a = 0; a < nu; a++) d.qpos[cfg->actuator_qposadr[a]] *= rng_uniform(&r, RSLOT_QSCALE + a, 0.5, 1.5);
  double vr = L.task == DUCK_TASK_STANDING ? 0.5 : 0.05;
  for (int k = 0; k < 6; k++) d.qvel[k] = rng_uniform(&r, RSLOT_QVEL + k, -vr, vr);
  for (int a = 0; a < nu; a++) d.ctrl[a] = d.qpos[cfg->actuator_qposadr[a]];
  oracle_forward(m, &d); /* mjx_env.init -> mjx.forward */
  double cmd[7];
  sample_command(cfg, &r, RSLOT_CMD, cmd);
  double push_interval = rng_uniform(&r, RSLOT_PUSH, cfg->push_interval_range[0], cfg->push_interval_range[1]);
  is[L.push_interval] = (int32_t)nearbyint((double)(float)(push_interval / cfg->ctrl_dt));
  is[L.rng_key] = (int32_t)r.key[0];
  is[L.rng_key + 1] = (int32_t)r.key[1];
  is[L.rng_ctr] = 1;
  for (int k = 0; k < 7; k++) fs[L.command + k] = cmd[k];
  for (int a = 0; a < nu; a++) fs[L.motor_targets + a] = L.task == DUCK_TASK_STANDING ? 0.0 : cfg->default_actuator[a];
  if (L.imitation) oracle_reference_motion(ref, cmd[0], cmd[1], cmd[2], 0, fs + L.ref_motion);
  store_data(&L, &d, fs);
  double contact[2] = {geoms_colliding(&d, cfg->left_foot_geom, cfg->floor_geom),
                       geoms_colliding(&d, cfg->right_foot_geom, cfg->floor_geom)};
  get_obs(m, cfg, &L, &d, fs, &r, RSLOT_OBS, contact, obs, priv);
  if (L.task == DUCK_TASK_JOYSTICK) priv[L.priv_size - 3] = is[L.imitation_i];
  /* AutoReset first-state snapshot */
  memcpy(fs + L.first_qpos, fs + L.qpos, sizeof(double) * m->nq);
  memcpy(fs + L.first_qvel, fs + L.qvel, sizeof(double) * m->nv);
  memcpy(fs + L.first_qacc_warmstart, fs + L.qacc_warmstart, sizeof(double) * m->nv);
  memcpy(fs + L.first_ctrl, fs + L.ctrl, sizeof(double) * nu);
  memcpy(fs + L.first_obs, obs, sizeof(double) * L.obs_size);
  memcpy(fs + L.first_priv, priv, sizeof(double) * L.priv_size);
  return 0;
}

/* test aid (tests/teacher_forcing.py substep_trace): when set, oracle_env_step on this thread records every substep's
 * input state (qpos, qvel, qacc_warmstart, ctrl) into the buffer, n_substeps records */
static _Thread_local double* g_trace;
void oracle_set_trace(double* buf) { g_trace = buf; }

/* Joystick.step (joystick.py:323-481) + EpisodeWrapper + BraxAutoResetWrapper when cfg->auto_reset */
int oracle_env_step(const oracle_model* m, const duck_env_config* cfg, const duck_refmotion* ref, double* fs,
                    int32_t* is, const double* action, double* obs, double* priv, double* reward_out,
                    double* done_out, oracle_data* d_out) {
  duck_layout L = duck_layout_make(m->nq, m->nv, m->nu, cfg->use_imitation, cfg->task);
  int nu = m->nu;
  double dt = cfg->ctrl_dt;
  if (cfg->auto_reset) {
    if (fs[L.done] != 0) is[L.ep_steps] = 0;
  }
  rng_t r;
  r.key[0] = (uint32_t)is[L.rng_key];
  r.key[1] = (uint32_t)is[L.rng_key + 1];
  r.ctr = (uint32_t)is[L.rng_ctr];
  /* imitation phase (:325-355) */
  if (L.imitation) {
    int nb = ref->nb_steps_in_period;
    is[L.imitation_i] = (is[L.imitation_i] + 1) % nb;
    double ph = (double)(float)((double)is[L.imitation_i] / nb) * 2 * PI;
    fs[L.imitation_phase] = cos(ph);
    fs[L.imitation_phase + 1] = sin(ph);
    oracle_reference_motion(ref, fs[L.command], fs[L.command + 1], fs[L.command + 2], is[L.imitation_i],
                            fs + L.ref_motion);
  } else {
    is[L.imitation_i] = 0;
  }
  /* action delay (:362-376) */
  double* ah = fs + L.action_history;
  for (int k = 3 * nu - 1; k >= nu; k--) ah[k] = ah[k - nu];
  for (int a = 0; a < nu; a++) ah[a] = action[a];
  int didx = rng_randint(&r, SLOT_ACTION_DELAY, cfg->action_min_delay, cfg->action_max_delay);
  const double* adel = ah + didx * nu;
  /* push (:381-400) */
  double theta = rng_uniform(&r, SLOT_PUSH_THETA, 0.0, 2 * PI);
  double mag = rng_uniform(&r, SLOT_PUSH_MAG, cfg->push_magnitude_range[0], cfg->push_magnitude_range[1]);
  /* jp.mod by a zero interval returns the dividend (XLA): no push */
  double gate = (is[L.push_interval] != 0 && (is[L.push_step] + 1) % is[L.push_interval] == 0) ? 1.0 : 0.0;
  double push[2] = {cos(theta) * gate * cfg->push_enable, sin(theta) * gate * cfg->push_enable};
  oracle_data dd, *d = d_out ? d_out : &dd;
  load_data(&L, fs, d);
  d->qvel[0] += push[0] * mag;
  d->qvel[1] += push[1] * mag;
  /* motor targets (:404-417) */
  double mt[DUCK_MAXU];
  for (int a = 0; a < nu; a++) {
    mt[a] = cfg->default_actuator[a] + adel[a] * cfg->action_scale;
    if (cfg->use_motor_speed_limits) {
      double prev = fs[L.motor_targets + a], lim = cfg->max_motor_velocity * dt;
      mt[a] = fmin(fmax(mt[a], prev - lim), prev + lim);
    }
    d->ctrl[a] = mt[a];
  }
  /* physics (:420) */
  for (int s = 0; s < cfg->n_substeps; s++) {
    if (g_trace) { /* test aid: each substep's input state */
      double* t = g_trace + (size_t)s * (m->nq + 2 * m->nv + nu);
      memcpy(t, d->qpos, sizeof(double) * m->nq);
      memcpy(t + m->nq, d->qvel, sizeof(double) * m->nv);
      memcpy(t + m->nq + m->nv, d->qacc_warmstart, sizeof(double) * m->nv);
      memcpy(t + m->nq + 2 * m->nv, d->ctrl, sizeof(double) * nu);
    }
    oracle_forward(m, d);
    euler(m, d);
  }
  for (int a = 0; a < nu; a++) fs[L.motor_targets + a] = mt[a];
  /* contacts and feet bookkeeping (:424-435) */
  double contact[2] = {geoms_colliding(d, cfg->left_foot_geom, cfg->floor_geom),
                       geoms_colliding(d, cfg->right_foot_geom, cfg->floor_geom)};
  for (int k = 0; k < 2; k++) {
    fs[L.feet_air_time + k] += dt;
    int site = k == 0 ? cfg->left_foot_site : cfg->right_foot_site;
    fs[L.swing_peak + k] = fmax(fs[L.swing_peak + k], d->site_xpos[site][2]);
  }
  store_data(&L, d, fs);
  get_obs(m, cfg, &L, d, fs, &r, 0, contact, obs, priv);
  if (L.task == DUCK_TASK_JOYSTICK) priv[L.priv_size - 3] = is[L.imitation_i];
  /* termination (:483-485) */
  int nan = 0;
  for (int i = 0; i < m->nq; i++) nan |= isnan(d->qpos[i]);
  for (int i = 0; i < m->nv; i++) nan |= isnan(d->qvel[i]);
  double done = (d->sensordata[cfg->sens_upvector + 2] < 0.0 || nan) ? 1.0 : 0.0;
  /* rewards (:440-447, :622-669) */
  double jq[DUCK_MAXU], jqd[DUCK_MAXU], la[DUCK_MAXU], act[DUCK_MAXU];
  for (int a = 0; a < nu; a++) {
    jq[a] = d->qpos[cfg->actuator_qposadr[a]];
    jqd[a] = d->qvel[cfg->actuator_qveladr[a]];
    la[a] = fs[L.last_act + a];
    act[a] = action[a];
  }
  double rr[5], cmd[7], q0[DUCK_MAXU];
  for (int k = 0; k < 7; k++) cmd[k] = fs[L.command + k];
  for (int a = 0; a < nu; a++) q0[a] = cfg->default_actuator[a];
  oracle_rewards(cmd, d->sensordata + cfg->sens_local_linvel, d->sensordata + cfg->sens_gyro, d->actuator_force, act,
                 la, jq, jqd, q0, nu, cfg->tracking_sigma, rr);
  double imit = 0;
  if (L.imitation) {
    double c2[2] = {contact[0], contact[1]};
    imit = oracle_reward_imitation(d->qpos, d->qvel, jq, jqd, c2, fs + L.ref_motion, cmd, nu);
  }
  double terms[7] = {rr[0] * cfg->scale_tracking_lin_vel, rr[1] * cfg->scale_tracking_ang_vel,
                     rr[2] * cfg->scale_torques, rr[3] * cfg->scale_action_rate, 1.0 * cfg->scale_alive,
                     imit * cfg->scale_imitation, rr[4] * cfg->scale_stand_still};
  double scales[7] = {cfg->scale_tracking_lin_vel, cfg->scale_tracking_ang_vel, cfg->scale_torques,
                      cfg->scale_action_rate, cfg->scale_alive, cfg->scale_imitation, cfg->scale_stand_still};
  if (L.task == DUCK_TASK_STANDING) {
    /* Standing._get_reward (standing.py:584-606) */
    double st[6];
    oracle_standing_rewards(cmd, d->sensordata + cfg->sens_upvector, d->actuator_force, act, la, jq, jqd, q0, nu, st);
    double ss[7] = {cfg->scale_orientation, cfg->scale_torques, cfg->scale_action_rate, cfg->scale_alive,
                    cfg->scale_stand_still, cfg->scale_head_pos, 0.0};
    for (int k = 0; k < 7; k++) {
      scales[k] = ss[k];
      terms[k] = k < 6 ? st[k] * ss[k] : 0.0;
    }
  }
  double sum = 0;
  for (int k = 0; k < 7; k++) sum += terms[k];
  double reward = fmin(fmax(sum * dt, 0.0), 10000.0);
  /* info bookkeeping (:449-477) */
  fs[L.push] = push[0];
  fs[L.push + 1] = push[1];
  is[L.step] += 1;
  is[L.push_step] += 1;
  for (int a = 0; a < nu; a++) {
    fs[L.last_last_last_act + a] = fs[L.last_last_act + a];
    fs[L.last_last_act + a] = fs[L.last_act + a];
    fs[L.last_act + a] = action[a];
  }
  if (is[L.step] > 500) {
    sample_command(cfg, &r, SLOT_CMD, cmd);
    for (int k = 0; k < 7; k++) fs[L.command + k] = cmd[k];
  }
  if (done != 0 || is[L.step] > 500) is[L.step] = 0;
  for (int k = 0; k < 2; k++) {
    fs[L.feet_air_time + k] *= contact[k] ? 0.0 : 1.0;
    fs[L.last_contact + k] = contact[k];
    fs[L.swing_peak + k] *= contact[k] ? 0.0 : 1.0;
  }
  for (int k = 0; k < 7; k++) fs[L.metrics + k] = scales[k] > 0 ? terms[k] : -terms[k];
  fs[L.metrics + DUCK_M_SWING_PEAK] = 0.5 * (fs[L.swing_peak] + fs[L.swing_peak + 1]);
  is[L.rng_ctr] = (int32_t)(r.ctr + 1);
  /* training wrappers */
  double trunc = 0;
  if (cfg->auto_reset) {
    is[L.ep_steps] += 1;
    if (is[L.ep_steps] >= cfg->episode_length) { trunc = 1.0 - done; done = 1.0; }
    if (done != 0) {
      memcpy(fs + L.qpos, fs + L.first_qpos, sizeof(double) * m->nq);
      memcpy(fs + L.qvel, fs + L.first_qvel, sizeof(double) * m->nv);
      memcpy(fs + L.qacc_warmstart, fs + L.first_qacc_warmstart, sizeof(double) * m->nv);
      memcpy(fs + L.ctrl, fs + L.first_ctrl, sizeof(double) * nu);
      memcpy(obs, fs + L.first_obs, sizeof(double) * L.obs_size);
      memcpy(priv, fs + L.first_priv, sizeof(double) * L.priv_size);
    }
  }
  fs[L.reward] = reward;
  fs[L.done] = done;
  fs[L.truncation] = trunc;
  if (reward_out) *reward_out = reward;
  if (done_out) *done_out = done;
  return 0;
}

/* ------------------------------------------------------------------------------------ */
/* batched entry points (CPU baseline)                                                  */
/* ------------------------------------------------------------------------------------ */

int oracle_batch_reset(const oracle_model* const* models, int n_models, const duck_env_config* cfg,
                       const duck_refmotion* ref, int n, uint64_t seed, int64_t env_offset, double* fstate,
                       int32_t* istate, double* obs, double* priv, int n_threads) {
  const oracle_model* m0 = models[0];
  duck_layout L = duck_layout_make(m0->nq, m0->nv, m0->nu, cfg->use_imitation, cfg->task);
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(static)
#endif
  for (int e = 0; e < n; e++) {
    const oracle_model* m = models[n_models == 1 ? 0 : e];
    double fs[1024];
    int32_t is[16];
    oracle_env_reset(m, cfg, ref, seed, env_offset + e, fs, is, obs + (size_t)e * L.obs_size,
                     priv + (size_t)e * L.priv_size);
    for (int k = 0; k < L.nfloat; k++) fstate[(size_t)k * n + e] = fs[k];
    for (int k = 0; k < L.nint; k++) istate[(size_t)k * n + e] = is[k];
  }
  return 0;
}

int oracle_batch_step(const oracle_model* const* models, int n_models, const duck_env_config* cfg,
                      const duck_refmotion* ref, int n, double* fstate, int32_t* istate, const double* actions,
                      double* obs, double* priv, double* reward, double* done, int n_threads) {
  const oracle_model* m0 = models[0];
  duck_layout L = duck_layout_make(m0->nq, m0->nv, m0->nu, cfg->use_imitation, cfg->task);
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(static)
#endif
  for (int e = 0; e < n; e++) {
    const oracle_model* m = models[n_models == 1 ? 0 : e];
    double fs[1024];
    int32_t is[16];
    for (int k = 0; k < L.nfloat; k++) fs[k] = fstate[(size_t)k * n + e];
    for (int k = 0; k < L.nint; k++) is[k] = istate[(size_t)k * n + e];
    oracle_env_step(m, cfg, ref, fs, is, actions + (size_t)e * m->nu, obs + (size_t)e * L.obs_size,
                    priv + (size_t)e * L.priv_size, reward + e, done + e, NULL);
    for (int k = 0; k < L.nfloat; k++) fstate[(size_t)k * n + e] = fs[k];
    for (int k = 0; k < L.nint; k++) istate[(size_t)k * n + e] = is[k];
  }
  return 0;
}
