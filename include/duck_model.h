/* duck_model.h — flat model descriptor handed across the C ABI.
 *
 * Replaces the reference's compiled model objects:
 *   mujoco.MjModel  (playground/open_duck_mini_v2/base.py:53-56)
 *   mjx.Model       (base.py:61, mjx.put_model)
 * restricted to the fields the Joystick hot path reads. All arrays are host pointers,
 * row-major, float64 for reals and int32 for indices; the callee copies what it needs
 * during *_create and never keeps the pointers.
 */
#ifndef DUCK_MODEL_H_
#define DUCK_MODEL_H_

#ifdef __cplusplus
extern "C" {
#endif

#define DUCK_MAXBODY 20
#define DUCK_MAXJNT 32
#define DUCK_MAXQ 40
#define DUCK_MAXV 32
#define DUCK_MAXU 16
#define DUCK_MAXGEOM 64
#define DUCK_MAXSITE 8
#define DUCK_MAXSENSOR 16
#define DUCK_MAXSENSORDATA 64
#define DUCK_MAXPAIR 4
#define DUCK_MAXHULLV 32
#define DUCK_MAXHULLF 48
#define DUCK_MAXHULLE 64
#define DUCK_CON_PER_PAIR 4
#define DUCK_MAXCON (DUCK_MAXPAIR * DUCK_CON_PER_PAIR)

enum { DUCK_JNT_FREE = 0, DUCK_JNT_BALL = 1, DUCK_JNT_SLIDE = 2, DUCK_JNT_HINGE = 3 };
enum { DUCK_GEOM_PLANE = 0, DUCK_GEOM_HFIELD = 1, DUCK_GEOM_MESH = 7 };
enum {
  DUCK_SENS_GYRO = 0, DUCK_SENS_VELOCIMETER, DUCK_SENS_ACCELEROMETER, DUCK_SENS_FRAMEZAXIS,
  DUCK_SENS_FRAMEXAXIS, DUCK_SENS_FRAMELINVEL, DUCK_SENS_FRAMEANGVEL, DUCK_SENS_FRAMEPOS,
  DUCK_SENS_FRAMEQUAT
};

typedef struct duck_model_desc {
  /* sizes */
  int nq, nv, nu, nbody, njnt, ngeom, nsite, nsensor, nsensordata, npair;
  /* options (mjOption subset) */
  double timestep, gravity[3], impratio, tolerance, ls_tolerance, meaninertia;
  int iterations, ls_iterations, eulerdamp;
  /* bodies [nbody] */
  const int *body_parentid, *body_rootid, *body_weldid, *body_jntnum, *body_jntadr, *body_dofnum, *body_dofadr;
  const double *body_pos /*3*/, *body_quat /*4*/, *body_ipos /*3*/, *body_iquat /*4*/, *body_mass,
      *body_inertia /*3*/, *body_invweight0 /*2*/;
  /* joints [njnt] */
  const int *jnt_type, *jnt_qposadr, *jnt_dofadr, *jnt_bodyid, *jnt_limited;
  const double *jnt_pos /*3*/, *jnt_axis /*3*/, *jnt_range /*2*/, *jnt_margin, *jnt_solref /*2*/,
      *jnt_solimp /*5*/;
  /* dofs [nv] */
  const int *dof_bodyid, *dof_jntid, *dof_parentid;
  const double *dof_armature, *dof_damping, *dof_frictionloss, *dof_invweight0, *dof_solref /*2*/,
      *dof_solimp /*5*/;
  /* geoms [ngeom] */
  const int *geom_type, *geom_bodyid, *geom_dataid;
  const double *geom_pos /*3*/, *geom_quat /*4*/, *geom_rbound, *geom_size /*3*/;
  /* collision pairs [npair]: geom1 is the lower geom type (plane/hfield before mesh) */
  const int *pair_geom1, *pair_geom2, *pair_condim;
  const double *pair_friction /*5*/, *pair_solref /*2*/, *pair_solimp /*5*/, *pair_margin;
  /* convex hull of the (single) collision mesh, geom-local coordinates */
  int hull_nvert, hull_nface, hull_nedge;
  const double *hull_vert /*3*/, *hull_face_normal /*3*/, *hull_face_offset;
  const int *hull_edge /*2*/;
  /* height field (rough scenes); nrow = 0 when absent */
  int hfield_nrow, hfield_ncol;
  double hfield_size[4];
  const double *hfield_data; /* [nrow*ncol], elevation in [0,1], row 0 at -y */
  /* sites [nsite] */
  const int *site_bodyid;
  const double *site_pos /*3*/, *site_quat /*4*/;
  /* actuators [nu] (<position> servos: force = kp*(ctrl - q) - kv*qdot) */
  const int *actuator_trnid, *actuator_ctrllimited, *actuator_forcelimited;
  const double *actuator_kp, *actuator_kv, *actuator_gear, *actuator_ctrlrange /*2*/,
      *actuator_forcerange /*2*/;
  /* sensors [nsensor] */
  const int *sensor_type, *sensor_objid, *sensor_adr, *sensor_dim;
  /* qpos0 [nq] */
  const double *qpos0;
} duck_model_desc;

#ifdef __cplusplus
}
#endif
#endif /* DUCK_MODEL_H_ */
