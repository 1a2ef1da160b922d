// duck_capi.hip — the C ABI of libduck.so (include/duck.h): argument checks, handle
// lifetime, device uploads of the shared tables, and dispatch to the compiled model
// variant (variant_*.hip). Every entry returns DUCK_OK or a negative code with a
// thread-local message; no entry allocates, synchronises or throws on the step path.
#include "duck_common.h"

// the compiled model variants of this library (codegen.variant_registry; generated/ for libduck.so,
// a per-model build directory for a library compiled for another model, native.model_library)
#define DUCK_VARIANT(name) const VariantOps* duck_variant_##name();
#include "duck_variants.inc"
#undef DUCK_VARIANT
#define DUCK_VARIANT(name) duck_variant_##name(),
static const VariantOps* const kVariants[] = {
#include "duck_variants.inc"
};
#undef DUCK_VARIANT
static constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

static thread_local std::string g_err;
int duck_fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// a kernel of this handle set the sticky device error word (DUCK_DEVERR_*): every later launch on the
// handle is refused until duck_device_error(clear) -- the state the failed launch wrote is not valid
static int device_error_fail(const duck_sim* s) {
  const unsigned w = *s->err_h;
  std::string why;
  if (w & DUCK_DEVERR_LAT_TIMEOUT)
    why += "a latency-kernel cross-wave event wait timed out (broken stage schedule); the envs of that "
           "workgroup were written with NaN qpos";
  return duck_fail(DUCK_EDEVICE, "device error word 0x" + [&] {
    char b[16];
    snprintf(b, sizeof(b), "%x", w);
    return std::string(b);
  }() + " set by an earlier launch: " + why);
}

// FNV-1a 64 over the model values a compiled variant bakes (duck_model_fingerprint)
namespace {
struct Fnv {
  uint64_t h = 1469598103934665603ull;
  void bytes(const void* p, size_t n) {
    const unsigned char* c = (const unsigned char*)p;
    for (size_t i = 0; i < n; i++) { h ^= c[i]; h *= 1099511628211ull; }
  }
  void i32(const int* a, int n) {
    for (int i = 0; i < n; i++) { int32_t v = a ? a[i] : 0; bytes(&v, 4); }
  }
  void f32(const double* a, int n) {  // the kernels bake float32: hash what they see
    for (int i = 0; i < n; i++) { float v = a ? (float)a[i] : 0.0f; bytes(&v, 4); }
  }
};
}  // namespace

extern "C" {

uint64_t duck_model_fingerprint(const duck_model_desc* m) {
  if (!m) return 0;
  Fnv f;
  const int nb = m->nbody, nj = m->njnt, nv = m->nv, ng = m->ngeom, np = m->npair, ns = m->nsite, nu = m->nu;
  const int sizes[] = {m->nq, m->nv, m->nu, m->nbody, m->njnt, m->ngeom, m->nsite, m->nsensor, m->nsensordata,
                       m->npair, m->iterations, m->ls_iterations, m->eulerdamp};
  f.i32(sizes, 13);
  const double opt[] = {m->timestep, m->gravity[0], m->gravity[1], m->gravity[2], m->impratio, m->tolerance,
                        m->ls_tolerance, m->meaninertia};
  f.f32(opt, 8);
  f.i32(m->body_parentid, nb); f.i32(m->body_rootid, nb); f.i32(m->body_weldid, nb); f.i32(m->body_jntnum, nb);
  f.i32(m->body_jntadr, nb); f.i32(m->body_dofnum, nb); f.i32(m->body_dofadr, nb);
  f.f32(m->body_pos, 3 * nb); f.f32(m->body_quat, 4 * nb); f.f32(m->body_ipos, 3 * nb); f.f32(m->body_iquat, 4 * nb);
  f.f32(m->body_mass, nb); f.f32(m->body_inertia, 3 * nb); f.f32(m->body_invweight0, 2 * nb);
  f.i32(m->jnt_type, nj); f.i32(m->jnt_qposadr, nj); f.i32(m->jnt_dofadr, nj); f.i32(m->jnt_bodyid, nj);
  f.i32(m->jnt_limited, nj);
  f.f32(m->jnt_pos, 3 * nj); f.f32(m->jnt_axis, 3 * nj); f.f32(m->jnt_range, 2 * nj); f.f32(m->jnt_margin, nj);
  f.f32(m->jnt_solref, 2 * nj); f.f32(m->jnt_solimp, 5 * nj);
  f.i32(m->dof_bodyid, nv); f.i32(m->dof_jntid, nv); f.i32(m->dof_parentid, nv);
  f.f32(m->dof_armature, nv); f.f32(m->dof_damping, nv); f.f32(m->dof_frictionloss, nv); f.f32(m->dof_invweight0, nv);
  f.f32(m->dof_solref, 2 * nv); f.f32(m->dof_solimp, 5 * nv);
  f.i32(m->geom_type, ng); f.i32(m->geom_bodyid, ng); f.i32(m->geom_dataid, ng);
  f.f32(m->geom_pos, 3 * ng); f.f32(m->geom_quat, 4 * ng); f.f32(m->geom_rbound, ng); f.f32(m->geom_size, 3 * ng);
  f.i32(m->pair_geom1, np); f.i32(m->pair_geom2, np); f.i32(m->pair_condim, np);
  f.f32(m->pair_friction, 5 * np); f.f32(m->pair_solref, 2 * np); f.f32(m->pair_solimp, 5 * np);
  f.f32(m->pair_margin, np);
  const int hull[] = {m->hull_nvert, m->hull_nface, m->hull_nedge, m->hfield_nrow, m->hfield_ncol};
  f.i32(hull, 5);
  f.f32(m->hull_vert, 3 * m->hull_nvert); f.f32(m->hull_face_normal, 3 * m->hull_nface);
  f.f32(m->hull_face_offset, m->hull_nface); f.i32(m->hull_edge, 2 * m->hull_nedge);
  f.f32(m->hfield_size, 4);  // the elevation itself is uploaded by duck_create, not baked
  f.i32(m->site_bodyid, ns); f.f32(m->site_pos, 3 * ns); f.f32(m->site_quat, 4 * ns);
  f.i32(m->actuator_trnid, nu); f.i32(m->actuator_ctrllimited, nu); f.i32(m->actuator_forcelimited, nu);
  f.f32(m->actuator_kp, nu); f.f32(m->actuator_kv, nu); f.f32(m->actuator_gear, nu);
  f.f32(m->actuator_ctrlrange, 2 * nu); f.f32(m->actuator_forcerange, 2 * nu);
  f.i32(m->sensor_type, m->nsensor); f.i32(m->sensor_objid, m->nsensor); f.i32(m->sensor_adr, m->nsensor);
  f.i32(m->sensor_dim, m->nsensor);
  f.f32(m->qpos0, m->nq);
  return f.h;
}

int duck_version(void) { return DUCK_VERSION; }

#ifndef DUCK_BUILD_ID
#define DUCK_BUILD_ID "unknown"
#endif
const char* duck_build_id(void) { return DUCK_BUILD_ID; }

int duck_model_supported(const duck_model_desc* model) {
  if (!model) return 0;
  for (int i = 0; i < kNumVariants; i++)
    if (kVariants[i]->matches(model)) return 1;
  return 0;
}
const char* duck_last_error(void) { return g_err.c_str(); }

int duck_layout_get(int nq, int nv, int nu, int imitation, int task, duck_layout* out) {
  if (!out) return duck_fail(DUCK_EINVAL, "null out");
  *out = duck_layout_make(nq, nv, nu, imitation, task);
  return DUCK_OK;
}

int duck_aux_size(const duck_sim* sim) {
  if (!sim) return duck_fail(DUCK_EINVAL, "null sim");
  return kVariants[sim->variant]->aux_size();
}

void duck_destroy(duck_sim* s) {
  if (!s) return;
  if (s->frames_d) (void)hipFree(s->frames_d);
  if (s->hfield_d) (void)hipFree(s->hfield_d);
  if (s->err_h) (void)hipHostFree((void*)s->err_h);
  delete s;
}

int duck_create(const duck_model_desc* model, const duck_env_config* cfg, const duck_refmotion* ref, int device,
                duck_sim** out) {
  g_err.clear();
  if (!model || !cfg || !out) return duck_fail(DUCK_EINVAL, "null argument");
  int v = -1;
  for (int i = 0; i < kNumVariants && v < 0; i++)
    if (kVariants[i]->matches(model)) v = i;
  if (v < 0)
    return duck_fail(DUCK_EUNSUPPORTED,
                     "no kernel of this library is compiled for this model (duck_model_fingerprint differs); "
                     "compile one with native.model_library / codegen");
  if (cfg->use_imitation && !ref) return duck_fail(DUCK_EINVAL, "use_imitation requires a reference-motion table");
  if (cfg->n_substeps < 1 || cfg->action_max_delay < 1 || cfg->action_max_delay > 3)
    return duck_fail(DUCK_EINVAL, "bad config (n_substeps >= 1, 1 <= action_max_delay <= 3)");
  // the throughput kernel must fit; a latency split that does not is simply not compiled (lds 0)
  if (kVariants[v]->lds_bytes() > 160 * 1024) return duck_fail(DUCK_EUNSUPPORTED, "per-workgroup LDS over 160 KiB");
  // the elevation is uploaded here, not baked (the fingerprint covers nrow / ncol / size only)
  if (kVariants[v]->floor_type == 1 && (!model->hfield_data || model->hfield_nrow < 2 || model->hfield_ncol < 2))
    return duck_fail(DUCK_EINVAL, "height-field model without hfield_data [nrow >= 2][ncol >= 2]");
  HIPCHECK(hipSetDevice(device));
  duck_sim* s = new duck_sim();
  memset(s, 0, sizeof(*s));
  s->device = device;
  s->variant = v;
  s->step_mode = DUCK_STEP_AUTO;
  s->lat_ok = kVariants[v]->lds_bytes_lat() != 0;
  s->lat2_ok = kVariants[v]->lds_bytes_lat2() != 0;
  s->latx2_ok = kVariants[v]->lds_bytes_lat_x2() != 0;
  {
    hipError_t e = hipDeviceGetAttribute(&s->n_cu, hipDeviceAttributeMultiprocessorCount, device);
    if (e != hipSuccess) {
      delete s;
      return duck_fail(DUCK_EHIP, std::string("hipDeviceGetAttribute: ") + hipGetErrorString(e));
    }
  }
  {
    // the sticky device error word: host memory the kernels write through their device mapping, so
    // that the next call reads it without synchronising (duck_device_error)
    void* p = nullptr;
    hipError_t e = hipHostMalloc(&p, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&s->err_d, p, 0);
    if (e != hipSuccess) {
      if (p) (void)hipHostFree(p);
      delete s;
      return duck_fail(DUCK_EHIP, std::string("device error word: ") + hipGetErrorString(e));
    }
    s->err_h = (volatile unsigned*)p;
    *s->err_h = 0;
  }
  s->cfg = *cfg;
  s->nq = model->nq; s->nv = model->nv; s->nu = model->nu;
  s->lay = duck_layout_make(model->nq, model->nv, model->nu, cfg->use_imitation, cfg->task);
  s->drl = duck_dr_layout_make(model->nbody, model->nu);
  if (ref) {
    if (ref->n_dim != 40 || ref->n_dx > 16 || ref->n_dy > 16 || ref->n_dtheta > 16 || ref->nb_steps_in_period < 1 ||
        !ref->frames) {
      duck_destroy(s);  // frees the pinned error word allocated above
      return duck_fail(DUCK_EINVAL, "reference-motion table must be [<=16][<=16][<=16][nb][40] frames");
    }
    s->ref.n_dx = ref->n_dx; s->ref.n_dy = ref->n_dy; s->ref.n_dtheta = ref->n_dtheta;
    s->ref.n_dim = ref->n_dim; s->ref.n_coef = ref->n_coef; s->ref.nb = ref->nb_steps_in_period;
    memcpy(s->ref.dxs, ref->dxs, sizeof(ref->dxs)); memcpy(s->ref.dys, ref->dys, sizeof(ref->dys));
    memcpy(s->ref.dthetas, ref->dthetas, sizeof(ref->dthetas));
    memcpy(s->ref.dx_range, ref->dx_range, 8); memcpy(s->ref.dy_range, ref->dy_range, 8);
    memcpy(s->ref.dtheta_range, ref->dtheta_range, 8);
    const size_t nbytes =
        sizeof(float) * (size_t)ref->n_dx * ref->n_dy * ref->n_dtheta * ref->nb_steps_in_period * ref->n_dim;
    hipError_t e = hipMalloc(&s->frames_d, nbytes);
    if (e == hipSuccess) e = hipMemcpy(s->frames_d, ref->frames, nbytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      duck_destroy(s);
      return duck_fail(DUCK_EHIP, std::string("reference table upload: ") + hipGetErrorString(e));
    }
  }
  if (kVariants[v]->floor_type == 1) {  // height field elevation, [nrow][ncol] in [0, 1]
    const size_t nn = (size_t)model->hfield_nrow * model->hfield_ncol;
    float* h = new float[nn];
    for (size_t i = 0; i < nn; i++) h[i] = (float)model->hfield_data[i];
    hipError_t e = hipMalloc(&s->hfield_d, nn * sizeof(float));
    if (e == hipSuccess) e = hipMemcpy(s->hfield_d, h, nn * sizeof(float), hipMemcpyHostToDevice);
    delete[] h;
    if (e != hipSuccess) {
      duck_destroy(s);
      return duck_fail(DUCK_EHIP, std::string("height field upload: ") + hipGetErrorString(e));
    }
  }
  *out = s;
  return DUCK_OK;
}

int duck_reset(duck_sim* s, int n, float* fstate, int32_t* istate, const uint8_t* mask, uint64_t seed,
               int64_t env_offset, const float* dr, float* obs, float* priv, void* stream) {
  g_err.clear();
  if (!s || n < 0 || !fstate || !istate || !obs || !priv) return duck_fail(DUCK_EINVAL, "bad argument");
  if (*s->err_h) return device_error_fail(s);
  if (n == 0) return DUCK_OK;
  HIPCHECK(hipSetDevice(s->device));
  return kVariants[s->variant]->reset(s, n, fstate, istate, mask, seed, env_offset, dr, obs, priv,
                                      (hipStream_t)stream);
}

int duck_step(duck_sim* s, int n, float* fstate, int32_t* istate, const float* dr, const float* action, float* obs,
              float* priv, float* reward, float* done, float* scratch, void* stream) {
  g_err.clear();
  if (!s || n < 0 || !fstate || !istate || !action || !obs || !priv || !reward || !done)
    return duck_fail(DUCK_EINVAL, "bad argument");
  if (*s->err_h) return device_error_fail(s);
  if (n == 0) return DUCK_OK;
  HIPCHECK(hipSetDevice(s->device));
  return kVariants[s->variant]->step(s, n, fstate, istate, dr, action, obs, priv, reward, done, scratch,
                                     (hipStream_t)stream);
}

int duck_randomize(duck_sim* s, int n, float* dr, uint64_t seed, int64_t env_offset, void* stream) {
  g_err.clear();
  if (!s || n < 0 || !dr) return duck_fail(DUCK_EINVAL, "bad argument");
  if (n == 0) return DUCK_OK;
  HIPCHECK(hipSetDevice(s->device));
  return kVariants[s->variant]->randomize(s, n, dr, seed, env_offset, (hipStream_t)stream);
}

int duck_physics_step(duck_sim* s, int n, float* qpos, float* qvel, float* warm, const float* ctrl, const float* dr,
                      int nsub, float* aux, float* scratch, void* stream) {
  g_err.clear();
  if (!s || n < 0 || !qpos || !qvel || !warm || !ctrl || nsub < 0) return duck_fail(DUCK_EINVAL, "bad argument");
  if (*s->err_h) return device_error_fail(s);
  if (n == 0) return DUCK_OK;
  HIPCHECK(hipSetDevice(s->device));
  return kVariants[s->variant]->physics(s, n, qpos, qvel, warm, ctrl, dr, nsub, aux, scratch, (hipStream_t)stream);
}

int duck_set_step_mode(duck_sim* s, int mode) {
  g_err.clear();
  if (!s || mode < DUCK_STEP_AUTO || mode > DUCK_STEP_LATENCY_X2) return duck_fail(DUCK_EINVAL, "bad argument");
  if ((mode == DUCK_STEP_LATENCY && !s->lat_ok) || (mode == DUCK_STEP_PAIRED && !s->lat2_ok) ||
      (mode == DUCK_STEP_LATENCY_X2 && !s->latx2_ok))
    return duck_fail(DUCK_EUNSUPPORTED, "that step kernel is not compiled for this model (LDS budget, or "
                                        "LATENCY_X2 outside the plane-floor scenes; AUTO skips it)");
  s->step_mode = mode;
  return DUCK_OK;
}

int duck_step_kernel_for(const duck_sim* s, int n) {
  if (!s || n < 0) return duck_fail(DUCK_EINVAL, "bad argument");
  return step_kernel_choice(s, n);
}

int duck_device_error(duck_sim* s, unsigned* out, int clear) {
  if (!s || !out) return duck_fail(DUCK_EINVAL, "bad argument");
  *out = *s->err_h;
  if (clear) *s->err_h = 0;
  return DUCK_OK;
}

int duck_debug_lat_timeouts(const duck_sim* s, unsigned* out, int reset) {
  if (!s || !out) return duck_fail(DUCK_EINVAL, "bad argument");
  HIPCHECK(hipSetDevice(s->device));
  return kVariants[s->variant]->lat_timeouts(out, reset);
}

// debug: per-stage cycle counters of a -DDUCK_STAGE_PROF build (DUCK_EUNSUPPORTED otherwise)
int duck_debug_stage_cycles(const duck_sim* s, unsigned long long* out, int reset) {
  if (!s || !out) return duck_fail(DUCK_EINVAL, "bad argument");
  return kVariants[s->variant]->stage_cycles(out, reset);
}

}  // extern "C"
