// duck_common.h — shared declarations of the MI355X Open Duck kernels (host + device).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <string>

#include "../../include/duck.h"

#define DUCK_VERSION 100  // 0.1.0

// error reporting of the C ABI (duck_capi.hip)
int duck_fail(int code, const std::string& msg);
#define HIPCHECK(x)                                                                                   \
  do {                                                                                                \
    hipError_t _e = (x);                                                                              \
    if (_e != hipSuccess) return duck_fail(DUCK_EHIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

struct RefMeta {
  int n_dx, n_dy, n_dtheta, n_dim, n_coef, nb;
  float dxs[16], dys[16], dthetas[16];
  float dx_range[2], dy_range[2], dtheta_range[2];
};

// envs per latency-mode workgroup (duck_team.h LAT_WG; the host side of DUCK_STEP_AUTO)
constexpr int LAT_WG_HOST = 4;

// per-handle state (device pointers owned by the handle)
struct duck_sim {
  int device;
  int variant;
  duck_env_config cfg;
  duck_layout lay;
  duck_dr_layout drl;
  RefMeta ref;
  float* frames_d;
  float* hfield_d;
  int nq, nv, nu;
  int step_mode;  // DUCK_STEP_*
  int n_cu;       // compute units of the device (DUCK_STEP_AUTO)
  int lat_ok, lat2_ok;  // the latency / paired latency kernels are compiled for this model (TLay::FITS)
  int latx2_ok;         // the two-workgroups-per-CU latency kernel is (LatX2::PAYS)
  volatile unsigned* err_h;  // sticky device error word (DUCK_DEVERR_*), host-mapped pinned memory
  unsigned* err_d;           // its device mapping (KArgs::err)
};

// per-variant entry points, one table per compiled model variant (variant_*.hip)
struct VariantOps {
  const char* name;
  bool (*matches)(const duck_model_desc*);
  int (*aux_size)();
  size_t (*lds_bytes)();
  int floor_type;
  int (*reset)(duck_sim*, int n, float* fs, int32_t* is, const uint8_t* mask, uint64_t seed, int64_t env_offset,
               const float* dr, float* obs, float* priv, hipStream_t st);
  int (*step)(duck_sim*, int n, float* fs, int32_t* is, const float* dr, const float* action, float* obs,
              float* priv, float* reward, float* done, float* scratch, hipStream_t st);
  int (*randomize)(duck_sim*, int n, float* dr, uint64_t seed, int64_t env_offset, hipStream_t st);
  int (*physics)(duck_sim*, int n, float* qpos, float* qvel, float* warm, const float* ctrl, const float* dr,
                 int nsub, float* aux, float* scratch, hipStream_t st);
  int (*stage_cycles)(unsigned long long* out, int reset);
  int (*lat_timeouts)(unsigned* out, int reset);
  size_t (*lds_bytes_lat)();
  size_t (*lds_bytes_lat2)();
  size_t (*lds_bytes_lat_x2)();
};

// the step kernel duck_step launches for n envs (DUCK_STEP_THROUGHPUT / _LATENCY / _PAIRED /
// _LATENCY_X2): the mode asked for, or under AUTO the latency kernel while n <= 4 envs per CU, then
// while n <= 8 per CU the two-workgroups-per-CU latency kernel where the model has it (flat scenes)
// or else the paired latency kernel, else the throughput kernel; a split a model does not fit
// (lat_ok / lat2_ok / latx2_ok) is skipped
inline int step_kernel_choice(const duck_sim* s, int n) {
  if (s->step_mode != DUCK_STEP_AUTO) return s->step_mode;
  if (s->lat_ok && n <= LAT_WG_HOST * s->n_cu) return DUCK_STEP_LATENCY;
  if (n <= 2 * LAT_WG_HOST * s->n_cu) {
    if (s->latx2_ok) return DUCK_STEP_LATENCY_X2;
    if (s->lat2_ok) return DUCK_STEP_PAIRED;
  }
  return DUCK_STEP_THROUGHPUT;
}
