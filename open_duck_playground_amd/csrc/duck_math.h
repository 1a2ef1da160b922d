// duck_math.h — small fp32 device helpers for the per-env (one env per lane) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DK __device__ __forceinline__

DK float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
DK void cross3(float* r, const float* a, const float* b) {
  float t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
DK void mulmv3(float* r, const float* M, const float* v) {
  float t0 = M[0] * v[0] + M[1] * v[1] + M[2] * v[2];
  float t1 = M[3] * v[0] + M[4] * v[1] + M[5] * v[2];
  float t2 = M[6] * v[0] + M[7] * v[1] + M[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
DK void mulmtv3(float* r, const float* M, const float* v) {
  float t0 = M[0] * v[0] + M[3] * v[1] + M[6] * v[2];
  float t1 = M[1] * v[0] + M[4] * v[1] + M[7] * v[2];
  float t2 = M[2] * v[0] + M[5] * v[1] + M[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
DK void mulmm3(float* r, const float* A, const float* B) {
  float t[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = t[i];
}
DK void qmul(float* r, const float* a, const float* b) {
  float t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  float t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  float t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  float t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
DK void qnormalize(float* q) {
  float n2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  if (n2 < 1e-30f) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  float s = 1.0f / sqrtf(n2);
  q[0] *= s; q[1] *= s; q[2] *= s; q[3] *= s;
}
DK void q2m(float* R, const float* q) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}
// MuJoCo com-based spatial algebra: motion/force = [angular; linear]
DK void mul_inert_vec(float* r, const float* I, const float* v) {
  r[0] = I[0] * v[0] + I[3] * v[1] + I[4] * v[2] - I[8] * v[4] + I[7] * v[5];
  r[1] = I[3] * v[0] + I[1] * v[1] + I[5] * v[2] + I[8] * v[3] - I[6] * v[5];
  r[2] = I[4] * v[0] + I[5] * v[1] + I[2] * v[2] - I[7] * v[3] + I[6] * v[4];
  r[3] = I[8] * v[1] - I[7] * v[2] + I[9] * v[3];
  r[4] = I[6] * v[2] - I[8] * v[0] + I[9] * v[4];
  r[5] = I[7] * v[0] - I[6] * v[1] + I[9] * v[5];
}
DK void cross_motion(float* r, const float* v, const float* u) {
  float r0 = -v[2] * u[1] + v[1] * u[2];
  float r1 = v[2] * u[0] - v[0] * u[2];
  float r2 = -v[1] * u[0] + v[0] * u[1];
  float r3 = -v[2] * u[4] + v[1] * u[5] - v[5] * u[1] + v[4] * u[2];
  float r4 = v[2] * u[3] - v[0] * u[5] + v[5] * u[0] - v[3] * u[2];
  float r5 = -v[1] * u[3] + v[0] * u[4] - v[4] * u[0] + v[3] * u[1];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}
DK void cross_force(float* r, const float* v, const float* f) {
  float r0 = -v[2] * f[1] + v[1] * f[2] - v[5] * f[4] + v[4] * f[5];
  float r1 = v[2] * f[0] - v[0] * f[2] + v[5] * f[3] - v[3] * f[5];
  float r2 = -v[1] * f[0] + v[0] * f[1] - v[4] * f[3] + v[3] * f[4];
  float r3 = -v[2] * f[4] + v[1] * f[5];
  float r4 = v[2] * f[3] - v[0] * f[5];
  float r5 = -v[1] * f[3] + v[0] * f[4];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}

// ---- threefry2x32, 20 rounds (Salmon et al. 2011; same cipher JAX's PRNG uses) ----
DK uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
DK void threefry2x32(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t& o0, uint32_t& o1) {
  const uint32_t k2 = 0x1BD11BDAu ^ k0 ^ k1;
  uint32_t x0 = c0 + k0, x1 = c1 + k1;
  const int R[8] = {13, 15, 26, 6, 17, 29, 16, 24};
#pragma unroll
  for (int r = 0; r < 20; r++) {
    x0 += x1;
    x1 = rotl32(x1, R[r % 8]);
    x1 ^= x0;
    if (r % 4 == 3) {
      const uint32_t s = (uint32_t)(r / 4 + 1);
      const uint32_t ks[3] = {k0, k1, k2};
      x0 += ks[s % 3];
      x1 += ks[(s + 1) % 3] + s;
    }
  }
  o0 = x0; o1 = x1;
}

struct Rng {
  uint32_t k0, k1, ctr;
  // slot -> 23-bit uniform in [0,1) (exact in fp32)
  DK float u(int slot) const {
    uint32_t a, b;
    threefry2x32(k0, k1, ctr, (uint32_t)(slot >> 1), a, b);
    uint32_t w = (slot & 1) ? b : a;
    return (float)(w >> 9) * (1.0f / 8388608.0f);
  }
  DK float uniform(int slot, float lo, float hi) const { return lo + (hi - lo) * u(slot); }
  DK int randint(int slot, int lo, int hi) const {
    int k = (int)floorf(u(slot) * (float)(hi - lo));
    return lo + (k > hi - lo - 1 ? hi - lo - 1 : k);
  }
};

// The first 64 slots of a step's stream drawn by the team in parallel (lane l runs the threefry
// blocks l and l + 16) and read back from LDS; later slots fall back to direct evaluation.
struct RngTab : Rng {
  static constexpr int N = 64;
  const __attribute__((address_space(3))) float* tab;
  DK float u(int slot) const { return slot < N ? tab[slot] : Rng::u(slot); }
  DK float uniform(int slot, float lo, float hi) const { return lo + (hi - lo) * u(slot); }
  DK int randint(int slot, int lo, int hi) const {
    int k = (int)floorf(u(slot) * (float)(hi - lo));
    return lo + (k > hi - lo - 1 ? hi - lo - 1 : k);
  }
  // fill tab[0..N) (team lane `lane` of 16 writes 4 entries)
  DK void fill(__attribute__((address_space(3))) float* t, int lane) const {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int j = lane + 16 * h;
      uint32_t a, b;
      threefry2x32(k0, k1, ctr, (uint32_t)j, a, b);
      t[2 * j] = (float)(a >> 9) * (1.0f / 8388608.0f);
      t[2 * j + 1] = (float)(b >> 9) * (1.0f / 8388608.0f);
    }
  }
};

DK void derive_key(uint64_t seed, int64_t env_id, uint32_t tag, uint32_t& k0, uint32_t& k1) {
  threefry2x32((uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)env_id, tag ^ (uint32_t)((uint64_t)env_id >> 32), k0,
               k1);
}
