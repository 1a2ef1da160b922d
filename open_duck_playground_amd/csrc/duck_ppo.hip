// Learner-side kernels of the PPO outer loop (include/duck_ppo.h).
#include "duck_common.h"
#include "../../include/duck_ppo.h"

namespace {

// One thread per trajectory, walking time backwards; every [T][B] access is a coalesced row.
// The recursion is sequential in t, so the work per thread is T dependent FMAs over 5 loads:
// HBM-bound at 6 * 4 B in + 2 * 4 B out per (t, b).
__global__ __launch_bounds__(256) void gae_kernel(int T, int B, const float* __restrict__ trunc,
                                                  const float* __restrict__ term, const float* __restrict__ rew,
                                                  const float* __restrict__ val, const float* __restrict__ boot,
                                                  float lam, float disc, float* __restrict__ vs,
                                                  float* __restrict__ adv) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    float v_next = boot[b];   // v_{t+1}
    float vs_next = boot[b];  // vs_{t+1}
    float acc = 0.f;
    for (int t = T - 1; t >= 0; --t) {
        const size_t i = (size_t)t * B + b;
        const float keep = 1.f - trunc[i];
        const float cont = disc * (1.f - term[i]);
        const float r = rew[i], v = val[i];
        const float delta = (r + cont * v_next - v) * keep;
        acc = delta + cont * keep * lam * acc;
        const float vs_t = acc + v;
        adv[i] = (r + cont * vs_next - v) * keep;
        vs[i] = vs_t;
        v_next = v;
        vs_next = vs_t;
    }
}

}  // namespace

extern "C" int duck_gae(int T, int B, const float* truncation, const float* termination, const float* reward,
                        const float* value, const float* bootstrap, float lambda_, float discount, float* vs,
                        float* adv, void* stream) {
    if (T < 0 || B < 0) return duck_fail(DUCK_EINVAL, "duck_gae: negative size");
    if (T == 0 || B == 0) return DUCK_OK;
    if (!truncation || !termination || !reward || !value || !bootstrap || !vs || !adv)
        return duck_fail(DUCK_EINVAL, "duck_gae: null pointer");
    hipLaunchKernelGGL(gae_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, T, B, truncation,
                       termination, reward, value, bootstrap, lambda_, discount, vs, adv);
    HIPCHECK(hipGetLastError());
    return DUCK_OK;
}
