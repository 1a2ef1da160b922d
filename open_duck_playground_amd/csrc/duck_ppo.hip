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


// Block-wide sum over the 1024 threads of one workgroup (wave DPP-free: LDS tree, 16 waves).
__device__ float block_sum(float v, float* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
    if (threadIdx.x < 64) {
        t = threadIdx.x < (blockDim.x >> 6) ? red[threadIdx.x] : 0.f;
        for (int o = 32; o > 0; o >>= 1) t += __shfl_down(t, o, 64);
        if (threadIdx.x == 0) red[0] = t;
    }
    __syncthreads();
    const float r = red[0];
    __syncthreads();
    return r;
}

// GAE straight from the rollout fields, with the advantage statistics, in one workgroup (B <= 1024
// trajectories: the learner's minibatch is 256): termination = done (1 - truncation) and the reward
// scaling (what ppo.FusedGrad computed with three torch launches), the recursion of gae_kernel, then
// the mean and population std of all T x B advantages as adv_stats_kernel computes them (two passes;
// each thread re-reads the advantages it wrote). One launch instead of five per minibatch.
__global__ __launch_bounds__(1024) void gae_stats_kernel(int T, int B, const float* __restrict__ trunc,
                                                        const float* __restrict__ done, const float* __restrict__ rew,
                                                        float rscale, const float* __restrict__ val,
                                                        const float* __restrict__ boot, float lam, float disc,
                                                        float* __restrict__ vs, float* adv, int normalize,
                                                        float* __restrict__ stats) {
    __shared__ float red[16];
    const int b = threadIdx.x;
    float s = 0.f;
    if (b < B) {
        float v_next = boot[b], vs_next = boot[b], acc = 0.f;
        for (int t = T - 1; t >= 0; --t) {
            const size_t i = (size_t)t * B + b;
            const float tr = trunc[i];
            const float keep = 1.f - tr;
            // rounded products (no FMA contraction into the sums below): the values the separate torch
            // launches produced, so the recursion is gae_kernel's bit for bit
            const float term = __fmul_rn(done[i], 1.f - tr);
            const float cont = disc * (1.f - term);
            const float r = __fmul_rn(rew[i], rscale), v = val[i];
            const float delta = (r + cont * v_next - v) * keep;
            acc = delta + cont * keep * lam * acc;
            const float vs_t = acc + v;
            const float a = (r + cont * vs_next - v) * keep;
            adv[i] = a;
            vs[i] = vs_t;
            s += a;
            v_next = v;
            vs_next = vs_t;
        }
    }
    const float invN = 1.f / (float)(T * B);
    float mean = 0.f, inv_std = 1.f;
    if (normalize) {
        mean = block_sum(s, red) * invN;
        float q = 0.f;
        if (b < B)
            for (int t = 0; t < T; t++) {
                const float d = adv[(size_t)t * B + b] - mean;
                q += d * d;
            }
        inv_std = 1.f / (sqrtf(block_sum(q, red) * invN) + 1e-8f);
    }
    if (threadIdx.x == 0) {
        stats[0] = mean;
        stats[1] = inv_std;
    }
}

// gae_stats_kernel with its inputs staged in LDS first (T x B <= GAE_LDS_MAX): every thread of the 1,024
// issues its share of the four fields' loads at once, then the recursion's threads read LDS instead of
// waiting on four global loads per time step (the learner's minibatch, 20 x 256: 13.5 us as a chain of
// 20 dependent global round trips); the advantages stay in LDS for the second statistics pass. The same
// arithmetic in the same order (block_sum's extra waves add zeros): the same bits.
constexpr int GAE_LDS_MAX = 6144;  // 120 KB of staged fields
__global__ __launch_bounds__(1024) void gae_stats_lds_kernel(int T, int B, const float* __restrict__ trunc,
                                                            const float* __restrict__ done,
                                                            const float* __restrict__ rew, float rscale,
                                                            const float* __restrict__ val,
                                                            const float* __restrict__ boot, float lam, float disc,
                                                            float* __restrict__ vs, float* __restrict__ adv,
                                                            int normalize, float* __restrict__ stats) {
    __shared__ float red[16];
    extern __shared__ float gl[];  // [5][T * B]: trunc, done, reward, value, advantage
    const int n = T * B;
    float* const s_tr = gl;
    float* const s_dn = gl + n;
    float* const s_rw = gl + 2 * n;
    float* const s_v = gl + 3 * n;
    float* const s_a = gl + 4 * n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float a = trunc[i], d = done[i], r = rew[i], v = val[i];
        s_tr[i] = a;
        s_dn[i] = d;
        s_rw[i] = r;
        s_v[i] = v;
    }
    __syncthreads();
    const int b = threadIdx.x;
    float s = 0.f;
    if (b < B) {
        float v_next = boot[b], vs_next = boot[b], acc = 0.f;
        for (int t = T - 1; t >= 0; --t) {
            const int i = t * B + b;
            const float tr = s_tr[i];
            const float keep = 1.f - tr;
            const float term = __fmul_rn(s_dn[i], 1.f - tr);
            const float cont = disc * (1.f - term);
            const float r = __fmul_rn(s_rw[i], rscale), v = s_v[i];
            const float delta = (r + cont * v_next - v) * keep;
            acc = delta + cont * keep * lam * acc;
            const float vs_t = acc + v;
            const float a = (r + cont * vs_next - v) * keep;
            adv[i] = a;
            s_a[i] = a;
            vs[i] = vs_t;
            s += a;
            v_next = v;
            vs_next = vs_t;
        }
    }
    const float invN = 1.f / (float)(T * B);
    float mean = 0.f, inv_std = 1.f;
    if (normalize) {
        mean = block_sum(s, red) * invN;  // (its barriers also order the s_a stores before the reads below)
        float q = 0.f;
        if (b < B)
            for (int t = 0; t < T; t++) {
                const float d = s_a[t * B + b] - mean;
                q += d * d;
            }
        inv_std = 1.f / (sqrtf(block_sum(q, red) * invN) + 1e-8f);
    }
    if (threadIdx.x == 0) {
        stats[0] = mean;
        stats[1] = inv_std;
    }
}

__device__ __forceinline__ float softplusf(float x) { return x > 20.f ? x : log1pf(expf(x)); }
__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + expf(-x)); }
// log |d tanh(x)/dx| = 2 (log 2 - x - softplus(-2x)) and its derivative -2 tanh(x)
__device__ __forceinline__ float ldjf(float x) { return 2.f * (0.69314718055994531f - x - softplusf(-2.f * x)); }

// The PPO loss of one minibatch and its gradient with respect to the policy logits and the value
// baseline in three launches: the advantage statistics (one workgroup, two-pass mean / population
// std), then one thread per sample (the NormalTanh log-probability ratio, the clipped surrogate, the
// value error and the entropy estimate at loc + scale eps, with their derivatives; per-workgroup
// partial sums), then the sums of the partials (one workgroup): deterministic, and it replaces ~150
// small autograd kernels per minibatch. Gradients follow torch's rules: minimum() splits a tie
// evenly, clamp() passes the gradient on its closed interval.
__global__ __launch_bounds__(1024) void adv_stats_kernel(int N, const float* __restrict__ adv, int normalize,
                                                         float* __restrict__ stats) {
    __shared__ float red[16];
    const float invN = 1.f / (float)N;
    float mean = 0.f, inv_std = 1.f;
    if (normalize) {
        float s = 0.f;
        for (int i = threadIdx.x; i < N; i += blockDim.x) s += adv[i];
        mean = block_sum(s, red) * invN;
        float q = 0.f;
        for (int i = threadIdx.x; i < N; i += blockDim.x) {
            const float d = adv[i] - mean;
            q += d * d;
        }
        inv_std = 1.f / (sqrtf(block_sum(q, red) * invN) + 1e-8f);
    }
    if (threadIdx.x == 0) {
        stats[0] = mean;
        stats[1] = inv_std;
    }
}

constexpr int PPO_TPB = 128;

// One thread per sample; the workgroup's rows of logits / raw actions / entropy draws are staged in
// LDS by coalesced loads (a thread's own row is 2A or A consecutive floats: read directly, a wave's
// accesses would be 64 rows apart) and the logits gradient leaves the same way. Row strides in LDS are
// odd, so the per-sample reads of a wave fall on distinct banks.
__global__ __launch_bounds__(PPO_TPB) void ppo_loss_kernel(int N, int A, const float* __restrict__ logits,
                                                            const float* __restrict__ raw_action,
                                                            const float* __restrict__ old_logprob,
                                                            const float* __restrict__ adv,
                                                            const float* __restrict__ vs,
                                                            const float* __restrict__ baseline,
                                                            const float* __restrict__ eps, float clip_eps,
                                                            float entropy_cost, const float* __restrict__ stats,
                                                            float* __restrict__ partial, float* __restrict__ g_logits,
                                                            float* __restrict__ g_baseline) {
    extern __shared__ float sh[];
    const int SL = 2 * A + 1, SA = A + 1;  // odd LDS row strides
    float* s_lg = sh;                      // [PPO_TPB][SL]: logits in, their gradient out
    float* s_ra = s_lg + PPO_TPB * SL;     // [PPO_TPB][SA]
    float* s_ep = s_ra + PPO_TPB * SA;     // [PPO_TPB][SA]
    __shared__ float red[3][PPO_TPB / 64];
    const int i0 = blockIdx.x * PPO_TPB, nr = min(PPO_TPB, N - i0);
    for (int k = threadIdx.x; k < nr * 2 * A; k += PPO_TPB) {
        const int r = k / (2 * A);
        s_lg[r * SL + (k - r * 2 * A)] = logits[(size_t)i0 * 2 * A + k];
    }
    for (int k = threadIdx.x; k < nr * A; k += PPO_TPB) {
        const int r = k / A, c = k - r * A;
        s_ra[r * SA + c] = raw_action[(size_t)i0 * A + k];
        s_ep[r * SA + c] = eps[(size_t)i0 * A + k];
    }
    __syncthreads();
    const float invN = 1.f / (float)N;
    const float HL2PI = 0.91893853320467274f;  // 0.5 log(2 pi)
    const int i = i0 + threadIdx.x;
    float spl = 0.f, svl = 0.f, sent = 0.f;
    if (threadIdx.x < nr) {
        const float mean = stats[0], inv_std = stats[1];
        float* lg = s_lg + threadIdx.x * SL;
        const float* ra = s_ra + threadIdx.x * SA;
        const float* ep = s_ep + threadIdx.x * SA;
        float lp = 0.f, ent = 0.f;
        for (int j = 0; j < A; j++) {
            const float loc = lg[j], sc = softplusf(lg[A + j]) + 1e-3f, a = ra[j];
            const float z = (a - loc) / sc, ls = logf(sc);
            lp += -0.5f * z * z - ls - HL2PI - ldjf(a);
            ent += 0.5f + HL2PI + ls + ldjf(loc + sc * ep[j]);
        }
        const float rho = expf(lp - old_logprob[i]);
        const float an = (adv[i] - mean) * inv_std;
        const float lo = 1.f - clip_eps, hi = 1.f + clip_eps;
        const float s1 = rho * an, s2 = fminf(fmaxf(rho, lo), hi) * an;
        const bool inr = rho >= lo && rho <= hi;
        // d(-min(s1, s2))/d lp
        const float gmin = s1 < s2 ? rho * an : (s1 > s2 ? (inr ? rho * an : 0.f) : 0.5f * rho * an * (inr ? 2.f : 1.f));
        const float g_lp = -gmin * invN, g_ent = -entropy_cost * invN;
        spl = -fminf(s1, s2);
        const float dv = vs[i] - baseline[i];
        svl = dv * dv;
        sent = ent;
        g_baseline[i] = -0.5f * dv * invN;
        for (int j = 0; j < A; j++) {  // the gradient overwrites the staged logits row (j and A + j read first)
            const float loc = lg[j], r = lg[A + j], sc = softplusf(r) + 1e-3f, a = ra[j], e = ep[j];
            const float isc = 1.f / sc, z = (a - loc) * isc;
            const float dldj = -2.f * tanhf(loc + sc * e);
            lg[j] = g_lp * z * isc + g_ent * dldj;
            lg[A + j] = sigmoidf(r) * (g_lp * (z * z - 1.f) * isc + g_ent * (isc + dldj * e));
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < nr * 2 * A; k += PPO_TPB) {
        const int r = k / (2 * A);
        g_logits[(size_t)i0 * 2 * A + k] = s_lg[r * SL + (k - r * 2 * A)];
    }
    for (int o = 32; o > 0; o >>= 1) {
        spl += __shfl_down(spl, o, 64);
        svl += __shfl_down(svl, o, 64);
        sent += __shfl_down(sent, o, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][w] = spl;
        red[1][w] = svl;
        red[2][w] = sent;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        float t = 0.f;
        for (int k = 0; k < PPO_TPB / 64; k++) t += red[threadIdx.x][k];
        partial[(size_t)blockIdx.x * 3 + threadIdx.x] = t;
    }
}

// The same loss with 16 lanes per sample (A <= 16): lane j of a sample's group takes action dimension j,
// and the log-probability and entropy sums over the dimensions are 16-lane butterfly sums. 16 samples
// per 256-thread workgroup: 320 workgroups at the learner's 5,120 rows instead of 40 (the one-thread-per-
// sample kernel ran its 14 dimensions' transcendentals back to back on 40 CUs: 29 us per minibatch).
constexpr int PPO_SPW = 16;  // samples per workgroup of the team kernel
__device__ __forceinline__ float sum16(float v) {
    v += __shfl_xor(v, 8, 16);
    v += __shfl_xor(v, 4, 16);
    v += __shfl_xor(v, 2, 16);
    v += __shfl_xor(v, 1, 16);
    return v;
}
__global__ __launch_bounds__(256) void ppo_loss_team_kernel(int N, int A, const float* __restrict__ logits,
                                                             const float* __restrict__ raw_action,
                                                             const float* __restrict__ old_logprob,
                                                             const float* __restrict__ adv,
                                                             const float* __restrict__ vs,
                                                             const float* __restrict__ baseline,
                                                             const float* __restrict__ eps, float clip_eps,
                                                             float entropy_cost, const float* __restrict__ stats,
                                                             float* __restrict__ partial, float* __restrict__ g_logits,
                                                             float* __restrict__ g_baseline) {
    __shared__ float red[3][4];
    const int g = threadIdx.x >> 4, j = threadIdx.x & 15;
    const int i = blockIdx.x * PPO_SPW + g;
    const bool ok = i < N, dj = ok && j < A;
    const float invN = 1.f / (float)N;
    const float HL2PI = 0.91893853320467274f;  // 0.5 log(2 pi)
    const size_t ic = ok ? (size_t)i : 0;
    float loc = 0.f, r = 0.f, a = 0.f, e = 0.f;
    if (dj) {
        loc = logits[ic * 2 * A + j];
        r = logits[ic * 2 * A + A + j];
        a = raw_action[ic * A + j];
        e = eps[ic * A + j];
    }
    const float sc = softplusf(r) + 1e-3f, isc = 1.f / sc, z = (a - loc) * isc, ls = logf(sc);
    const float lp = sum16(dj ? -0.5f * z * z - ls - HL2PI - ldjf(a) : 0.f);
    const float ent = sum16(dj ? 0.5f + HL2PI + ls + ldjf(loc + sc * e) : 0.f);
    const float mean = stats[0], inv_std = stats[1];
    const float rho = expf(lp - old_logprob[ic]);
    const float an = (adv[ic] - mean) * inv_std;
    const float lo = 1.f - clip_eps, hi = 1.f + clip_eps;
    const float s1 = rho * an, s2 = fminf(fmaxf(rho, lo), hi) * an;
    const bool inr = rho >= lo && rho <= hi;
    // d(-min(s1, s2))/d lp (torch: minimum() splits a tie evenly, clamp() passes on its closed interval)
    const float gmin = s1 < s2 ? rho * an : (s1 > s2 ? (inr ? rho * an : 0.f) : 0.5f * rho * an * (inr ? 2.f : 1.f));
    const float g_lp = -gmin * invN, g_ent = -entropy_cost * invN;
    const float dv = vs[ic] - baseline[ic];
    if (dj) {
        const float dldj = -2.f * tanhf(loc + sc * e);
        g_logits[ic * 2 * A + j] = g_lp * z * isc + g_ent * dldj;
        g_logits[ic * 2 * A + A + j] = sigmoidf(r) * (g_lp * (z * z - 1.f) * isc + g_ent * (isc + dldj * e));
    }
    const bool head = ok && j == 0;
    if (head) g_baseline[i] = -0.5f * dv * invN;
    float spl = head ? -fminf(s1, s2) : 0.f, svl = head ? dv * dv : 0.f, sent = head ? ent : 0.f;
    for (int o = 32; o > 0; o >>= 1) {
        spl += __shfl_down(spl, o, 64);
        svl += __shfl_down(svl, o, 64);
        sent += __shfl_down(sent, o, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][w] = spl;
        red[1][w] = svl;
        red[2][w] = sent;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        float t = 0.f;
        for (int k = 0; k < 4; k++) t += red[threadIdx.x][k];
        partial[(size_t)blockIdx.x * 3 + threadIdx.x] = t;
    }
}

__global__ __launch_bounds__(1024) void ppo_loss_sum_kernel(int N, int nblk, const float* __restrict__ partial,
                                                             float entropy_cost, float* __restrict__ out) {
    __shared__ float red[16];
    const float invN = 1.f / (float)N;
    float s[3] = {0.f, 0.f, 0.f};
    for (int b = threadIdx.x; b < nblk; b += blockDim.x)
        for (int k = 0; k < 3; k++) s[k] += partial[(size_t)b * 3 + k];
    const float pl = block_sum(s[0], red) * invN, vl = 0.25f * block_sum(s[1], red) * invN;
    const float en = block_sum(s[2], red) * invN;
    if (threadIdx.x == 0) {
        out[0] = pl + vl - entropy_cost * en;
        out[1] = pl;
        out[2] = vl;
        out[3] = en;
    }
}

struct GatherArgs {
    duck_gather_field f[DUCK_GATHER_MAX];
    long long start[DUCK_GATHER_MAX + 1];  // prefix sums of T_f m w_f
    const float* mean[DUCK_GATHER_MAX];    // per-field normaliser (duck_gather_columns_norm), or null
    const float* istd[DUCK_GATHER_MAX];
};

// GATHER_PER floats per thread (elements base + t + 256 q of the workgroup's 256 x GATHER_PER): for each,
// the field by the prefix sums, then (t, j, c); every element's index and source loads are issued before
// the first store (one element per thread was a chain of two dependent global loads per thread with
// three rounds of resident workgroups: 14.2 us for the learner's 1.5 M floats). I = int when the launch
// covers < 2^31 floats: 32-bit divisions, 64-bit arithmetic only for the source address.
constexpr int GATHER_PER = 4;
template <typename I>
__global__ __launch_bounds__(256) void gather_kernel(int nf, GatherArgs a, const long long* __restrict__ idx, int m) {
    const I base = (I)blockIdx.x * (256 * GATHER_PER) + (I)threadIdx.x;
    const I tot = (I)a.start[nf];
    int fq[GATHER_PER], cq[GATHER_PER];
    I oq[GATHER_PER];
    float xq[GATHER_PER];
#pragma unroll
    for (int q = 0; q < GATHER_PER; q++) {
        const I g = base + (I)(256 * q);
        const I gc = g < tot ? g : tot - 1;
        int f = 0;
        for (int k = 1; k < nf; k++) f += (long long)gc >= a.start[k] ? 1 : 0;
        const I o = gc - (I)a.start[f];
        const int w = a.f[f].w;
        const I row = o / (I)w;
        const int c = (int)(o - row * (I)w);
        const int t = (int)(row / (I)m), j = (int)(row - (I)t * (I)m);
        xq[q] = a.f[f].src[((long long)t * a.f[f].B + idx[j]) * w + c];
        fq[q] = f;
        cq[q] = c;
        oq[q] = o;
    }
#pragma unroll
    for (int q = 0; q < GATHER_PER; q++) {
        if (base + (I)(256 * q) >= tot) break;
        const int f = fq[q], c = cq[q];
        a.f[f].dst[oq[q]] = a.mean[f] ? (xq[q] - a.mean[f][c]) * a.istd[f][c] : xq[q];
    }
}

// Column sums and sums of squares of a rollout batch x [N][F] in fp64 (brax running_statistics.update,
// ppo.RunningStatistics). Pass 1: workgroup (rb, ct) takes rows rb * CS_ROWS .. + CS_ROWS - 1 of the 64
// columns of tile ct; lane = column (one coalesced 256-B row segment per wave load), wave w every 4th row
// from w; the 4 waves' sums combined in wave order. Pass 2: one thread per column sums the row blocks'
// partials in order. Fixed order throughout: the same bits on every run.
constexpr int CS_ROWS = 1024;
__global__ __launch_bounds__(256) void column_stats_kernel(int N, int F, const float* __restrict__ x,
                                                           double* __restrict__ part) {
    __shared__ double red[2][4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.y * 64 + lane, r0 = blockIdx.x * CS_ROWS;
    const int r1 = min(N, r0 + CS_ROWS);
    double s = 0.0, q = 0.0;
    if (c < F) {
        int r = r0 + w;
        // four rows in flight per iteration (independent loads, then the dependent sums in row order)
        for (; r + 12 < r1; r += 16) {
            const float a0 = x[(size_t)r * F + c], a1 = x[(size_t)(r + 4) * F + c];
            const float a2 = x[(size_t)(r + 8) * F + c], a3 = x[(size_t)(r + 12) * F + c];
            s += (double)a0; q += (double)a0 * (double)a0;
            s += (double)a1; q += (double)a1 * (double)a1;
            s += (double)a2; q += (double)a2 * (double)a2;
            s += (double)a3; q += (double)a3 * (double)a3;
        }
        for (; r < r1; r += 4) {
            const double a = (double)x[(size_t)r * F + c];
            s += a; q += a * a;
        }
    }
    red[0][w][lane] = s;
    red[1][w][lane] = q;
    __syncthreads();
    if (w == 0 && c < F) {
        const double ts = ((red[0][0][lane] + red[0][1][lane]) + red[0][2][lane]) + red[0][3][lane];
        const double tq = ((red[1][0][lane] + red[1][1][lane]) + red[1][2][lane]) + red[1][3][lane];
        part[(size_t)blockIdx.x * 2 * F + c] = ts;
        part[(size_t)blockIdx.x * 2 * F + F + c] = tq;
    }
}
__global__ __launch_bounds__(256) void column_stats_sum_kernel(int F, int nrb, const double* __restrict__ part,
                                                               double* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;  // 0 .. 2F - 1: sums then squares
    if (i >= 2 * F) return;
    double t = 0.0;
    for (int b = 0; b < nrb; b++) t += part[(size_t)b * 2 * F + i];
    out[i] = t;
}

}  // namespace

extern "C" int duck_column_stats_scratch(int N, int F) {
    if (N <= 0 || F <= 0) return 0;
    return ((N + CS_ROWS - 1) / CS_ROWS) * 2 * F;
}

extern "C" int duck_column_stats(int N, int F, const float* x, double* out, double* scratch, void* stream) {
    if (N < 0 || F <= 0) return duck_fail(DUCK_EINVAL, "duck_column_stats: bad size");
    if (!out || (N > 0 && (!x || !scratch))) return duck_fail(DUCK_EINVAL, "duck_column_stats: null pointer");
    hipStream_t st = (hipStream_t)stream;
    if (N == 0) {
        HIPCHECK(hipMemsetAsync(out, 0, sizeof(double) * 2 * (size_t)F, st));
        return DUCK_OK;
    }
    const int nrb = (N + CS_ROWS - 1) / CS_ROWS;
    hipLaunchKernelGGL(column_stats_kernel, dim3(nrb, (F + 63) / 64), dim3(256), 0, st, N, F, x, scratch);
    hipLaunchKernelGGL(column_stats_sum_kernel, dim3((2 * F + 255) / 256), dim3(256), 0, st, F, nrb, scratch, out);
    HIPCHECK(hipGetLastError());
    return DUCK_OK;
}

extern "C" int duck_gather_columns_norm(int nf, const duck_gather_field* fields, const float* const* norm,
                                        const long long* idx, int m, void* stream) {
    if (nf < 0 || nf > DUCK_GATHER_MAX || m < 0) return duck_fail(DUCK_EINVAL, "duck_gather_columns: bad field count or size");
    if (nf == 0 || m == 0) return DUCK_OK;
    if (!fields || !idx) return duck_fail(DUCK_EINVAL, "duck_gather_columns: null pointer");
    GatherArgs a;
    memset(&a, 0, sizeof(a));
    a.start[0] = 0;
    for (int k = 0; k < nf; k++) {
        const duck_gather_field& f = fields[k];
        if (!f.src || !f.dst || f.T < 0 || f.B < 1 || f.w < 1)
            return duck_fail(DUCK_EINVAL, "duck_gather_columns: bad field");
        a.f[k] = f;
        a.start[k + 1] = a.start[k] + (long long)f.T * m * f.w;
        if (norm) {
            a.mean[k] = norm[2 * k];
            a.istd[k] = norm[2 * k + 1];
            if (!a.mean[k] != !a.istd[k]) return duck_fail(DUCK_EINVAL, "duck_gather_columns_norm: mean without istd");
        }
    }
    const long long tot = a.start[nf];
    if (tot == 0) return DUCK_OK;
    const dim3 grid((unsigned)((tot + 256 * GATHER_PER - 1) / (256 * GATHER_PER)));
    if (tot + 256 < (1ll << 31))
        hipLaunchKernelGGL(gather_kernel<int>, grid, dim3(256), 0, (hipStream_t)stream, nf, a, idx, m);
    else
        hipLaunchKernelGGL(gather_kernel<long long>, grid, dim3(256), 0, (hipStream_t)stream, nf, a, idx, m);
    HIPCHECK(hipGetLastError());
    return DUCK_OK;
}

extern "C" int duck_gather_columns(int nf, const duck_gather_field* fields, const long long* idx, int m, void* stream) {
    return duck_gather_columns_norm(nf, fields, nullptr, idx, m, stream);
}

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

extern "C" int duck_gae_stats(int T, int B, const float* truncation, const float* done, const float* reward,
                              float reward_scale, const float* value, const float* bootstrap, float lambda_,
                              float discount, float* vs, float* adv, int normalize_advantage, float* stats,
                              void* stream) {
    if (T <= 0 || B <= 0 || B > 1024) return duck_fail(DUCK_EINVAL, "duck_gae_stats: 1 <= B <= 1024 trajectories, T >= 1");
    if (!truncation || !done || !reward || !value || !bootstrap || !vs || !adv || !stats)
        return duck_fail(DUCK_EINVAL, "duck_gae_stats: null pointer");
    if (T * B <= GAE_LDS_MAX) {
        hipLaunchKernelGGL(gae_stats_lds_kernel, dim3(1), dim3(1024), sizeof(float) * 5 * T * B, (hipStream_t)stream, T,
                           B, truncation, done, reward, reward_scale, value, bootstrap, lambda_, discount, vs, adv,
                           normalize_advantage, stats);
    } else {
        const int tpb = ((B + 63) / 64) * 64;
        hipLaunchKernelGGL(gae_stats_kernel, dim3(1), dim3(tpb), 0, (hipStream_t)stream, T, B, truncation, done, reward,
                           reward_scale, value, bootstrap, lambda_, discount, vs, adv, normalize_advantage, stats);
    }
    HIPCHECK(hipGetLastError());
    return DUCK_OK;
}

static int ppo_loss_launch(int N, int A, const float* logits, const float* raw_action, const float* old_logprob,
                           const float* advantage, const float* value_target, const float* baseline,
                           const float* eps, float clip_eps, float entropy_cost, int normalize_advantage,
                           const float* stats_in, float* out, float* grad_logits, float* grad_baseline, void* stream,
                           bool sums = true);

extern "C" int duck_ppo_loss(int N, int A, const float* logits, const float* raw_action, const float* old_logprob,
                             const float* advantage, const float* value_target, const float* baseline,
                             const float* eps, float clip_eps, float entropy_cost, int normalize_advantage,
                             float* out, float* grad_logits, float* grad_baseline, void* stream) {
    return ppo_loss_launch(N, A, logits, raw_action, old_logprob, advantage, value_target, baseline, eps, clip_eps,
                           entropy_cost, normalize_advantage, nullptr, out, grad_logits, grad_baseline, stream);
}

extern "C" int duck_ppo_loss_stats(int N, int A, const float* logits, const float* raw_action,
                                   const float* old_logprob, const float* advantage, const float* value_target,
                                   const float* baseline, const float* eps, float clip_eps, float entropy_cost,
                                   const float* stats, float* out, float* grad_logits, float* grad_baseline,
                                   void* stream) {
    if (!stats) return duck_fail(DUCK_EINVAL, "duck_ppo_loss_stats: null stats");
    return ppo_loss_launch(N, A, logits, raw_action, old_logprob, advantage, value_target, baseline, eps, clip_eps,
                           entropy_cost, 1, stats, out, grad_logits, grad_baseline, stream);
}

static int ppo_loss_launch(int N, int A, const float* logits, const float* raw_action, const float* old_logprob,
                           const float* advantage, const float* value_target, const float* baseline,
                           const float* eps, float clip_eps, float entropy_cost, int normalize_advantage,
                           const float* stats_in, float* out, float* grad_logits, float* grad_baseline, void* stream,
                           bool sums) {
    if (N <= 0 || A <= 0) return duck_fail(DUCK_EINVAL, "duck_ppo_loss: empty batch");
    const size_t lds = sizeof(float) * PPO_TPB * (4 * A + 3);
    if (lds > 64 * 1024) return duck_fail(DUCK_EINVAL, "duck_ppo_loss: action size too large");
    if (!logits || !raw_action || !old_logprob || !advantage || !value_target || !baseline || !eps || !out ||
        !grad_logits || !grad_baseline)
        return duck_fail(DUCK_EINVAL, "duck_ppo_loss: null pointer");
    // the team kernel (16 lanes per sample) for A <= 16, else one thread per sample
    const bool team = A <= 16;
    const int nblk = team ? (N + PPO_SPW - 1) / PPO_SPW : (N + PPO_TPB - 1) / PPO_TPB;
    // scratch: out[4 ..) of the caller's duck_ppo_loss_out_size(N) floats holds the statistics and the partial sums
    float* stats = out + 4;
    float* partial = out + 6;
    hipStream_t st = (hipStream_t)stream;
    if (stats_in)  // computed by duck_gae_stats
        stats = const_cast<float*>(stats_in);
    else
        hipLaunchKernelGGL(adv_stats_kernel, dim3(1), dim3(1024), 0, st, N, advantage, normalize_advantage, stats);
    if (team)
        hipLaunchKernelGGL(ppo_loss_team_kernel, dim3(nblk), dim3(256), 0, st, N, A, logits, raw_action, old_logprob,
                           advantage, value_target, baseline, eps, clip_eps, entropy_cost, stats, partial, grad_logits,
                           grad_baseline);
    else
        hipLaunchKernelGGL(ppo_loss_kernel, dim3(nblk), dim3(PPO_TPB), lds, st, N, A, logits, raw_action, old_logprob,
                           advantage, value_target, baseline, eps, clip_eps, entropy_cost, stats, partial, grad_logits,
                           grad_baseline);
    if (sums) hipLaunchKernelGGL(ppo_loss_sum_kernel, dim3(1), dim3(1024), 0, st, N, nblk, partial, entropy_cost, out);
    HIPCHECK(hipGetLastError());
    return DUCK_OK;
}

extern "C" int duck_ppo_loss_grad(int N, int A, const float* logits, const float* raw_action, const float* old_logprob,
                                  const float* advantage, const float* value_target, const float* baseline,
                                  const float* eps, float clip_eps, float entropy_cost, const float* stats, float* out,
                                  float* grad_logits, float* grad_baseline, void* stream) {
    if (!stats) return duck_fail(DUCK_EINVAL, "duck_ppo_loss_grad: null stats");
    if (A > 16) return duck_fail(DUCK_EINVAL, "duck_ppo_loss_grad: action size above 16");
    return ppo_loss_launch(N, A, logits, raw_action, old_logprob, advantage, value_target, baseline, eps, clip_eps,
                           entropy_cost, 1, stats, out, grad_logits, grad_baseline, stream, false);
}

extern "C" int duck_ppo_loss_sums(int N, int A, float entropy_cost, float* out, void* stream) {
    if (N <= 0 || A <= 0 || A > 16) return duck_fail(DUCK_EINVAL, "duck_ppo_loss_sums: bad size");
    if (!out) return duck_fail(DUCK_EINVAL, "duck_ppo_loss_sums: null pointer");
    const int nblk = (N + PPO_SPW - 1) / PPO_SPW;
    hipLaunchKernelGGL(ppo_loss_sum_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, N, nblk, out + 6,
                       entropy_cost, out);
    HIPCHECK(hipGetLastError());
    return DUCK_OK;
}

// (enough for either kernel: the team kernel's 16-sample workgroups give the most partial sums)
extern "C" int duck_ppo_loss_out_size(int N) { return 4 + 2 + 3 * (((N > 0 ? N : 0) + PPO_SPW - 1) / PPO_SPW); }
