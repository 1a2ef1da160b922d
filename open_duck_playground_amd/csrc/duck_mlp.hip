// The PPO networks' MLP layers on fp32 MFMA (include/duck_ppo.h: duck_mlp_gemm, duck_mlp_wgrad,
// duck_mlp_wgrad_reduce). brax's MLP (ppo/networks.py: Dense layers with swish between them, the
// reference reaches it through common/runner.py:104-118) forward and backward for a minibatch of
// N rows as a handful of GEMM launches with the elementwise work fused into their loads and stores:
//
//   forward   Z = op(X) W^T + b, H = silu(Z)       (op: the observation normaliser on the first layer)
//   backward  dZ_prev = (dZ W) * silu'(Z_prev)      (the activation's derivative in the epilogue)
//   weights   dW = dZ^T H_prev, db = sum_n dZ        (split over the batch rows; the partial products
//                                                    summed in fixed order by duck_mlp_wgrad_reduce:
//                                                    deterministic, no atomics)
//
// v_mfma_f32_16x16x4_f32 (exact f32 products, fp32 accumulation: a k-ordered fmaf chain). A
// 256-thread workgroup computes a 64 x 64 output tile, each wave 32 x 32 as 2 x 2 MFMA tiles (four
// independent accumulators cover the instruction's 40-cycle dependent latency); operands pass
// through LDS in 32-deep reduction chunks, the next chunk's global loads issued before the current
// chunk's MFMAs (software pipelined), LDS rows padded to 33 floats (conflict-free fragment reads).
#include <hip/hip_runtime.h>

#include "duck_common.h"
#include "duck_math.h"
#include "../../include/duck_ppo.h"

namespace {

constexpr int MT = 64;    // output tile rows (the batch dimension for the forward / dX GEMMs)
constexpr int NT = 64;    // output tile columns
constexpr int KC = 32;    // reduction chunk
constexpr int LDP = KC + 1;
using f4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ float sigm(float z) { return 1.f / (1.f + __expf(-z)); }

// A tile [64 rows][KC] from a matrix whose REDUCTION index is contiguous (row stride ld): X for
// the forward (rows n, reduction k), dZ for dX (rows n, reduction m). 256 threads x 2 float4.
// norm: (x - mean[k]) * istd[k] on the way in (the first layer's observation normaliser).
struct LoadRowMajor {
  float v[8];
  __device__ void load(const float* __restrict__ A, int ld, int rows, int red, int r0, int k0,
                       const float* __restrict__ mean, const float* __restrict__ istd) {
#pragma unroll
    for (int p = 0; p < 2; p++) {
      const int t = threadIdx.x + 256 * p, r = t >> 3, c = 4 * (t & 7);
      const int gr = r0 + r;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int gk = k0 + c + q;
        float x = (gr < rows && gk < red) ? A[(size_t)gr * ld + gk] : 0.f;
        if (mean && gk < red) x = (x - mean[gk]) * istd[gk];
        v[4 * p + q] = x;
      }
    }
  }
  __device__ void store(float* S) const {  // S[row][k]
#pragma unroll
    for (int p = 0; p < 2; p++) {
      const int t = threadIdx.x + 256 * p, r = t >> 3, c = 4 * (t & 7);
#pragma unroll
      for (int q = 0; q < 4; q++) S[r * LDP + c + q] = v[4 * p + q];
    }
  }
};

// A tile [64 columns][KC] from a matrix whose OUTPUT index is contiguous and whose reduction index
// runs over its rows (W for dX: W[m][k'], reduction m; dZ and H for the weight gradient: rows n):
// global rows k0..k0+31, columns c0..c0+63, stored transposed as S[column][k].
struct LoadColMajor {
  float v[8];
  __device__ void load(const float* __restrict__ B, int ld, int red, int cols, int k0, int c0) {
#pragma unroll
    for (int p = 0; p < 2; p++) {
      const int t = threadIdx.x + 256 * p, r = t >> 4, c = 4 * (t & 15);
      const int gk = k0 + r;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int gc = c0 + c + q;
        v[4 * p + q] = (gk < red && gc < cols) ? B[(size_t)gk * ld + gc] : 0.f;
      }
    }
  }
  __device__ void store(float* S) const {
#pragma unroll
    for (int p = 0; p < 2; p++) {
      const int t = threadIdx.x + 256 * p, r = t >> 4, c = 4 * (t & 15);
#pragma unroll
      for (int q = 0; q < 4; q++) S[(c + q) * LDP + r] = v[4 * p + q];
    }
  }
};

// the 2 x 2 MFMA tiles of this wave over one LDS chunk: As[row][k], Bs[col][k]
__device__ __forceinline__ void mma_chunk(const float* As, const float* Bs, int wr, int wc, f4 (&acc)[2][2]) {
  const int l = threadIdx.x & 63, li = l & 15, lk = l >> 4;
#pragma unroll
  for (int s = 0; s < KC / 4; s++) {
    const int k = 4 * s + lk;
    const float a0 = As[(wr + li) * LDP + k], a1 = As[(wr + 16 + li) * LDP + k];
    const float b0 = Bs[(wc + li) * LDP + k], b1 = Bs[(wc + 16 + li) * LDP + k];
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
  }
}

// Forward (MODE 0: Y = op(X) W^T + b; MODE 1: the same, Y = Z and Y2 = silu(Z)) and the backward
// data GEMM (MODE 2: Y = (dZ W) * silu'(Zp), Zp = aux). Output [N][Mo], tile (blockIdx.x: rows,
// blockIdx.y: columns).
template <int MODE>
__global__ __launch_bounds__(256) void mlp_gemm_kernel(int N, int R, int Mo, const float* __restrict__ A,
                                                       const float* __restrict__ W, const float* __restrict__ bias,
                                                       const float* __restrict__ aux, float* __restrict__ Y,
                                                       float* __restrict__ Y2, const float* __restrict__ mean,
                                                       const float* __restrict__ istd) {
  __shared__ float As[2][MT * LDP], Bs[2][NT * LDP];
  const int r0 = blockIdx.x * MT, c0 = blockIdx.y * NT;
  const int w = threadIdx.x >> 6, wr = 32 * (w >> 1), wc = 32 * (w & 1);
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  LoadRowMajor la;
  LoadRowMajor lbr;  // MODE 0/1: W[m][k], reduction k contiguous (as X)
  LoadColMajor lbc;  // MODE 2: W[m][k'], reduction m over rows
  const int ldA = R;
  auto load = [&](int k0) {
    la.load(A, ldA, N, R, r0, k0, MODE == 2 ? nullptr : mean, istd);
    if (MODE == 2) lbc.load(W, Mo, R, Mo, k0, c0);
    else lbr.load(W, R, Mo, R, c0, k0, nullptr, nullptr);
  };
  auto store = [&](int b) {
    la.store(As[b]);
    if (MODE == 2) lbc.store(Bs[b]);
    else lbr.store(Bs[b]);
  };
  const int nch = (R + KC - 1) / KC;
  load(0);
  store(0);
  __syncthreads();
  for (int c = 0; c < nch; c++) {
    const int b = c & 1;
    if (c + 1 < nch) load(KC * (c + 1));  // in flight while this chunk's MFMAs run
    mma_chunk(As[b], Bs[b], wr, wc, acc);
    if (c + 1 < nch) store(b ^ 1);
    __syncthreads();
  }
  // epilogue: acc[i][j][q] is C[wr + 16 i + 4 (l >> 4) + q][wc + 16 j + (l & 15)]
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const int col = c0 + wc + 16 * j + (l & 15);
      if (col >= Mo) continue;
      const float bj = (MODE != 2 && bias) ? bias[col] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int row = r0 + wr + 16 * i + 4 * (l >> 4) + q;
        if (row >= N) continue;
        const size_t o = (size_t)row * Mo + col;
        const float z = acc[i][j][q] + bj;
        if (MODE == 0) {
          Y[o] = z;
        } else if (MODE == 1) {
          Y[o] = z;
          Y2[o] = z * sigm(z);
        } else {
          const float zp = aux[o], s = sigm(zp);
          Y[o] = z * (s * (1.f + zp * (1.f - s)));
        }
      }
    }
}

// dW[m][k] = sum over this block's rows n of dZ[n][m] H[n][k] (+ the bias partial sum_n dZ[n][m]
// on the k-tile-0 blocks): partial s = blockIdx.z of S, written to part + s * P at the layer's
// offsets (weights at offw, bias at offb, P = the parameter count of the whole network).
__global__ __launch_bounds__(256) void mlp_wgrad_kernel(int N, int Mo, int Ki, const float* __restrict__ dZ,
                                                        const float* __restrict__ H, const float* __restrict__ mean,
                                                        const float* __restrict__ istd, int rows_per_split,
                                                        float* __restrict__ part, int P, int offw, int offb) {
  __shared__ float As[2][MT * LDP], Bs[2][NT * LDP];
  const int m0 = blockIdx.x * MT, k0c = blockIdx.y * NT, s = blockIdx.z;
  const int n_lo = s * rows_per_split, n_hi = min(N, n_lo + rows_per_split);
  const int w = threadIdx.x >> 6, wr = 32 * (w >> 1), wc = 32 * (w & 1);
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  LoadColMajor la, lb;  // A = dZ^T (columns m, reduction n over rows), B = H (columns k, rows n)
  float bsum = 0.f;     // bias partial of column m0 + (tid & 63) (k-tile 0 only)
  const bool dob = blockIdx.y == 0;
  auto load = [&](int n0) {
    la.load(dZ + (size_t)n_lo * Mo, Mo, n_hi - n_lo, Mo, n0, m0);
    lb.load(H + (size_t)n_lo * Ki, Ki, n_hi - n_lo, Ki, n0, k0c);
    if (mean) {  // the first layer's input is the normalised observation
#pragma unroll
      for (int p = 0; p < 2; p++) {
        const int t = threadIdx.x + 256 * p, r = t >> 4, c = 4 * (t & 15);
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int gk = k0c + c + q;
          if (n0 + r < n_hi - n_lo && gk < Ki) lb.v[4 * p + q] = (lb.v[4 * p + q] - mean[gk]) * istd[gk];
        }
      }
    }
  };
  auto store = [&](int b) {
    la.store(As[b]);
    lb.store(Bs[b]);
  };
  const int R = n_hi - n_lo;
  const int nch = (R + KC - 1) / KC;
  if (nch > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int c = 0; c < nch; c++) {
    const int b = c & 1;
    if (c + 1 < nch) load(KC * (c + 1));
    mma_chunk(As[b], Bs[b], wr, wc, acc);
    if (dob && threadIdx.x < 64) {
#pragma unroll 8
      for (int k = 0; k < KC; k++) bsum += As[b][threadIdx.x * LDP + k];
    }
    if (c + 1 < nch) store(b ^ 1);
    __syncthreads();
  }
  float* out = part + (size_t)s * P;
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const int col = k0c + wc + 16 * j + (l & 15);
      if (col >= Ki) continue;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int row = m0 + wr + 16 * i + 4 * (l >> 4) + q;
        if (row < Mo) out[offw + (size_t)row * Ki + col] = acc[i][j][q];
      }
    }
  if (dob && threadIdx.x < 64 && m0 + (int)threadIdx.x < Mo) out[offb + m0 + threadIdx.x] = bsum;
}

// grad[i] = sum_s part[s * P + i], s in order (deterministic)
__global__ __launch_bounds__(256) void mlp_reduce_kernel(int P, int S, const float* __restrict__ part,
                                                         float* __restrict__ grad) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= P) return;
  float a = 0.f;
  for (int s = 0; s < S; s++) a += part[(size_t)s * P + i];
  grad[i] = a;
}


// brax NormalTanhDistribution sampling for the rollout (ppo/networks.py; ppo.NormalTanh): one thread
// per env row, raw = loc + scale eps with scale = softplus(pre) + 1e-3 and eps ~ N(0, 1) by
// Box-Muller from threefry2x32 (key = seed, counter = (row, 8 draw + pair)), action = tanh(raw),
// log_prob = sum_j -z^2/2 - log scale - log(2 pi)/2 - log|tanh'(raw)| with z = (raw - loc) / scale
// (the same expression the loss recomputes). The draw counter lives in device memory and the
// following one-thread launch advances it, so a captured rollout draws fresh noise on every replay.
__global__ __launch_bounds__(256) void policy_sample_kernel(int N, int A, const float* __restrict__ logits,
                                                            uint32_t k0, uint32_t k1, const uint32_t* __restrict__ ctr,
                                                            float* __restrict__ raw, float* __restrict__ logprob,
                                                            float* __restrict__ action) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const uint32_t c = *ctr;
  const float* lg = logits + (size_t)n * 2 * A;
  float lp = 0.f;
  for (int j0 = 0; j0 < A; j0 += 2) {
    uint32_t a, b;
    threefry2x32(k0, k1, (uint32_t)n, c * 8u + (uint32_t)(j0 >> 1), a, b);
    const float u1 = ((float)(a >> 9) + 1.f) * (1.f / 8388608.f);  // (0, 1]
    const float u2 = (float)(b >> 9) * (1.f / 8388608.f);
    const float r = sqrtf(-2.f * logf(u1));
    float sn, cs;
    sincosf(6.283185307179586f * u2, &sn, &cs);
    const float e2[2] = {r * cs, r * sn};
    for (int h = 0; h < 2 && j0 + h < A; h++) {
      const int j = j0 + h;
      const float loc = lg[j], pre = lg[A + j];
      const float scale = (pre > 20.f ? pre : log1pf(__expf(pre))) + 1e-3f;
      const float x = loc + scale * e2[h];
      const float z = (x - loc) / scale;
      const float sp = -2.f * x > 20.f ? -2.f * x : log1pf(__expf(-2.f * x));
      lp += -0.5f * z * z - logf(scale) - 0.91893853320467274f - 2.f * (0.69314718055994531f - x - sp);
      raw[(size_t)n * A + j] = x;
      action[(size_t)n * A + j] = tanhf(x);
    }
  }
  logprob[n] = lp;
}

__global__ void ctr_inc_kernel(uint32_t* ctr) { *ctr += 1u; }

}  // namespace

extern "C" int duck_mlp_gemm(int mode, int N, int R, int M, const float* A, const float* W, const float* bias,
                             const float* aux, float* Y, float* Y2, const float* mean, const float* istd,
                             void* stream) {
  if (N < 0 || R <= 0 || M <= 0) return duck_fail(DUCK_EINVAL, "duck_mlp_gemm: bad size");
  if (N == 0) return DUCK_OK;
  if (!A || !W || !Y || (mode == 1 && !Y2) || (mode == 2 && !aux) || (!mean) != (!istd))
    return duck_fail(DUCK_EINVAL, "duck_mlp_gemm: null pointer");
  const dim3 grid((N + MT - 1) / MT, (M + NT - 1) / NT);
  hipStream_t st = (hipStream_t)stream;
  switch (mode) {
    case 0: hipLaunchKernelGGL(mlp_gemm_kernel<0>, grid, dim3(256), 0, st, N, R, M, A, W, bias, aux, Y, Y2, mean, istd); break;
    case 1: hipLaunchKernelGGL(mlp_gemm_kernel<1>, grid, dim3(256), 0, st, N, R, M, A, W, bias, aux, Y, Y2, mean, istd); break;
    case 2:
      if (mean) return duck_fail(DUCK_EINVAL, "duck_mlp_gemm: the data gradient takes no normaliser");
      hipLaunchKernelGGL(mlp_gemm_kernel<2>, grid, dim3(256), 0, st, N, R, M, A, W, bias, aux, Y, Y2, mean, istd);
      break;
    default: return duck_fail(DUCK_EINVAL, "duck_mlp_gemm: mode must be 0, 1 or 2");
  }
  HIPCHECK(hipGetLastError());
  return DUCK_OK;
}

extern "C" int duck_mlp_wgrad(int N, int M, int K, const float* dZ, const float* H, const float* mean,
                              const float* istd, int splits, float* partial, int P, int off_w, int off_b,
                              void* stream) {
  if (N <= 0 || M <= 0 || K <= 0 || splits <= 0) return duck_fail(DUCK_EINVAL, "duck_mlp_wgrad: bad size");
  if (!dZ || !H || !partial || (!mean) != (!istd)) return duck_fail(DUCK_EINVAL, "duck_mlp_wgrad: null pointer");
  if (off_w < 0 || off_b < 0 || (long long)off_w + (long long)M * K > P || off_b + M > P)
    return duck_fail(DUCK_EINVAL, "duck_mlp_wgrad: offsets outside the parameter vector");
  const int rps = (N + splits - 1) / splits;
  const dim3 grid((M + MT - 1) / MT, (K + NT - 1) / NT, splits);
  hipLaunchKernelGGL(mlp_wgrad_kernel, grid, dim3(256), 0, (hipStream_t)stream, N, M, K, dZ, H, mean, istd, rps,
                     partial, P, off_w, off_b);
  HIPCHECK(hipGetLastError());
  return DUCK_OK;
}

extern "C" int duck_mlp_wgrad_reduce(int P, int splits, const float* partial, float* grad, void* stream) {
  if (P <= 0 || splits <= 0) return duck_fail(DUCK_EINVAL, "duck_mlp_wgrad_reduce: bad size");
  if (!partial || !grad) return duck_fail(DUCK_EINVAL, "duck_mlp_wgrad_reduce: null pointer");
  hipLaunchKernelGGL(mlp_reduce_kernel, dim3((P + 255) / 256), dim3(256), 0, (hipStream_t)stream, P, splits, partial,
                     grad);
  HIPCHECK(hipGetLastError());
  return DUCK_OK;
}

extern "C" int duck_policy_sample(int N, int A, const float* logits, unsigned long long seed, unsigned int* ctr,
                                  float* raw, float* logprob, float* action, void* stream) {
  if (N < 0 || A <= 0 || A > 16) return duck_fail(DUCK_EINVAL, "duck_policy_sample: bad size");
  if (N == 0) return DUCK_OK;
  if (!logits || !ctr || !raw || !logprob || !action) return duck_fail(DUCK_EINVAL, "duck_policy_sample: null pointer");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(policy_sample_kernel, dim3((N + 255) / 256), dim3(256), 0, st, N, A, logits, (uint32_t)seed,
                     (uint32_t)(seed >> 32), ctr, raw, logprob, action);
  hipLaunchKernelGGL(ctr_inc_kernel, dim3(1), dim3(1), 0, st, ctr);
  HIPCHECK(hipGetLastError());
  return DUCK_OK;
}
