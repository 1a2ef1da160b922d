// The PPO networks' MLP layers on fp32 MFMA (include/duck_ppo.h: duck_mlp_gemm, duck_mlp_wgrad,
// duck_mlp_wgrad_reduce, duck_policy_sample). brax's MLP (ppo/networks.py: Dense layers with swish
// between them, the reference reaches it through common/runner.py:104-118) forward and backward for a
// minibatch of N rows as a handful of GEMM launches with the elementwise work fused into their loads
// and stores:
//
//   forward   Z = op(X) W^T + b, H = silu(Z)       (op: the observation normaliser on the first layer)
//   backward  dZ_prev = (dZ W) * silu'(Z_prev)      (the activation's derivative in the epilogue)
//   weights   [dW | db] = dZ^T [H | 1]             (the bias gradient as one more column of ones; split
//                                                    over row blocks of the batch, the partial products
//                                                    summed in fixed order by duck_mlp_wgrad_reduce:
//                                                    deterministic, no atomics)
//
// v_mfma_f32_16x16x4_f32 (exact f32 products, fp32 accumulation: a k-ordered fmaf chain). A
// 256-thread workgroup computes a 64 x 32 output tile, each wave 32 x 16 as 2 x 1 MFMA tiles; operands
// pass through one LDS buffer per operand in 32-deep reduction chunks, the next chunk's global loads
// in flight during the current chunk's MFMAs; 12.7 KB of LDS and small tiles keep several
// workgroups per CU resident, so one workgroup's load latency hides behind another's MFMAs (the
// learner's GEMMs are 5120 rows deep and at most 512 wide: a 64 x 64 tile left ~1 workgroup per CU
// and ran 3-4x slower). LDS tile layouts: see swz_word / tile_ksteps below.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "duck_common.h"
#include "duck_math.h"
#include "../../include/duck_ppo.h"

#ifndef DUCK_MLP_KC
#define DUCK_MLP_KC 32
#endif
// resident waves per SIMD the grouped 64 x 32-tile kernel is compiled for (6: 80 registers, no spills;
// uncapped it takes 82 and holds 5)
#ifndef DUCK_MLP_WPE
#define DUCK_MLP_WPE 6
#endif

namespace {

#ifndef DUCK_MLP_BM
#define DUCK_MLP_BM 64
#endif
constexpr int BM = DUCK_MLP_BM;  // output tile rows (the batch rows for the forward / data-gradient GEMMs)
constexpr int BN = 32;    // output tile columns (duck_mlp_gemm / duck_mlp_wgrad; duck_mlp_group_bn takes 32 or 64)
// reduction chunk. Deeper chunks mean fewer memory round trips per tile but more LDS per workgroup:
// KC = 128 (49.5 KB, 3 workgroups per CU) made training 1.9 -> 1.2 M env-steps/s same-box against
// KC = 32 (12.7 KB): the resident workgroups hiding each other's load latency matter more
constexpr int KC = DUCK_MLP_KC;
constexpr int KPT = KC / 8;  // reduction indices per thread of a row tile (8 threads cover a chunk row)
using f4 = __attribute__((ext_vector_type(4))) float;

// LDS tile layouts (round 6). An MFMA 16x16x4 k-step reads, per lane (li = l & 15, lk = l >> 4), element
// (row li, k 4 s + lk) of each operand. With [row][k] rows padded to 33 words those ds_read_b32 met 2-way
// bank conflicts in every 32-lane group, 24 of them per wave and chunk:
//  * operands whose reduction index is contiguous in memory (RowTile: X, dZ, W's rows) are stored
//    [row][lk][s] -- a lane's 8 k-steps of a chunk in 8 consecutive words, read as two ds_read_b128 -- with
//    the 4-word blocks of row r XOR-swizzled by f(r) = (2 r + (r >> 3)) & 7 (r mod 16): conflict-free for
//    the b128 reads' 16-lane groups and for the tile stores' ds_write_b32 (a search over swizzles);
//  * operands whose reduction runs over their rows (ColTile: W in the data gradient, dZ and H in the
//    weight gradient) are stored as they are loaded, [k][col] with rows padded to COLS + 16 words: one
//    ds_write_b128 per loaded vector, and ds_read_b32 reads whose two 16-lane halves fall 16 banks apart.
// Every lane feeds the MFMAs the same values in the same k order as before: bit-identical results.
static_assert(KC == 32, "the tile layouts assume 32-deep reduction chunks");
__device__ __forceinline__ int swz_word(int row, int k) {
  const int kp = (k & 3) * 8 + (k >> 2), r = row & 15;
  return row * KC + ((((kp >> 2) ^ ((2 * r + (r >> 3)) & 7))) << 2) + (kp & 3);
}
template <int COLS>
constexpr int nat_ld() { return COLS + 16; }
template <int ROWS, int COLS>
constexpr int tile_words() {  // LDS words of a tile buffer that holds either layout
  return ROWS * KC > KC * nat_ld<COLS>() ? ROWS * KC : KC * nat_ld<COLS>();
}

__device__ __forceinline__ float sigm(float z) { return 1.f / (1.f + __expf(-z)); }

// ROWS x KC tile of a matrix whose REDUCTION index is contiguous (row stride ld): X for the forward
// (rows n, reduction k), dZ for the data gradient (rows n, reduction m). Thread t holds rows
// t / 8 (+ 32 p) and the KPT reduction indices KPT (t % 8) .. + KPT - 1 of every chunk (16-B loads
// where the rows are 16-B aligned); row pointers are formed once. norm: (x - mean[k]) * istd[k] on
// the way in (the first layer's normaliser).
template <int ROWS>
struct RowTile {
  static constexpr int P = ROWS / 32;
  const float* rp[P];
  bool ok[P];
  bool vec;
  float v[KPT * P];
  __device__ void init(const float* __restrict__ A, int ld, int rows, int r0) {
    vec = ((ld & 3) == 0) && (((size_t)A & 15) == 0);
#pragma unroll
    for (int p = 0; p < P; p++) {
      const int r = r0 + ((int)threadIdx.x >> 3) + 32 * p;
      ok[p] = r < rows;
      rp[p] = A + (size_t)(ok[p] ? r : 0) * ld;
    }
  }
  __device__ void load(int red, int k0, const float* __restrict__ mean, const float* __restrict__ istd) {
    const int c = k0 + KPT * ((int)threadIdx.x & 7);
    if (vec && c + KPT <= red) {
#pragma unroll
      for (int p = 0; p < P; p++)
#pragma unroll
        for (int q = 0; q < KPT; q += 4) {
          const f4 x = ok[p] ? *(const f4*)(rp[p] + c + q) : f4{0.f, 0.f, 0.f, 0.f};
          v[KPT * p + q] = x[0]; v[KPT * p + q + 1] = x[1]; v[KPT * p + q + 2] = x[2]; v[KPT * p + q + 3] = x[3];
        }
    } else {
#pragma unroll
      for (int p = 0; p < P; p++)
#pragma unroll
        for (int q = 0; q < KPT; q++) {
          const int k = c + q;
          v[KPT * p + q] = (ok[p] && k < red) ? rp[p][k] : 0.f;
        }
    }
    if (mean) {
#pragma unroll
      for (int p = 0; p < P; p++)
#pragma unroll
        for (int q = 0; q < KPT; q++) {
          const int k = c + q;
          v[KPT * p + q] = k < red ? (v[KPT * p + q] - mean[k]) * istd[k] : 0.f;
        }
    }
  }
  __device__ void store(float* S) const {  // the swizzled [row][lk][s] layout (swz_word)
    const int c = KPT * ((int)threadIdx.x & 7);
#pragma unroll
    for (int p = 0; p < P; p++) {
      const int r = ((int)threadIdx.x >> 3) + 32 * p;
#pragma unroll
      for (int q = 0; q < KPT; q++) S[swz_word(r, c + q)] = v[KPT * p + q];
    }
  }
};

// KC x COLS tile of a matrix whose OUTPUT index is contiguous and whose reduction index runs over its
// rows (W for the data gradient; dZ and H for the weight gradient), stored transposed as S[col][k].
// Thread t holds columns 4 (t % (COLS / 4)) .. + 3 of reduction rows t / (COLS / 4) (+ step).
// ones: column `cols` reads 1 (the bias gradient as one more weight-gradient column).
template <int COLS>
struct ColTile {
  static constexpr int TPR = COLS / 4, RSTEP = 256 / TPR, P = KC / RSTEP;
  float v[4 * P];
  __device__ void load(const float* __restrict__ B, int ld, int red, int cols, int k0, int c0, bool ones,
                       const float* __restrict__ mean, const float* __restrict__ istd) {
    const int c = c0 + 4 * ((int)threadIdx.x % TPR);
    const bool vec = ((ld & 3) == 0) && (((size_t)B & 15) == 0) && c + 3 < cols;
#pragma unroll
    for (int p = 0; p < P; p++) {
      const int k = k0 + (int)threadIdx.x / TPR + RSTEP * p;
      const bool kr = k < red;
      const float* row = B + (size_t)(kr ? k : 0) * ld;
      if (vec) {
        const f4 x = kr ? *(const f4*)(row + c) : f4{0.f, 0.f, 0.f, 0.f};
        v[4 * p] = x[0]; v[4 * p + 1] = x[1]; v[4 * p + 2] = x[2]; v[4 * p + 3] = x[3];
      } else {
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int cc = c + q;
          v[4 * p + q] = (kr && cc < cols) ? row[cc] : ((kr && ones && cc == cols) ? 1.f : 0.f);
        }
      }
      if (mean) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int cc = c + q;
          if (kr && cc < cols) v[4 * p + q] = (v[4 * p + q] - mean[cc]) * istd[cc];
        }
      }
    }
  }
  __device__ void store(float* S) const {  // [k][col], rows of nat_ld<COLS>() words
    const int c = 4 * ((int)threadIdx.x % TPR);
#pragma unroll
    for (int p = 0; p < P; p++) {
      const int r = (int)threadIdx.x / TPR + RSTEP * p;
      *(f4*)(S + r * nat_ld<COLS>() + c) = f4{v[4 * p], v[4 * p + 1], v[4 * p + 2], v[4 * p + 3]};
    }
  }
};

// k-steps 4 h .. 4 h + 3 of a lane's row (or column) x of one operand tile: one ds_read_b128 from the
// swizzled layout (SWZ, RowTile), or 4 ds_read_b32 from the [k][col] layout with rows of LD words (ColTile)
template <bool SWZ, int LD>
__device__ __forceinline__ f4 tile_ksteps(const float* S, int x, int lk, int h) {
  if constexpr (SWZ) {
    const int r = x & 15, f = (2 * r + (r >> 3)) & 7;
    return *(const f4*)(S + x * KC + (((2 * lk + h) ^ f) << 2));
  } else {
    f4 o;
#pragma unroll
    for (int s = 0; s < 4; s++) o[s] = S[(4 * (4 * h + s) + lk) * LD + x];
    return o;
  }
}

// this wave's TI x TJ MFMA tiles over one LDS chunk (layouts: tile_ksteps), in two halves of 4 k-steps
template <int TI, int TJ, bool ASWZ, int LDA, bool BSWZ, int LDB>
__device__ __forceinline__ void mma_chunk(const float* As, const float* Bs, int wr, int wc, f4 (&acc)[TI][TJ]) {
  const int l = threadIdx.x & 63, li = l & 15, lk = l >> 4;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    f4 a[TI], b[TJ];
#pragma unroll
    for (int i = 0; i < TI; i++) a[i] = tile_ksteps<ASWZ, LDA>(As, wr + 16 * i + li, lk, h);
#pragma unroll
    for (int j = 0; j < TJ; j++) b[j] = tile_ksteps<BSWZ, LDB>(Bs, wc + 16 * j + li, lk, h);
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
      for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < TJ; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
  }
}

// Forward (MODE 0: Y = op(A) W^T + b; MODE 1: the same, Y = Z and Y2 = silu(Z)) and the data gradient
// (MODE 2: Y = (A W) * silu'(aux), A = dZ [N][R], W [R][Mo], aux = Z_prev). Output [N][Mo].
template <int MODE, int BNT = BN, int BMT = BM>
__device__ __forceinline__ void gemm_tile(int bx, int by, float* As, float* Bs, int N, int R, int Mo,
                                          const float* __restrict__ A, const float* __restrict__ W,
                                          const float* __restrict__ bias, const float* __restrict__ aux,
                                          float* __restrict__ Y, float* __restrict__ Y2,
                                          const float* __restrict__ mean, const float* __restrict__ istd) {
  constexpr int TI = BMT / 32, TJ = BNT / 32;
  const int r0 = bx * BMT, c0 = by * BNT;
  const int w = threadIdx.x >> 6, wr = (BMT / 2) * (w >> 1), wc = (BNT / 2) * (w & 1);
  f4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; i++)
#pragma unroll
    for (int j = 0; j < TJ; j++) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  // two register sets of staged chunks (set k & 1 holds chunk k): chunk c + 2's loads are issued while
  // chunk c's MFMAs run and stored a whole chunk later, so each load has two chunks of MFMAs to land
  RowTile<BMT> la[2];
  RowTile<BNT> lbr[2];  // MODE 0/1: the rows of W (output columns), reduction contiguous
  ColTile<BNT> lbc[2];  // MODE 2: W [R][Mo], reduction over its rows
  for (int q = 0; q < 2; q++) {
    la[q].init(A, R, N, r0);
    if (MODE != 2) lbr[q].init(W, R, Mo, c0);
  }
  const float* mn = MODE == 2 ? nullptr : mean;
  auto load = [&](auto S, int k0) {
    constexpr int q = decltype(S)::value;
    la[q].load(R, k0, mn, istd);
    if (MODE == 2) lbc[q].load(W, Mo, R, Mo, k0, c0, false, nullptr, nullptr);
    else lbr[q].load(R, k0, nullptr, nullptr);
  };
  auto store = [&](auto S) {
    constexpr int q = decltype(S)::value;
    la[q].store(As);
    if (MODE == 2) lbc[q].store(Bs);
    else lbr[q].store(Bs);
  };
  const int nch = (R + KC - 1) / KC;
  const std::integral_constant<int, 0> S0;
  const std::integral_constant<int, 1> S1;
  load(S0, 0);
  if (nch > 1) load(S1, KC);
  store(S0);
  __syncthreads();
  auto body = [&](int c, auto S, auto SN) {
    if (c + 2 < nch) load(S, KC * (c + 2));  // set S held chunk c (already in LDS)
    mma_chunk<TI, TJ, true, 0, MODE != 2, nat_ld<BNT>()>(As, Bs, wr, wc, acc);
    __syncthreads();
    if (c + 1 < nch) {
      store(SN);
      __syncthreads();
    }
  };
  for (int c = 0; c < nch; c += 2) {
    body(c, S0, S1);
    if (c + 1 < nch) body(c + 1, S1, S0);
  }
  // epilogue: acc[i][j][q] is C[wr + 16 i + 4 (l >> 4) + q][wc + 16 j + (l & 15)]
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < TI; i++)
#pragma unroll
    for (int j = 0; j < TJ; j++) {
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

template <int MODE>
__global__ __launch_bounds__(256) void mlp_gemm_kernel(int N, int R, int Mo, const float* __restrict__ A,
                                                       const float* __restrict__ W, const float* __restrict__ bias,
                                                       const float* __restrict__ aux, float* __restrict__ Y,
                                                       float* __restrict__ Y2, const float* __restrict__ mean,
                                                       const float* __restrict__ istd) {
  __shared__ __attribute__((aligned(16))) float As[tile_words<BM, BM>()], Bs[tile_words<BN, BN>()];
  gemm_tile<MODE>(blockIdx.x, blockIdx.y, As, Bs, N, R, Mo, A, W, bias, aux, Y, Y2, mean, istd);
}

// [dW | db][m][k] = sum over this workgroup's rows n of dZ[n][m] [op(H) | 1][n][k]: partial s =
// blockIdx.z, written to part + s * P at the layer's offsets (weights at offw, bias at offb; P = the
// parameter count of the networks sharing the partial array).
template <int BNT = BN, int BMT = BM>
__device__ __forceinline__ void wgrad_tile(int bx, int by, int bz, float* As, float* Bs, int N, int Mo, int Ki,
                                           const float* __restrict__ dZ, const float* __restrict__ H,
                                           const float* __restrict__ mean, const float* __restrict__ istd,
                                           int rows_per_split, float* __restrict__ part, int P, int offw, int offb) {
  constexpr int TI = BMT / 32, TJ = BNT / 32;
  const int m0 = bx * BMT, k0c = by * BNT, s = bz;
  const int n_lo = s * rows_per_split, R = min(N, n_lo + rows_per_split) - n_lo;
  const int w = threadIdx.x >> 6, wr = (BMT / 2) * (w >> 1), wc = (BNT / 2) * (w & 1);
  f4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; i++)
#pragma unroll
    for (int j = 0; j < TJ; j++) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  ColTile<BMT> la[2];  // A = dZ^T: columns m, reduction n over the rows (two staged chunks, as above)
  ColTile<BNT> lb[2];  // B = [op(H) | 1]: columns k, rows n
  const float* dz = dZ + (size_t)(R > 0 ? n_lo : 0) * Mo;
  const float* h = H + (size_t)(R > 0 ? n_lo : 0) * Ki;
  auto load = [&](auto S, int n0) {
    constexpr int q = decltype(S)::value;
    la[q].load(dz, Mo, R, Mo, n0, m0, false, nullptr, nullptr);
    lb[q].load(h, Ki, R, Ki, n0, k0c, true, mean, istd);
  };
  auto store = [&](auto S) {
    constexpr int q = decltype(S)::value;
    la[q].store(As);
    lb[q].store(Bs);
  };
  const int nch = (R + KC - 1) / KC;
  const std::integral_constant<int, 0> S0;
  const std::integral_constant<int, 1> S1;
  if (nch > 0) {
    load(S0, 0);
    if (nch > 1) load(S1, KC);
    store(S0);
  }
  __syncthreads();
  auto body = [&](int c, auto S, auto SN) {
    if (c + 2 < nch) load(S, KC * (c + 2));
    mma_chunk<TI, TJ, false, nat_ld<BMT>(), false, nat_ld<BNT>()>(As, Bs, wr, wc, acc);
    __syncthreads();
    if (c + 1 < nch) {
      store(SN);
      __syncthreads();
    }
  };
  for (int c = 0; c < nch; c += 2) {
    body(c, S0, S1);
    if (c + 1 < nch) body(c + 1, S1, S0);
  }
  float* out = part + (size_t)s * P;
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < TI; i++)
#pragma unroll
    for (int j = 0; j < TJ; j++) {
      const int col = k0c + wc + 16 * j + (l & 15);
      if (col > Ki) continue;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int row = m0 + wr + 16 * i + 4 * (l >> 4) + q;
        if (row < Mo) out[col < Ki ? offw + (size_t)row * Ki + col : offb + row] = acc[i][j][q];
      }
    }
}

__global__ __launch_bounds__(256) void mlp_wgrad_kernel(int N, int Mo, int Ki, const float* __restrict__ dZ,
                                                        const float* __restrict__ H, const float* __restrict__ mean,
                                                        const float* __restrict__ istd, int rows_per_split,
                                                        float* __restrict__ part, int P, int offw, int offb) {
  __shared__ __attribute__((aligned(16))) float As[tile_words<BM, BM>()], Bs[tile_words<BN, BN>()];
  wgrad_tile(blockIdx.x, blockIdx.y, blockIdx.z, As, Bs, N, Mo, Ki, dZ, H, mean, istd, rows_per_split, part, P, offw,
             offb);
}

// Several independent layer problems in one launch (duck_mlp_group): the learner's GEMMs are short
// chains of dependent memory round trips (a few reduction chunks each), so two or four of them
// side by side take about as long as one; the policy's and the value network's layers at the same
// depth, forward and backward, share a launch. A workgroup finds its problem by the tile prefix sums.
struct MlpGroupArgs {
  int n;
  int start[DUCK_MLP_GROUP_MAX + 1];
  int gx[DUCK_MLP_GROUP_MAX], gy[DUCK_MLP_GROUP_MAX], rps[DUCK_MLP_GROUP_MAX];
  duck_mlp_problem p[DUCK_MLP_GROUP_MAX];
};
// BMT = 32 (duck_mlp_group_tiles): half-height tiles, twice the workgroups, 58 registers and 12 KB of LDS
// (8 waves per SIMD) -- for the launches with few tiles and short reductions (FusedGrad._row_tile)
template <int BNT, int BMT = BM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BNT == 32 ? (BMT == 32 ? 8 : DUCK_MLP_WPE) : 1))) void mlp_group_kernel(MlpGroupArgs g) {
  __shared__ __attribute__((aligned(16))) float As[tile_words<BMT, BMT>()], Bs[tile_words<BNT, BNT>()];
  const int b = blockIdx.x;
  int q = 0;
#pragma unroll
  for (int k = 1; k < DUCK_MLP_GROUP_MAX; k++) q += (k < g.n && b >= g.start[k]) ? 1 : 0;
  const duck_mlp_problem& p = g.p[q];
  const int t = b - g.start[q], gx = g.gx[q], gy = g.gy[q];
  const int bz = t / (gx * gy), rem = t - bz * gx * gy, by = rem / gx, bx = rem - by * gx;
  switch (p.kind) {
    case 0: gemm_tile<0, BNT, BMT>(bx, by, As, Bs, p.N, p.R, p.M, p.A, p.W, p.bias, p.aux, p.Y, p.Y2, p.mean, p.istd); break;
    case 1: gemm_tile<1, BNT, BMT>(bx, by, As, Bs, p.N, p.R, p.M, p.A, p.W, p.bias, p.aux, p.Y, p.Y2, p.mean, p.istd); break;
    case 2: gemm_tile<2, BNT, BMT>(bx, by, As, Bs, p.N, p.R, p.M, p.A, p.W, p.bias, p.aux, p.Y, p.Y2, nullptr, nullptr); break;
    default:
      wgrad_tile<BNT, BMT>(bx, by, bz, As, Bs, p.N, p.M, p.R, p.A, p.W, p.mean, p.istd, g.rps[q], p.partial, p.P,
                           p.off_w, p.off_b);
  }
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


// The learner's update after the gradient all-reduce, on the flat parameter / gradient / moment
// buffers of both networks (ppo.FusedGrad): torch.nn.utils.clip_grad_norm_ then torch.optim.Adam
// (optax.adam in brax: the same moments and bias corrections), in two launches instead of ~10.
// Launch 1: per-workgroup partial sums of g^2 (fixed order), and the step counter advanced (a
// captured graph replays with the device counter). Launch 2: every workgroup sums the partials in
// the same order (the same norm everywhere), scales by min(1, max_norm / (norm + 1e-6)) and applies
// m = b1 m + (1 - b1) g, v = b2 v + (1 - b2) g^2, p -= lr / (1 - b1^t) m / (sqrt(v) / sqrt(1 - b2^t) + eps).
constexpr int ADAM_TPB = 256, ADAM_PER = 8;  // a workgroup covers 2048 entries

__global__ __launch_bounds__(ADAM_TPB) void adam_norm_kernel(int P, const float* __restrict__ g,
                                                             float* __restrict__ partial, int* __restrict__ step) {
  __shared__ float red[ADAM_TPB / 64];
  const int base = blockIdx.x * ADAM_TPB * ADAM_PER;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < ADAM_PER; j++) {
    const int i = base + j * ADAM_TPB + threadIdx.x;
    const float x = i < P ? g[i] : 0.f;
    s += x * x;
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < ADAM_TPB / 64; w++) t += red[w];
    partial[blockIdx.x] = t;
    if (blockIdx.x == 0) *step += 1;
  }
}

// Launch 1 with the split-K weight-gradient partials summed first (duck_clip_adam_reduce, one rank): each
// thread forms its 8 gradient entries as duck_mlp_wgrad_reduce does (splits in order), stores them and
// sums their squares in adam_norm_kernel's order -- the same gradient and the same norm, one launch fewer.
__global__ __launch_bounds__(ADAM_TPB) void adam_reduce_norm_kernel(int P, int S, const float* __restrict__ part,
                                                                    float* __restrict__ g,
                                                                    float* __restrict__ partial,
                                                                    int* __restrict__ step) {
  __shared__ float red[ADAM_TPB / 64];
  const int base = blockIdx.x * ADAM_TPB * ADAM_PER;
  // (the 8 entries' sums side by side, split s outer: 8 independent loads per split in flight; each
  // entry still sums its splits in order)
  float gi[ADAM_PER];
#pragma unroll
  for (int j = 0; j < ADAM_PER; j++) gi[j] = 0.f;
  for (int s = 0; s < S; s++) {
    const float* ps = part + (size_t)s * P;
#pragma unroll
    for (int j = 0; j < ADAM_PER; j++) {
      const int i = base + j * ADAM_TPB + threadIdx.x;
      gi[j] += i < P ? ps[i] : 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < ADAM_PER; j++) {
    const int i = base + j * ADAM_TPB + threadIdx.x;
    if (i < P) g[i] = gi[j];
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < ADAM_PER; j++) s += gi[j] * gi[j];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < ADAM_TPB / 64; w++) t += red[w];
    partial[blockIdx.x] = t;
    if (blockIdx.x == 0) *step += 1;
  }
}

__global__ __launch_bounds__(ADAM_TPB) void adam_update_kernel(int P, int nblk, float* __restrict__ p,
                                                               const float* __restrict__ g, float* __restrict__ m,
                                                               float* __restrict__ v, const float* __restrict__ partial,
                                                               const int* __restrict__ step, float lr, float b1,
                                                               float b2, float eps, float max_norm) {
  // the partials' sum in one fixed order in every workgroup (the same norm everywhere): thread t sums
  // partials t, t + 256, .. in double, then the wave sums and the 4 wave totals in order. (A serial
  // sum on thread 0 -- 230 dependent loads at the learner's 0.47 M parameters -- took 3/4 of this
  // launch's 15.7 us, profiles/r06_ppo_trace_summary_before.txt)
  __shared__ double wsum[ADAM_TPB / 64];
  __shared__ float coef;
  {
    double t = 0.0;
    for (int b = threadIdx.x; b < nblk; b += ADAM_TPB) t += partial[b];
    for (int o = 32; o > 0; o >>= 1) t += __shfl_down(t, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < ADAM_TPB / 64; w++) t += wsum[w];
    const float norm = sqrtf((float)t);
    const float c = max_norm > 0.f ? max_norm / (norm + 1e-6f) : 1.f;
    coef = c < 1.f ? c : 1.f;
  }
  __syncthreads();
  const float k = coef;
  const float ts = (float)*step;
  const float bc1 = 1.f - powf(b1, ts), bc2s = sqrtf(1.f - powf(b2, ts));
  const float step_size = lr / bc1;
  const int base = blockIdx.x * ADAM_TPB * ADAM_PER;
#pragma unroll
  for (int j = 0; j < ADAM_PER; j++) {
    const int i = base + j * ADAM_TPB + threadIdx.x;
    if (i >= P) continue;
    const float gi = g[i] * k;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] -= step_size * mi / (sqrtf(vi) / bc2s + eps);
  }
}

}  // namespace

extern "C" int duck_mlp_gemm(int mode, int N, int R, int M, const float* A, const float* W, const float* bias,
                             const float* aux, float* Y, float* Y2, const float* mean, const float* istd,
                             void* stream) {
  if (N < 0 || R <= 0 || M <= 0) return duck_fail(DUCK_EINVAL, "duck_mlp_gemm: bad size");
  if (N == 0) return DUCK_OK;
  if (!A || !W || !Y || (mode == 1 && !Y2) || (mode == 2 && !aux) || (!mean) != (!istd))
    return duck_fail(DUCK_EINVAL, "duck_mlp_gemm: null pointer");
  const dim3 grid((N + BM - 1) / BM, (M + BN - 1) / BN);
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
  const dim3 grid((M + BM - 1) / BM, (K + 1 + BN - 1) / BN, splits);  // K + 1: the bias column
  hipLaunchKernelGGL(mlp_wgrad_kernel, grid, dim3(256), 0, (hipStream_t)stream, N, M, K, dZ, H, mean, istd, rps,
                     partial, P, off_w, off_b);
  HIPCHECK(hipGetLastError());
  return DUCK_OK;
}

extern "C" int duck_mlp_group_tiles(int n, const duck_mlp_problem* probs, int bm, int bn, void* stream) {
  if (n < 0 || n > DUCK_MLP_GROUP_MAX) return duck_fail(DUCK_EINVAL, "duck_mlp_group: 0 .. DUCK_MLP_GROUP_MAX problems");
  if (bn != 32 && bn != 64) return duck_fail(DUCK_EINVAL, "duck_mlp_group_bn: tile width 32 or 64");
  if ((bm != 32 && bm != BM) || (bm == 32 && bn != 32))
    return duck_fail(DUCK_EINVAL, "duck_mlp_group_tiles: tiles 64 x 32, 64 x 64 or 32 x 32");
  const int BN = bn, BM = bm;  // (shadow the default tile sizes for the grid arithmetic below)
  if (n == 0) return DUCK_OK;
  if (!probs) return duck_fail(DUCK_EINVAL, "duck_mlp_group: null pointer");
  MlpGroupArgs g;
  memset(&g, 0, sizeof(g));
  g.n = n;
  long long tot = 0;
  for (int k = 0; k < n; k++) {
    const duck_mlp_problem& p = probs[k];
    g.p[k] = p;
    g.start[k] = (int)tot;
    if (p.kind >= 0 && p.kind <= 2) {  // the checks of duck_mlp_gemm
      if (p.N < 0 || p.R <= 0 || p.M <= 0) return duck_fail(DUCK_EINVAL, "duck_mlp_group: bad gemm size");
      if (!p.A || !p.W || !p.Y || (p.kind == 1 && !p.Y2) || (p.kind == 2 && !p.aux) || (!p.mean) != (!p.istd) ||
          (p.kind == 2 && p.mean))
        return duck_fail(DUCK_EINVAL, "duck_mlp_group: bad gemm operands");
      g.gx[k] = (p.N + BM - 1) / BM;
      g.gy[k] = (p.M + BN - 1) / BN;
      tot += (long long)g.gx[k] * g.gy[k];
    } else if (p.kind == 3) {  // the checks of duck_mlp_wgrad (R = K inputs, M outputs)
      if (p.N <= 0 || p.M <= 0 || p.R <= 0 || p.splits <= 0) return duck_fail(DUCK_EINVAL, "duck_mlp_group: bad wgrad size");
      if (!p.A || !p.W || !p.partial || (!p.mean) != (!p.istd)) return duck_fail(DUCK_EINVAL, "duck_mlp_group: null pointer");
      if (p.off_w < 0 || p.off_b < 0 || (long long)p.off_w + (long long)p.M * p.R > p.P || p.off_b + p.M > p.P)
        return duck_fail(DUCK_EINVAL, "duck_mlp_group: offsets outside the parameter vector");
      g.gx[k] = (p.M + BM - 1) / BM;
      g.gy[k] = (p.R + 1 + BN - 1) / BN;
      g.rps[k] = (p.N + p.splits - 1) / p.splits;
      tot += (long long)g.gx[k] * g.gy[k] * p.splits;
    } else {
      return duck_fail(DUCK_EINVAL, "duck_mlp_group: kind must be 0, 1, 2 or 3");
    }
  }
  g.start[n] = (int)tot;
  for (int k = n; k <= DUCK_MLP_GROUP_MAX; k++) g.start[k] = (int)tot;
  if (tot == 0) return DUCK_OK;
  if (bn == 64)
    hipLaunchKernelGGL(mlp_group_kernel<64>, dim3((unsigned)tot), dim3(256), 0, (hipStream_t)stream, g);
  else if (bm == 32)
    hipLaunchKernelGGL((mlp_group_kernel<32, 32>), dim3((unsigned)tot), dim3(256), 0, (hipStream_t)stream, g);
  else
    hipLaunchKernelGGL(mlp_group_kernel<32>, dim3((unsigned)tot), dim3(256), 0, (hipStream_t)stream, g);
  HIPCHECK(hipGetLastError());
  return DUCK_OK;
}

extern "C" int duck_mlp_group_bn(int n, const duck_mlp_problem* probs, int bn, void* stream) {
  return duck_mlp_group_tiles(n, probs, BM, bn, stream);
}

extern "C" int duck_mlp_group(int n, const duck_mlp_problem* probs, void* stream) {
  return duck_mlp_group_bn(n, probs, 32, stream);
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

extern "C" int duck_clip_adam(int P, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                              float* scratch, int* step, float lr, float beta1, float beta2, float eps,
                              float max_norm, void* stream) {
  if (P <= 0) return duck_fail(DUCK_EINVAL, "duck_clip_adam: empty parameter vector");
  if (!param || !grad || !exp_avg || !exp_avg_sq || !scratch || !step)
    return duck_fail(DUCK_EINVAL, "duck_clip_adam: null pointer");
  const int nblk = (P + ADAM_TPB * ADAM_PER - 1) / (ADAM_TPB * ADAM_PER);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(adam_norm_kernel, dim3(nblk), dim3(ADAM_TPB), 0, st, P, grad, scratch, step);
  hipLaunchKernelGGL(adam_update_kernel, dim3(nblk), dim3(ADAM_TPB), 0, st, P, nblk, param, grad, exp_avg, exp_avg_sq,
                     scratch, step, lr, beta1, beta2, eps, max_norm);
  HIPCHECK(hipGetLastError());
  return DUCK_OK;
}

extern "C" int duck_clip_adam_reduce(int P, int splits, const float* partial, float* param, float* grad,
                                     float* exp_avg, float* exp_avg_sq, float* scratch, int* step, float lr,
                                     float beta1, float beta2, float eps, float max_norm, void* stream) {
  if (P <= 0 || splits <= 0) return duck_fail(DUCK_EINVAL, "duck_clip_adam_reduce: bad size");
  if (!partial || !param || !grad || !exp_avg || !exp_avg_sq || !scratch || !step)
    return duck_fail(DUCK_EINVAL, "duck_clip_adam_reduce: null pointer");
  const int nblk = (P + ADAM_TPB * ADAM_PER - 1) / (ADAM_TPB * ADAM_PER);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(adam_reduce_norm_kernel, dim3(nblk), dim3(ADAM_TPB), 0, st, P, splits, partial, grad, scratch,
                     step);
  hipLaunchKernelGGL(adam_update_kernel, dim3(nblk), dim3(ADAM_TPB), 0, st, P, nblk, param, grad, exp_avg, exp_avg_sq,
                     scratch, step, lr, beta1, beta2, eps, max_norm);
  HIPCHECK(hipGetLastError());
  return DUCK_OK;
}

extern "C" int duck_clip_adam_scratch_size(int P) { return (P + ADAM_TPB * ADAM_PER - 1) / (ADAM_TPB * ADAM_PER); }
