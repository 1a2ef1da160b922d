/* duck_ppo.h — C ABI of the learner-side kernels of the PPO outer loop (libduck.so).
 *
 *   duck_gae       brax losses.compute_gae (the advantage/value-target recursion brax PPO runs in
 *                  its loss; the reference reaches it through ppo.train at common/runner.py:104-118)
 *   duck_ppo_loss  brax losses.compute_ppo_loss after GAE: clipped surrogate + value loss + entropy
 *                  bonus of one minibatch and its gradient w.r.t. the policy logits and the value
 *                  baseline (open_duck_playground_amd/ppo.py:ppo_loss is the same computation in torch)
 *   duck_gather_columns  a minibatch's trajectories out of the rollout buffers (all fields, one launch)
 *
 * Same conventions as duck.h: DEVICE pointers, float32, time-major [T][B] arrays (B = number of
 * trajectories, contiguous), `stream` a hipStream_t, negative return codes on error.
 */
#ifndef DUCK_PPO_H_
#define DUCK_PPO_H_

#ifdef __cplusplus
extern "C" {
#endif

/* The batch moments of brax running_statistics.update (ppo.RunningStatistics.update; brax
 * normalizes observations with it, the reference through ppo.train at common/runner.py:104-118):
 * x [N][F] float32 row-major -> out[f] = sum_n x[n][f], out[F + f] = sum_n x[n][f]^2, in fp64, in a
 * fixed order (two launches; the same bits on every run). scratch: duck_column_stats_scratch(N, F)
 * doubles of device memory. (Round 6: torch's fp64 column reductions took 1.8 ms per call.) */
int duck_column_stats(int N, int F, const float* x, double* out, double* scratch, void* stream);
int duck_column_stats_scratch(int N, int F);

/* vs[t][b], adv[t][b] from truncation/termination/reward/value [T][B] and bootstrap [B]:
 *   delta_t = (r_t + discount (1 - term_t) v_{t+1} - v_t)(1 - trunc_t),  v_T = bootstrap
 *   acc_t   = delta_t + discount (1 - term_t)(1 - trunc_t) lambda acc_{t+1},  vs_t = acc_t + v_t
 *   adv_t   = (r_t + discount (1 - term_t) vs_{t+1} - v_t)(1 - trunc_t),  vs_T = bootstrap */
/* duck_gae from the rollout's raw fields in one launch for B <= 1024 trajectories: termination =
 * done (1 - truncation), rewards scaled by reward_scale (brax's reward_scaling), then, when
 * normalize_advantage, stats[2] = {mean, 1 / (population std + 1e-8)} of all T x B advantages (else
 * {0, 1}) for duck_ppo_loss_stats. (Round 6: one launch instead of five per learner minibatch.) */
int duck_gae_stats(int T, int B, const float* truncation, const float* done, const float* reward, float reward_scale,
                   const float* value, const float* bootstrap, float lambda_, float discount, float* vs, float* adv,
                   int normalize_advantage, float* stats, void* stream);
int duck_gae(int T, int B, const float* truncation, const float* termination, const float* reward,
             const float* value, const float* bootstrap, float lambda_, float discount, float* vs, float* adv,
             void* stream);

/* The PPO loss of a minibatch of N samples, action size A (three launches; deterministic sums):
 *   logits [N][2A] (loc | pre-softplus scale), raw_action [N][A] (pre-tanh), old_logprob [N],
 *   advantage [N] (GAE, normalised inside when normalize_advantage: (a - mean) / (std + 1e-8)),
 *   value_target [N] (GAE vs), baseline [N] (value head), eps [N][A] (standard normal draws of the
 *   entropy estimate). scale = softplus(pre) + 1e-3; lp = sum_j log N(raw; loc, scale) - log|tanh'(raw)|;
 *   rho = exp(lp - old_logprob); policy = -mean(min(rho a, clip(rho, 1 - clip_eps, 1 + clip_eps) a));
 *   value = 0.25 mean((value_target - baseline)^2); entropy = mean sum_j (0.5 + 0.5 log 2 pi + log scale
 *   + log|tanh'(loc + scale eps)|). out[4] = {policy + value - entropy_cost entropy, policy, value,
 *   entropy}; grad_logits [N][2A], grad_baseline [N] = d out[0] / d logits, d out[0] / d baseline.
 *   out must hold duck_ppo_loss_out_size(N) floats (the rest is the launches' scratch). */
int duck_ppo_loss(int N, int A, const float* logits, const float* raw_action, const float* old_logprob,
                  const float* advantage, const float* value_target, const float* baseline, const float* eps,
                  float clip_eps, float entropy_cost, int normalize_advantage, float* out, float* grad_logits,
                  float* grad_baseline, void* stream);
/* duck_ppo_loss with the advantage statistics given (stats[2] = {mean, 1 / (std + 1e-8)} of the
 * advantages, as duck_gae_stats writes them; the advantages are normalised with them): one launch
 * fewer. Same out / gradient contract. (Round 6.) */
int duck_ppo_loss_stats(int N, int A, const float* logits, const float* raw_action, const float* old_logprob,
                        const float* advantage, const float* value_target, const float* baseline, const float* eps,
                        float clip_eps, float entropy_cost, const float* stats, float* out, float* grad_logits,
                        float* grad_baseline, void* stream);
/* duck_ppo_loss_stats without the loss sums (A <= 16): the gradients and the per-workgroup partial sums
 * only; duck_ppo_loss_sums(N, A, entropy_cost, out) forms out[0..3] from the partials the last call left
 * in out. The learner's epoch graph reports the last minibatch's loss only: one launch fewer for the
 * others. (Round 6.) */
int duck_ppo_loss_grad(int N, int A, const float* logits, const float* raw_action, const float* old_logprob,
                       const float* advantage, const float* value_target, const float* baseline, const float* eps,
                       float clip_eps, float entropy_cost, const float* stats, float* out, float* grad_logits,
                       float* grad_baseline, void* stream);
int duck_ppo_loss_sums(int N, int A, float entropy_cost, float* out, void* stream);
/* 4 + 2 + 3 ceil(N / 16): the length of duck_ppo_loss's out array (A <= 31) */
int duck_ppo_loss_out_size(int N);

/* One minibatch's trajectories out of the rollout buffers (brax ppo/train.py: the shuffled
 * jnp.take(data, permutation, axis=1) of each minibatch), every field in one launch: field f copies
 * dst[t][j][c] = src[t][idx[j]][c] for t < T_f, j < m, c < w_f (src [T_f][B_f][w_f], dst [T_f][m][w_f],
 * float32, row-major; idx int64 [m], each < B_f). At most DUCK_GATHER_MAX fields. */
#define DUCK_GATHER_MAX 8
typedef struct {
  const float* src;
  float* dst;
  int T, B, w;
} duck_gather_field;
int duck_gather_columns(int nfields, const duck_gather_field* fields, const long long* idx, int m, void* stream);
/* duck_gather_columns with an observation normaliser per field: norm[2 f], norm[2 f + 1] = mean[w_f],
 * 1 / std[w_f] (both NULL: a plain copy), dst = (src - mean[c]) * istd[c] -- the op(X) the first MLP
 * layers otherwise apply on their loads, in the same fp32 expression, so the results are unchanged.
 * (Round 6: the forward and weight-gradient GEMMs of the first layers then read plain rows.) */
int duck_gather_columns_norm(int nfields, const duck_gather_field* fields, const float* const* norm,
                             const long long* idx, int m, void* stream);

/* The policy / value MLP layers (brax ppo/networks.py: Dense + swish; nn.Linear weight layout
 * W [M][R] row-major, bias [M]) on fp32 MFMA, row-major activations [N][.]:
 *   mode 0  Y[N][M] = op(A)[N][R] W^T + b                    (the output layer)
 *   mode 1  Y = Z = op(A) W^T + b,  Y2 = silu(Z)             (a hidden layer: Z kept for the backward)
 *   mode 2  Y[N][M] = (A[N][R] W[R][M]) * silu'(aux[N][M])    (the data gradient: A = dZ of the layer
 *           above, W that layer's weight [R][M], aux = this layer's Z; bias, mean, istd unused)
 * op(A) = (A - mean) * istd per column when mean / istd are given (the observation normaliser), else A. */
int duck_mlp_gemm(int mode, int N, int R, int M, const float* A, const float* W, const float* bias, const float* aux,
                  float* Y, float* Y2, const float* mean, const float* istd, void* stream);
/* The weight gradient of one layer as `splits` partial products over row blocks of the batch:
 * partial[s][off_w + m K + k] = sum_{n in block s} dZ[n][m] op(H)[n][k], partial[s][off_b + m] =
 * sum_{n in block s} dZ[n][m]; P = the length of one partial (the network's parameter count), so all
 * layers of the networks share one partial array and one duck_mlp_wgrad_reduce. */
int duck_mlp_wgrad(int N, int M, int K, const float* dZ, const float* H, const float* mean, const float* istd,
                   int splits, float* partial, int P, int off_w, int off_b, void* stream);
/* Up to DUCK_MLP_GROUP_MAX independent layer problems in one launch (the policy's and the value
 * network's layers at one depth): kind 0, 1, 2 = duck_mlp_gemm's mode with (N, R, M, A, W, bias, aux,
 * Y, Y2, mean, istd); kind 3 = duck_mlp_wgrad with N rows, R = K inputs, M outputs, A = dZ, W = H,
 * mean, istd, splits, partial, P, off_w, off_b. The same results as the separate calls. */
#define DUCK_MLP_GROUP_MAX 4
typedef struct {
  int kind, N, R, M;
  const float *A, *W, *bias, *aux;
  float *Y, *Y2;
  const float *mean, *istd;
  int splits, P, off_w, off_b;
  float* partial;
} duck_mlp_problem;
int duck_mlp_group(int n, const duck_mlp_problem* problems, void* stream);
/* duck_mlp_group with output tiles 64 rows x `bn` columns (32 or 64; duck_mlp_group = 32). Every output
 * element's reduction runs in the same order whatever the tile, so the results are bit-identical;
 * 64-wide tiles halve the re-reads of the row operand for the wide layers. (Round 6.) */
int duck_mlp_group_bn(int n, const duck_mlp_problem* problems, int bn, void* stream);
/* duck_mlp_group with output tiles `bm` x `bn`: 64 x 32, 64 x 64 or 32 x 32 (bit-identical, as above). The
 * 32 x 32 tiles give a launch with few tiles and short reductions twice the workgroups (the learner's
 * third and fourth layers: 16 -> 12 us for the deepest backward launch). (Round 6.) */
int duck_mlp_group_tiles(int n, const duck_mlp_problem* problems, int bm, int bn, void* stream);
/* grad[i] = sum_{s < splits} partial[s][i] in order (deterministic), i < P */
int duck_mlp_wgrad_reduce(int P, int splits, const float* partial, float* grad, void* stream);
/* The rollout's policy sample (brax NormalTanhDistribution): for each of N rows of logits [N][2A]
 * (loc | pre-softplus scale), eps ~ N(0, 1) from threefry2x32 keyed by seed at counter (row,
 * 8 *ctr + pair) (Box-Muller), raw = loc + (softplus(pre) + 1e-3) eps -> raw [N][A], its NormalTanh
 * log-probability -> logprob [N], tanh(raw) -> action [N][A]; then *ctr += 1 (device counter: a
 * captured graph draws fresh noise on every replay). A <= 16. */
int duck_policy_sample(int N, int A, const float* logits, unsigned long long seed, unsigned int* ctr, float* raw,
                       float* logprob, float* action, void* stream);
/* The learner's parameter update on flat buffers of P floats (both networks): clip_grad_norm_(max_norm)
 * then Adam (torch.optim.Adam / optax.adam): g' = g min(1, max_norm / (|g| + 1e-6)),
 * m = b1 m + (1 - b1) g', v = b2 v + (1 - b2) g'^2, t = ++*step,
 * param -= lr / (1 - b1^t) m / (sqrt(v) / sqrt(1 - b2^t) + eps). Two launches; `step` a device int,
 * `scratch` duck_clip_adam_scratch_size(P) floats. */
int duck_clip_adam(int P, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, float* scratch,
                   int* step, float lr, float beta1, float beta2, float eps, float max_norm, void* stream);
int duck_clip_adam_scratch_size(int P);
/* duck_mlp_wgrad_reduce(P, splits, partial, grad) and duck_clip_adam in two launches instead of three
 * (one rank: no gradient all-reduce between them): grad is written as duck_mlp_wgrad_reduce writes it and
 * the update is bit-identical. (Round 6.) */
int duck_clip_adam_reduce(int P, int splits, const float* partial, float* param, float* grad, float* exp_avg,
                          float* exp_avg_sq, float* scratch, int* step, float lr, float beta1, float beta2, float eps,
                          float max_norm, void* stream);

#ifdef __cplusplus
}
#endif
#endif
