// Small fused kernels of the learner step (heads, losses, reductions, optimizer).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace acme {

// DuellingMLP head (acme/tf/networks/duelling.py:40-59) on the fused hidden layer
// h[rows][2H] (value hidden | advantage hidden):
//   v = h_v . wv + bv;  adv_a = h_a . wa[:, a] + ba[a];  q = v + (adv - mean_a(adv)).
int launch_duel_head(const float* h, int rows, int H, int A, const float* wv, const float* bv,
                     const float* wa, const float* ba, float* q, hipStream_t st);

// Backward of the duelling head for rows b < B with dq[b] = g[b] * onehot(a[b]):
// dZ_hidden (masked by the hidden ReLU) and the head weight / bias gradients.
int launch_duel_head_backward(const float* h, const float* g, const int32_t* a, int B, int H,
                              int A, const float* wv, const float* wa, float* dzh, float* dwv,
                              float* dbv, float* dwa, float* dba, hipStream_t st);

// dZ of a plain linear Q head: dz[b][j] = g[b] * (j == a[b]).
int launch_onehot_dq(const float* g, const int32_t* a, int B, int A, float* dz, hipStream_t st);

struct LossArgs {
  const float* q_on;  // [2B][A]: rows 0..B-1 q_tm1 (online o_tm1), B..2B-1 q_t_selector
  const float* q_tg;  // [B][A] q_t_value (target o_t)
  const int32_t* a;
  const float* r;
  const float* d;
  const double* probs;
  const double* global_min_prob;  // optional
  int B, A;
  float discount, beta, delta, max_abs_reward;
  float* loss;    // [1]
  float* td;      // [B]
  double* prio;   // [B]
  float* g;       // [B] dLoss / dq_tm1[b][a_b]
  int32_t* a_cache;
};
// trfl.double_qlearning + losses.huber + importance weighting + mean
// (acme/agents/tf/dqn/learning.py:128-144, acme/tf/losses/huber.py:45-57).
int launch_dqn_loss(const LossArgs& args, hipStream_t st);

// out[n] = sum_rows dz[row][n] (two deterministic passes through `partial`).
int launch_colsum(const float* dz, int64_t rows, int n, int chunks, float* partial, float* out,
                  hipStream_t st);
// out[i] = sum_{s < splits} slab[s][i] (fixed order).
int launch_slab_reduce(const float* slab, int splits, int64_t count, float* out, hipStream_t st);

}  // namespace acme
