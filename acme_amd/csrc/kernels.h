// Small fused kernels of the learner step (head epilogues, losses, split-K reductions,
// optimizer).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

typedef struct acme_replay acme_replay;  // include/acme_hip.h

namespace acme {
namespace gemm {
struct PScale;  // gemm_p3.h: the scale record of a plane tensor
}

// Step guard of a learner on the f16 plane engine: the "skip the step on overflow" rule of
// automatic mixed precision (a step whose f16 planes overflowed changes no parameter, Adam
// moment or count, priority or target; the next step runs at rescaled planes).  Producers
// raise their record's flag word (gemm_p3.h PScale::flag -> on / tt / prm); the gated
// kernels read the Gate below before their first store; the end-of-step rescale counts the
// step as applied or skipped and clears the flags.  Device memory, one per learner.
struct StepGuard {
  uint32_t on;       // the online forward's and the backward's records, this step
  uint32_t tt;       // the target forward's records (the target rescale moves it to t[])
  uint32_t prm;      // the parameter planes written by Adam
  uint32_t last;     // the last step that ended was skipped (read after the step)
  uint32_t t[2];     // the target forward of step s overflowed: t[s & 1]
  uint32_t qv;       // the last q_values forward overflowed
  uint32_t hold;     // sticky skip (RescaleGuard::sticky): every later step skips until a
                     // calibration clears it, so the host can re-issue the skipped steps in order
  int64_t applied;   // updates applied: Adam's t - 1
  int64_t skipped;   // steps skipped
  uint32_t vseq;     // the last verdict: (seq << 1) | skip, one agent-scope store (the data
                     // is its own flag: readers in the same launch spin on it)
  uint32_t vtimeout; // priority write-backs that timed out waiting for vseq (and so wrote
                     // nothing): acme_dqn_verdict_timeouts; DQNLearner raises on one
};
// What a gated kernel reads: skip = on | t[par] | (dp && *dp > 0), or `last` (use_last).
struct Gate {
  const StepGuard* g = nullptr;  // null: never skip
  int par = 0;
  int use_last = 0;
  const float* dp = nullptr;  // the data-parallel ranks' gate, all-reduced (a gradient word)
};
__device__ __forceinline__ bool gate_skip(const Gate& q) {
  if (!q.g) return false;
  if (q.use_last) return q.g->last != 0u;
  return (q.g->on | q.g->t[q.par]) != 0u || (q.dp && *q.dp > 0.f);
}
// The end-of-step rescale's work on the guard (launch_plane_rescale).
enum RescaleMode {
  kRgNone = 0,
  kRgTarget = 1,   // after the target forward: t[par] = tt | rescaled bad, tt = 0
  kRgStep = 2,     // before Adam: last = skip, applied or skipped += 1, on = prm = 0
  kRgClear = 3,    // after calibration: every flag 0 (the counts kept)
  kRgQValues = 4,  // after q_values: qv = tt, tt = 0
  kRgFlag = 5,     // on |= a record overflowed or underflowed (IMPALA: folded by grad_sumsq)
};
struct RescaleGuard {
  StepGuard* g = nullptr;
  int mode = kRgNone;
  Gate gate{};                      // kRgStep: the step's gate
  int64_t* host_skipped = nullptr;  // kRgStep: pinned host mirror of g->skipped (optional)
  // kRgStep: the verdict's sequence number (the host's count of issued verdicts), published
  // as g->vseq and into the pinned ring host_verdicts[seq & 63] = (seq << 1) | skip (optional).
  uint32_t seq = 0;
  uint32_t* host_verdicts = nullptr;
  int sticky = 0;  // kRgStep: a skip sets g->hold (every later step skips until cleared)
  // kRgStep: a one-launch LSTM's timeout words (tmo[0] this step, tmo[1] the count): a
  // timed-out step is skipped too, tmo[0] cleared and counted (optional).
  uint32_t* tmo = nullptr;
};

// Finishes the duelling head GEMM (conv.h DuelHeadFwd): sums the split-K slab
// [splits][rows][A+1], adds biases and forms q = v + (adv - mean_a(adv))
// (acme/tf/networks/duelling.py:51-57).
int launch_duel_head_finish(const float* slab, int splits, int rows, int A, const float* bv,
                            const float* ba, float* q, hipStream_t st);

// dZ of the fused hidden layer for rows b < B with dq[b] = g[b] * onehot(a[b]), masked by
// the hidden ReLU.
// With `planes` non-null the result is written as scaled f16 planes (gemm_p3.h Planes,
// plane stride `pstride` elements, scale record sc) instead of f32 to dzh.
int launch_duel_head_dz(const float* h, const float* g, const int32_t* a, int B, int H, int A,
                        const float* wv, const float* wa, float* dzh, hipStream_t st,
                        uint16_t* planes = nullptr, int64_t pstride = 0,
                        gemm::PScale* sc = nullptr);

// Fused DQN head forward: hid = relu(sum_s slab[s] + fcb) ([rows][2H], written) and the
// duelling q = v + adv - mean(adv) from it (replaces the slab reduction + DuelHeadFwd +
// duel_head_finish of the f32 path).
int launch_fc_head_forward(const float* slab, int splits, int rows, int H, const float* fcb,
                           const float* wv, const float* bv, const float* wa, const float* ba,
                           int A, float* hid, float* q, hipStream_t st);
// launch_duel_head_dz writing planes, 8 units per thread.
int launch_head_dz_planes(const float* h, const float* g, const int32_t* a, int B, int H, int A,
                          const float* wv, const float* wa, uint16_t* planes, int64_t pstride,
                          gemm::PScale* sc, hipStream_t st);

// Sums the DuelHeadWgrad slab [splits][2H+1][A+1] and scatters its block-diagonal parts
// into the head weight / bias gradients.
int launch_duel_head_grad_scatter(const float* slab, int splits, int H, int A, float* dwv,
                                  float* dbv, float* dwa, float* dba, hipStream_t st,
                                  const double* part = nullptr, int64_t nparts = 0,
                                  int mean_over = 1, float* loss = nullptr);

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
  int mean_over;  // the loss / gradient mean's denominator (B, or the global share, DP)
  float discount, beta, delta, max_abs_reward;
  int jax;        // JAX DQNLearner: f32 importance weights (agents/jax/dqn/learning.py:94-96)
  float* loss;    // [1]
  float* td;      // [B]
  double* prio;   // [B]
  float* g;       // [B] dLoss / dq_tm1[b][a_b]
  int32_t* a_cache;
  // launch_dqn_loss_head_dz only (optional): every block writes the f64 sum of its rows'
  // weighted Huber losses here and no block reduces the batch; launch_dqn_loss_sum then
  // forms the loss (off the critical path, e.g. on the side stream).
  double* loss_part = nullptr;
};
// trfl.double_qlearning + losses.huber + importance weighting + mean
// (acme/agents/tf/dqn/learning.py:128-144, acme/tf/losses/huber.py:45-57).
int launch_dqn_loss(const LossArgs& args, hipStream_t st);
// The loss fused with the duelling head's dZ planes (as launch_head_dz_planes, from the
// hidden activations h [B][2H]): one launch, the same bits as the two kernels.
int launch_dqn_loss_head_dz(const LossArgs& args, const float* h, int H, const float* wv,
                            const float* wa, uint16_t* planes, int64_t pstride, gemm::PScale* sc,
                            hipStream_t st);
// Blocks of launch_dqn_loss_head_dz for a batch of B rows (the loss_part entries written).
int64_t dqn_loss_head_dz_blocks(int B, int H);
// The online duelling head (from the fc split-K slab of 2B rows: o_tm1 then o_t) fused with
// the loss and the head dZ planes: one block per batch row; writes hid, args.q_on, the
// loss outputs and args.loss_part[b] (B partials).  Nature head only (H = 512, A = 18,
// splits 4 or 8): dqn_head_loss_dz_fusable.
bool dqn_head_loss_dz_fusable(int H, int A, int splits, const float* wv, const float* wa,
                              const float* fcb);
int launch_dqn_head_loss_dz(const LossArgs& args, const float* slab, int splits, int H,
                            const float* fcb, const float* wv, const float* bv, const float* wa,
                            const float* ba, float* hid, uint16_t* planes, int64_t pstride,
                            gemm::PScale* sc, hipStream_t st);
// loss[0] = (sum of the n partials, in order) / mean_over.
int launch_dqn_loss_sum(const double* part, int64_t n, int mean_over, float* loss, hipStream_t st);

// Deterministic split-K reduction: e in [0, count): v = sum_s slab[s * count + e] (fixed
// order), optionally + bias[e % ncols] and ReLU; written to out0[e] for e < split_at and
// to out1[e - split_at] otherwise (weights and bias gradient of one slab).
int launch_slab_reduce(const float* slab, int splits, int64_t count, float* out0,
                       int64_t split_at, float* out1, const float* bias, int ncols, int relu,
                       hipStream_t st);

// Gradient global norms of two parameter groups ([0, group0_4) and [group0_4, n4) in
// float4 units): f64 partial sums of squares per block into part[2][nparts], fixed order.
// Block 0 also advances *dev_step (the Adam t read by launch_clip_adam), so a captured
// step graph needs no per-step host argument.  With a guard, block 0 first folds the step's
// flags (guard->on | *lstm_tmo) into guard->last and counts the step as applied (dev_step
// advanced) or skipped; launch_clip_adam then reads `last` (Gate::use_last).
int launch_grad_sumsq(const float* g, int64_t n4, int64_t group0_4, double* part, int nparts,
                      int64_t* dev_step, hipStream_t st, StepGuard* guard = nullptr,
                      uint32_t* lstm_tmo = nullptr, int64_t* host_skipped = nullptr);

// tf.clip_by_global_norm per group (scale = clip * min(1/G, 1/clip) when clipping) then
// snt.Adam with t = *dev_step and a per-group learning rate.  Optionally block 0 also
// reduces two per-row loss buffers: *out_x = sum(sum_x[0:n_x]) / div_x.
struct ClipAdamArgs {
  float *p = nullptr, *m = nullptr, *v = nullptr;
  const float* g = nullptr;
  int64_t n4 = 0, group0_4 = 0;
  const double* part = nullptr;
  int nparts = 0;
  int clipping = 0;
  float clip_norm = 1e10f;
  // optix.chain(clip_by_global_norm, adam) (agents/jax/impala/agent.py:98-101): g * (c / G)
  // only when G >= c, and the optix Adam update lr * (m_hat / (sqrt(v_hat) + eps)).
  int optix = 0;
  float lr0 = 0.f, lr1 = 0.f, b1 = 0.9f, b2 = 0.999f, eps = 1e-8f;
  const int64_t* dev_step = nullptr;
  float* norms = nullptr;  // [2] (optional)
  const float* sum_a = nullptr;
  int n_a = 0;
  float div_a = 1.f;
  float* out_a = nullptr;
  const float* sum_b = nullptr;
  int n_b = 0;
  float div_b = 1.f;
  float* out_b = nullptr;
  Gate gate{};  // skip: p, m, v unchanged
};
int launch_clip_adam(const ClipAdamArgs& a, hipStream_t st);

// snt.Adam over n (multiple of 4) floats at step t (acme_adam_update); with `planes`
// non-null the updated parameters are also written as f16 planes (stride pstride) at the
// scale record psc's w (the record's amax comes from launch_param_amax).
// optix != 0: optix.adam's rounding order, p + (-lr) * (m_hat / (sqrt(v_hat) + eps)).
// dev_steps (optional): the step count lives on the device (bias corrections computed by
// the kernel): with `count`, t = *dev_steps + 1 and a one-thread launch after Adam advances
// it; without, the caller's rescale before Adam has counted this step and t = *dev_steps.
// `t` is then ignored.
// gate: a skipped step leaves p, m and v as they are and rewrites the planes of p at psc->w
// (so the record's read scale stays that of the stored planes).  A plane write that
// overflows commits the wave's max |p| to psc and raises its flag.
// The step's scale-record bookkeeping, done by the Adam launch's first workgroup (Adam runs
// after every reader of the step's planes): the guard's flags cleared; the read scales of
// transient records a deferred rescale left (RescaleJob::defer_r) moved to their wi; the
// parameter record's r = the wi of the planes Adam writes (at w); a target copy of them takes
// the same r.
struct AdamTail {
  StepGuard* clear = nullptr;
  gemm::PScale* commit = nullptr;
  int ncommit = 0, skip_lo = -1, skip_hi = -1;
  gemm::PScale* params = nullptr;
  gemm::PScale* target = nullptr;
};
int launch_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1,
                float b2, float eps, int64_t t, uint16_t* planes, int64_t pstride, hipStream_t st,
                int optix = 0, int64_t* dev_steps = nullptr, gemm::PScale* psc = nullptr,
                const Gate& gate = Gate{}, bool count = true, const AdamTail& tail = AdamTail{});

// launch_adam (snt.Adam, t >= 1) with some gradient ranges still split-K slabs: segment k
// updates float4 [off4, off4 + n4) of the flat buffers from the deterministic reduction of
// float4 [e4, e4 + n4) of a slab of `splits` rows of count4 float4 (the reduction and the
// sums of launch_slab_reduce, bit for bit; the reduced gradient is also stored in g);
// [dense_off4, dense_off4 + dense_n4) from g.  One launch.
struct AdamSlabs {
  static constexpr int kMaxSegs = 8;
  struct Seg {
    int64_t off4, n4;
    const float* slab;
    int splits;
    int64_t count4, e4;
  } seg[kMaxSegs];
  int nseg = 0;
  int block_end[kMaxSegs] = {};  // filled by the launcher
  int64_t dense_off4 = 0, dense_n4 = 0;
};
// t = *dev_steps (this step counted by the caller's rescale before Adam); gate as launch_adam.
int launch_adam_slabs(float* p, float* g, float* m, float* v, const AdamSlabs& slabs,
                      float lr, float b1, float b2, float eps, const int64_t* dev_steps,
                      uint16_t* planes, int64_t pstride, gemm::PScale* psc, int optix,
                      const Gate& gate, const AdamTail& tail, hipStream_t st);

// Two-plane split of n floats (n multiple of 4): planes[i * pstride + e], at the scale of
// max |x| (sets the record sc: w, r = wi = 1 / w; overflow |= 1 on a non-finite x).
// keep_scale: a record whose current read scale suits max |x| keeps it (checkpoint restore).
int launch_split_planes(const float* x, int64_t n, uint16_t* planes, int64_t pstride,
                        gemm::PScale* sc, hipStream_t st, int* overflow = nullptr,
                        int keep_scale = 0);
// Planes of x at the record's current w, max |x| committed to its amax slots (the record is
// rescaled at the end of the step: lagged amax).  One launch.
int launch_split_planes_lagged(const float* x, int64_t n, uint16_t* planes, int64_t pstride,
                               gemm::PScale* sc, hipStream_t st);
// max |x| of n floats into the record's amax slots (the parameter planes' next scale).
int launch_param_amax(const float* x, int64_t n, gemm::PScale* sc, hipStream_t st);
// dst0 <- src0 and dst1 <- src1 (16-byte multiples) in one launch, unless the gate's step was
// skipped (the DQN target copy: a skipped step copies nothing).
int launch_copy_gated(void* dst0, const void* src0, size_t bytes0, void* dst1, const void* src1,
                      size_t bytes1, const Gate& gate, hipStream_t st);
// End-of-step rescale of a record array (kernels.hip plane_rescale_kernel): records
// [0, n_transient) transient, [n_transient, n) persistent (rewritten by every Adam pass);
// copy_to >= n, if >= 0, took a plane copy of copy_from's latest write.  Records in
// [skip_lo, skip_hi) are left alone (rescaled on the stream that writes them).  A record
// whose maximum is not finite (planes computed from overflowed planes) takes the largest
// scale reduction of the group's overflowed records with a finite maximum (its inputs
// shrink by that factor at their new scale), else 2^-16.  rg: the step guard's work.
int launch_plane_rescale(gemm::PScale* recs, int n_transient, int n, int copy_from, int copy_to,
                         int* overflow, hipStream_t st, int skip_lo = -1, int skip_hi = -1,
                         const RescaleGuard& rg = RescaleGuard{}, int defer_r = 0);
struct RescaleJob;  // rescale.h
int launch_rescale_job(const RescaleJob& job, hipStream_t st);
// The replay's update_priorities (replay.hip) behind a gate: a skipped step writes none.
// job (optional): a scale rescale (rescale.h) run by an extra workgroup of the update's
// launch (or its own launch when the update takes several), so the learner's step pays one
// kernel boundary for both.
int replay_update_priorities_gated(acme_replay* r, const uint64_t* keys, const double* prios,
                                   int64_t n, const Gate& gate, hipStream_t st,
                                   const RescaleJob* job = nullptr);
// Data-parallel gate: *dst = the step's local skip (1.f or 0.f), a gradient word that the
// ranks' all-reduce then combines (any rank's skip makes it > 0 on every rank).
int launch_gate_publish(const Gate& gate, float* dst, hipStream_t st,
                        const gemm::PScale* s = nullptr, int n = 0, int skip_lo = -1,
                        int skip_hi = -1);
// uint8 frames -> exact f16 (one plane): out[f][e] = f16(frame f byte e) for rows frames
// of `frame_bytes` (multiple of 8), frames [0, split) from a and the rest from b.
int launch_frames_f16(const uint8_t* a, const uint8_t* b, int split, int rows, int frame_bytes,
                      uint16_t* out, hipStream_t st);
// Inverse ((h + l) r in f32) for n elements.
int launch_join_planes(const uint16_t* planes, int64_t pstride, int64_t n, float* x,
                       const gemm::PScale* sc, hipStream_t st);

}  // namespace acme
