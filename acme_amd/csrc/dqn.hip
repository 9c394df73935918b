// DQN learner step for MI355X: the replacement of DQNLearner._step
// (acme/agents/tf/dqn/learning.py:112-168) behind the C ABI (include/acme_hip.h).
//
// One call = the whole SGD step on one stream, no host synchronisation:
//   online forward on [o_tm1; o_t] (2B rows, shared weights: q_tm1 and q_t_selector)
//   target forward on o_t (B rows: q_t_value)                        (:123-125)
//   fused loss kernel: reward clip, discount, double-Q target, TD,    (:128-144)
//     Huber(delta), f64 importance weights / max, weighted mean, |td| priorities
//   backward through the duelling head, FC and three convolutions    (:147)
//   snt.Adam over the flat parameter buffer                          (:148)
//   target <- online when num_steps % period == 0, then num_steps++  (:157-161)
//
// Networks: DQNAtariNetwork = AtariTorso + DuellingMLP([512])
// (acme/tf/networks/atari.py:36-69, duelling.py:27-59) or snt.nets.MLP([..., A])
// (examples/bsuite/run_dqn.py:46-49).  The duelling value/advantage first layers are
// fused into one [7744, 1024] GEMM (columns 0..511 value, 512..1023 advantage).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "conv.h"
#include "rescale.h"
#include "conv_p3.h"
#include "gemm.h"
#include "gemm_p3.h"
#include "gemm_x6.h"
#include "kernels.h"
#include "profiler.h"
#include "rccl_dyn.h"
#include "torso.h"

using namespace acme;
using namespace acme::conv;
using acme::gemm::launch_gemm;

namespace {

// Nature DQN torso geometry (TF SAME padding, NHWC): torso.h.
using torso::G1;
constexpr int kFlat = torso::kFlat;  // 7744
constexpr int kHidden = 512;          // DuellingMLP hidden size
constexpr int kObsBytes = 84 * 84 * 4;

struct Tensor {
  std::string name;
  int64_t offset = 0, numel = 0;
  int ndim = 0;
  int64_t shape[4] = {1, 1, 1, 1};
};

struct Layer {  // dense layer of the MLP network
  int in = 0, out = 0;
  int w = -1, b = -1;  // tensor indices
  bool relu = true;
};

}  // namespace

struct acme_dqn {
  acme_dqn_config cfg;
  std::vector<Tensor> tensors;
  int64_t flat = 0, logical = 0;
  float *params = nullptr, *target = nullptr, *grads = nullptr, *m = nullptr, *v = nullptr;
  int64_t num_steps = 0;
  // Nature tensors
  int t_c1w = -1, t_c1b, t_c2w, t_c2b, t_c3w, t_c3b, t_fcw, t_fcb, t_vw, t_vb, t_aw, t_ab;
  // MLP
  std::vector<Layer> layers;
  // Workspace (device)
  std::vector<void*> allocs;
  float *x1 = nullptr, *x2 = nullptr, *x3 = nullptr, *hid = nullptr;  // online (2B rows)
  float *t1 = nullptr, *t2 = nullptr, *t3 = nullptr, *thid = nullptr; // target (B rows)
  std::vector<float*> mlp_act, mlp_tact, mlp_dz;                     // MLP activations
  float *q_on = nullptr, *q_tg = nullptr;
  float *dzh = nullptr, *dz3 = nullptr, *dz2 = nullptr, *dz1 = nullptr;
  float* slab = nullptr;
  int64_t slab_floats = 0;
  bool stamps_on = false;      // ACME_V_STAMPS=1: the online fc_fwd launch stamps its phases
  uint64_t* stamps = nullptr;  // [4096][8] (debug_buffer "gemm_stamps")
  float* g = nullptr;  // per-sample dLoss/dq_tm1[a]
  int32_t* a_cache = nullptr;  // actions of the current batch (for the backward kernels)
  float* loss_tmp = nullptr;
  float* td_tmp = nullptr;
  double* prio_tmp = nullptr;
  // Plane path (gemm_p3.h; Nature network on uint8 frames): scaled two-plane f16 copies of
  // the parameters / target parameters ([2][flat]) and of every GEMM operand.
  bool p3_capable = false;
  bool planes_stale = true;  // parameter planes need a refresh from the f32 buffers
  bool last_p3 = false;      // the last forward/backward ran the plane path
  uint16_t *wpl = nullptr, *tpl = nullptr;
  // Scale records of the plane tensors (kScale* below) and the sticky overflow flag.
  gemm::PScale* scales = nullptr;
  int* overflow = nullptr;
  bool scales_ok = false;    // the activation / gradient scales are calibrated
  bool calibrating = false;
  int64_t fwd_batch = 0;  // rows of the last stage-2 forward awaiting its stage 3
  uint16_t* frames = nullptr;  // f16 copies of [o_tm1; o_t] (2B frames)
  // conv1's input of the current step (l->frames, the f16 copy).
  torso::Frames cur_frames{nullptr};
  // Second stream of the plane path: the target forward runs beside the online forward,
  // and weight gradients beside input gradients (fork / join by events on the caller's
  // stream; side_slab is its split-K scratch).
  hipStream_t side = nullptr;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  // Fused step (acme_dqn_step): the conv weight gradients stay split-K slabs and Adam
  // reduces them on its read (launch_adam_slabs): three reduction launches fewer.
  float* slab2 = nullptr;    // conv2's slab (conv3's is side_slab, conv1's slab)
  bool fused_step = false;   // set by step_impl
  // acme_dqn_step_update: the replay's priority write-back issued inside the step (on the
  // second stream right after the loss), keys of the step's batch.
  acme_replay* upd_replay = nullptr;
  const uint64_t* upd_keys = nullptr;
  hipEvent_t upd_after = nullptr;  // the table's last device read (the update waits for it)
  const double* upd_prio = nullptr;
  int upd_n = 0;
  bool slabs_pending = false;
  torso::WgradSlab wslabs[3];
  float* side_slab = nullptr;
  // The target forward's split-K slab (its own: the fused step's Adam reads side_slab while
  // the side stream may already run the next step's target forward).
  float* tslab = nullptr;
  // The target forward starts on the side stream without ordering after the caller's
  // stream (the batch's inputs event only), unless the caller's stream wrote target state
  // since the last step: a target copy, q_values' forward, calibration.  The target's
  // activation scale records (kScT1..kScT3) are rescaled on the side stream after it.
  bool target_dirty = true;
  torso::Plane x1p{}, x2p{}, x3p{}, t1p{}, t2p{}, t3p{}, dzhp{}, dz3p{}, dz2p{}, dz1p{};
  // Plane path: the loss is launched together with the head dZ (launch_dqn_loss_head_dz)
  // by the backward; forward_backward_stage leaves its arguments here.
  LossArgs pending_la{};
  bool loss_pending = false;
  // The online forward left its duelling head (the fc split-K slab's reduction, hid, q_on) to
  // the loss launch (launch_dqn_head_loss_dz, head_splits splits); loss_nparts: the loss
  // partials the launch writes.
  bool head_deferred = false;
  int head_splits = 0;
  int64_t loss_nparts = 0;
  // The dense layers' gradients (grads[grad_split:]) of the last stage 3 / 4 are complete
  // at dense_ev: the side stream's event when their launches ran there, else ev_dense,
  // recorded on the caller's stream.
  hipEvent_t ev_dense = nullptr;
  hipEvent_t dense_ev = nullptr;
  bool dense_on_side = false;
  // Data parallelism over a caller-owned RCCL communicator (acme_dqn_dp_*): the collective
  // stream, its events, the global IS normaliser's minimum probability.
  void* dp_comm = nullptr;
  int dp_world = 0;
  hipStream_t dp_stream = nullptr;
  hipEvent_t dp_ev[4] = {nullptr, nullptr, nullptr, nullptr};
  double* dp_gmin = nullptr;
  double* loss_part = nullptr;  // per-block loss partials of the fused loss + head dZ
  // Schedule variants fixed at creation (tests compare them bit for bit): one stream
  // (ACME_V_SIDE=1), the single-role GEMM kernels instead of the producer / consumer ones
  // (ACME_V_WSN=1).
  bool single_stream = false;
  bool single_role = false;
  // conv1 reads the batch's uint8 frames (unless the batch carries the f16 copy, obs_f16, or
  // the frames are not 16-byte aligned: then the step makes the f16 copy, the round-4 path)
  bool frames_u8 = true;
  // Step guard (kernels.h StepGuard): the skip-on-overflow rule of the plane engine, Adam's
  // device step count (applied updates) on every path.  seq counts the steps issued (the
  // target forward's flag slot is seq & 1); host_skipped is a pinned mirror of the skipped
  // count the end-of-step rescale writes (read by the host without a synchronisation).
  StepGuard* guard = nullptr;
  int64_t* host_skipped = nullptr;
  int64_t seq = 0;
  // Step verdicts (re-issue of skipped steps, DQNLearner): every step's rescale publishes
  // (verdict_seq << 1) | skip into the pinned ring host_verdicts[verdict_seq & 63], read by
  // the host without a synchronisation; with `sticky`, a skip holds every later step skipped
  // until a calibration clears it, so the host can re-issue the skipped steps in order.
  uint32_t* host_verdicts = nullptr;
  uint32_t verdict_seq = 0;
  bool sticky = false;
  // Data parallelism: the ranks' skip decisions are combined through a padding word of the
  // torso gradient bucket (stage 1 publishes the local one; the all-reduce combines them).
  bool dp_gate = false;
  int64_t dp_gate_index = -1;
  // The step's transient rescale ran inside the priority write-back's launch (deferred read
  // scales, committed by Adam): apply_impl launches none of its own.
  bool step_rescaled = false;
};

namespace {

int64_t align64(int64_t x) { return (x + 63) & ~int64_t(63); }

// Scale records (gemm_p3.h PScale) of the plane tensors: the transient activations and
// gradients of one step first, then the two persistent parameter-plane buffers.
enum {
  kScX1, kScX2, kScX3, kScT1, kScT2, kScT3, kScDzh, kScDz3, kScDz2, kScDz1,
  kScTransient,
  kScParams = kScTransient, kScTarget,
  kScCount
};
constexpr int64_t kParamAmaxPeriod = 8;
constexpr int kVerdictRing = 64;  // the pinned ring of step verdicts (acme_dqn_step_verdict)

int add_tensor(acme_dqn* l, const char* name, std::initializer_list<int64_t> shape) {
  Tensor t;
  t.name = name;
  t.ndim = (int)shape.size();
  t.numel = 1;
  int i = 0;
  for (int64_t s : shape) {
    t.shape[i++] = s;
    t.numel *= s;
  }
  t.offset = l->flat;
  l->flat = align64(l->flat + t.numel);
  l->logical += t.numel;
  l->tensors.push_back(t);
  return (int)l->tensors.size() - 1;
}

template <class T>
int dev_alloc(acme_dqn* l, T** p, int64_t count) {
  void* q = nullptr;
  if (hipMalloc(&q, std::max<int64_t>(count, 1) * sizeof(T)) != hipSuccess) {
    set_error("hipMalloc of %lld bytes failed", (long long)(count * sizeof(T)));
    return ACME_ERR_OOM;
  }
  l->allocs.push_back(q);
  *p = static_cast<T*>(q);
  return ACME_OK;
}

int plane_alloc(acme_dqn* l, torso::Plane* x, int64_t count, int rec) {
  const int64_t stride = align64(count);
  uint16_t* p = nullptr;
  int rc = dev_alloc(l, &p, gemm::kPlanes * stride);
  if (rc != ACME_OK) return rc;
  *x = torso::Plane{p, stride, l->scales + rec};
  return ACME_OK;
}

inline const float* P(const acme_dqn* l, const float* base, int t) {
  return base + l->tensors[t].offset;
}
inline float* Pm(const acme_dqn* l, float* base, int t) { return base + l->tensors[t].offset; }
// Plane view of parameter tensor t in a [2][flat] parameter-plane buffer (wpl or tpl, whose
// scale records are kScParams / kScTarget).
inline torso::Plane WP(const acme_dqn* l, uint16_t* base, int t) {
  return torso::Plane{base + l->tensors[t].offset, l->flat,
                      l->scales + (base == l->tpl ? kScTarget : kScParams)};
}
inline CPlanes CP(const torso::Plane& x) { return CPlanes{x.p, x.stride, x.sc}; }
inline gemm::PlaneSrc SRC(const torso::Plane& x, int64_t elems) {
  return gemm::PlaneSrc{x.p, x.stride, (int32_t)(2 * elems), x.sc};
}
// f16 frames of obs_a (rows [0, split)) and obs_b (the rest) into l->frames.
int convert_frames(acme_dqn* l, const void* obs_a, const void* obs_b, int split, int rows,
                   hipStream_t st) {
  ACME_PROF("frames_f16", st, 0.0, 3.0 * (double)rows * kObsBytes);
  return launch_frames_f16(static_cast<const uint8_t*>(obs_a), static_cast<const uint8_t*>(obs_b),
                           split, rows, kObsBytes, l->frames, st);
}
inline Planes PP(const torso::Plane& x) { return Planes{x.p, x.stride, x.sc}; }
bool use_p3(const acme_dqn* l) { return l->p3_capable && gemm::use_x6(); }
// The gate of the step in flight (seq): its online records' flags, its target forward's, and
// with data parallelism every rank's (the all-reduced padding word).
Gate step_gate(const acme_dqn* l) {
  Gate q;
  q.g = l->guard;
  q.par = (int)(l->seq & 1);
  if (l->dp_gate) q.dp = l->grads + l->dp_gate_index;
  return q;
}
// Clears the guard's flags (not its counts) after a calibration.
int clear_guard_flags(acme_dqn* l, hipStream_t st) {
  ACME_HIP_TRY(hipMemsetAsync(l->guard, 0, offsetof(StepGuard, applied), st));
  return ACME_OK;
}
// The side stream is used unless the section profiler is on: profiled passes run every
// kernel alone on one stream, so their per-kernel durations are uncontended.
hipStream_t side_stream(const acme_dqn* l) { return prof::enabled() ? nullptr : l->side; }

// Split-K helper: chunk size (multiple of BK) for `splits` splits of K.
inline int chunk_for(int K, int splits) {
  int c = (int)ceil_div(K, splits);
  return (int)ceil_div(c, 32) * 32;
}

#define ACME_GEMM(BM, BN, WM, WN, prob, splits)                                      \
  do {                                                                               \
    hipError_t _e = gemm::launch_matmul<BM, BN, WM, WN>(prob, splits, st);          \
    if (_e != hipSuccess) {                                                          \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                           \
    }                                                                                \
  } while (0)
// Profiled launch: `flops` = algorithmic FLOPs of the launch (2 * useful MACs).
#define ACME_GEMM_F(name, flops, BM, BN, WM, WN, prob, splits) \
  do {                                                          \
    ACME_PROF_PEAK(name, st, (double)(flops), 0.0,              \
                   (gemm::matmul_peak_tflops<1, decltype(prob)>())); \
    ACME_GEMM(BM, BN, WM, WN, prob, splits);                    \
  } while (0)
#define ACME_GEMM_N(name, BM, BN, WM, WN, prob, splits) \
  ACME_GEMM_F(name, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, BM, BN, WM, WN, prob, splits)

// Same with an explicit reduction stage depth BK (16 or 32).
#define ACME_GEMM_NK(name, BM, BN, WM, WN, BKV, prob, splits)                                 \
  do {                                                                                         \
    ACME_PROF_PEAK(name, st, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, 0.0, \
                   (gemm::matmul_peak_tflops<1, decltype(prob)>()));                             \
    hipError_t _e = gemm::launch_matmul<BM, BN, WM, WN, BKV>(prob, splits, st);               \
    if (_e != hipSuccess) {                                                                    \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                     \
    }                                                                                          \
  } while (0)

#define ACME_P3_GEMM(name, BM, BN, WM, WN, BKV, prob, splits)                                \
  do {                                                                                         \
    ACME_PROF_PEAK(name, st, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, 0.0, \
                   gemm::p3_peak_tflops<decltype(prob)>());                                    \
    hipError_t _e = gemm::launch_gemm_p3<BM, BN, WM, WN, BKV>(prob, splits, st);              \
    if (_e != hipSuccess) {                                                                    \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                     \
    }                                                                                          \
  } while (0)

// Warp-specialised plane GEMM (gemm_p3ws_kernel: producer and consumer waves).
#define ACME_P3WS_GEMM(name, BM, BN, WM, WN, BKV, prob, splits, PIPE)                        \
  do {                                                                                         \
    ACME_PROF_PEAK(name, st, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, 0.0, \
                   gemm::p3_peak_tflops<decltype(prob)>());                                    \
    hipError_t _e = gemm::launch_gemm_p3ws<BM, BN, WM, WN, BKV, PIPE>(prob, splits, st);      \
    if (_e != hipSuccess) {                                                                    \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                     \
    }                                                                                          \
  } while (0)
#define ACME_P3G_GEMM(name, BM, BN, WM, WN, BKV, ST, prob, splits)                            \
  do {                                                                                         \
    ACME_PROF_PEAK(name, st, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, 0.0, \
                   gemm::p3_peak_tflops<decltype(prob)>());                                    \
    hipError_t _e = gemm::launch_gemm_p3g<BM, BN, WM, WN, BKV, ST>(prob, splits, st);         \
    if (_e != hipSuccess) {                                                                    \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                     \
    }                                                                                          \
  } while (0)

// Split counts (K-splits) of the launches whose natural grid is too small to fill 256 CUs.
constexpr int kFcFwdSplits = 8;  // [rows, 1024] x K 7744: 128x128 tiles: 8x8x8 = 512 blocks (online)
constexpr int kHeadFwdSplits = 16;  // [rows, A+1] x K 1024
constexpr int kHeadBwdSplits = 8;   // [1024, A+1] x K = batch

int64_t slab_floats_needed(int B, int A) {
  return std::max<int64_t>({torso::wgrad_slab_floats(), (int64_t)kFcFwdSplits * 2 * B * 2 * kHidden,
                            (int64_t)kHeadFwdSplits * 2 * B * (A + 1),
                            (int64_t)kHeadBwdSplits * (2 * kHidden + 1) * (A + 1)});
}

int slab_reduce(const float* slab, int splits, int64_t count, float* out0, int64_t split_at,
                float* out1, const float* bias, int ncols, int relu, const char* name,
                hipStream_t st) {
  ACME_PROF(name, st, 0.0, 4.0 * (double)(splits + 1) * (double)count);
  return launch_slab_reduce(slab, splits, count, out0, split_at, out1, bias, ncols, relu, st);
}

// snt.Adam over the flat range [off, off + n) (tensor-aligned): the parameter planes (plane
// path) are refreshed by the same pass.  t = num_steps + 1 (snt.Adam / optix.adam count this
// step first).  Every element's update is independent, so ranges compose bit-exactly.
int adam_range(acme_dqn* l, int64_t off, int64_t n, const Gate& gate, const AdamTail& tail,
               hipStream_t st) {
  const bool jax = l->cfg.semantics == ACME_SEMANTICS_JAX;
  // Plane path: the step's gate and count from the rescale before Adam; otherwise no gate
  // (f32 tensors cannot overflow) and a one-thread count after Adam.
  const bool p3 = l->p3_capable;
  return launch_adam(l->params + off, l->grads + off, l->m + off, l->v + off, n,
                     l->cfg.learning_rate, l->cfg.adam_beta1, l->cfg.adam_beta2,
                     l->cfg.adam_epsilon, 0, p3 ? l->wpl + off : nullptr, l->flat, st, jax ? 1 : 0,
                     &l->guard->applied, p3 ? l->scales + kScParams : nullptr, gate, !p3, tail);
}

torso::Weights torso_weights(const acme_dqn* l, const float* prm) {
  return torso::Weights{P(l, prm, l->t_c1w), P(l, prm, l->t_c1b), P(l, prm, l->t_c2w),
                        P(l, prm, l->t_c2b), P(l, prm, l->t_c3w), P(l, prm, l->t_c3b)};
}

// Duelling value/advantage outputs as one skinny split-K GEMM + epilogue kernel.
int head_forward(acme_dqn* l, const float* prm, int rows, const float* hid, float* q,
                 hipStream_t st) {
  const int A = l->cfg.num_actions;
  DuelHeadFwd p;
  p.M = rows; p.N = A + 1; p.K = 2 * kHidden; p.k_chunk = chunk_for(p.K, kHeadFwdSplits);
  p.H = kHidden; p.A = A; p.h = hid; p.wv = P(l, prm, l->t_vw); p.wa = P(l, prm, l->t_aw);
  p.slab = l->slab;
  ACME_GEMM_N("head_fwd", 64, 32, 2, 1, p, kHeadFwdSplits);
  ACME_PROF("head_fwd_finish", st, 0.0, 0.0);
  return launch_duel_head_finish(l->slab, kHeadFwdSplits, rows, A, P(l, prm, l->t_vb),
                                 P(l, prm, l->t_ab), q, st);
}

// ---------------------------------------------------------------- Nature forward
// rows = number of observations; first `split` rows from obs_a, the rest from obs_b.
int nature_forward(acme_dqn* l, const float* prm, const void* obs_a, const void* obs_b,
                   int split, int rows, float* x1, float* x2, float* x3, float* hid,
                   float* q, hipStream_t st) {
  const bool u8 = l->cfg.obs_dtype == ACME_OBS_U8_SCALED;
  int rc0 = torso::forward(torso_weights(l, prm), u8, obs_a, obs_b, split, rows,
                           torso::Acts{x1, x2, x3}, st);
  if (rc0 != ACME_OK) return rc0;
  {  // Fused duelling hidden layer, split-K partials then bias + ReLU in the reduction.
    DenseFwd<true> p;
    const int splits = kFcFwdSplits;
    p.M = rows; p.N = 2 * kHidden; p.K = kFlat; p.k_chunk = chunk_for(kFlat, splits);
    p.x = x3; p.x2 = x3; p.split_b = rows; p.ldx = kFlat;
    p.w = P(l, prm, l->t_fcw); p.bias = P(l, prm, l->t_fcb); p.y = hid; p.act = ACT_RELU;
    p.slab = l->slab;
    ACME_GEMM_NK("fc_fwd", 128, 128, 2, 2, 32, p, splits);
    const int64_t cnt = (int64_t)rows * 2 * kHidden;
    int rc = slab_reduce(l->slab, splits, cnt, hid, cnt, nullptr, P(l, prm, l->t_fcb),
                         2 * kHidden, 1, "fc_fwd_reduce", st);
    if (rc != ACME_OK) return rc;
  }
  return head_forward(l, prm, rows, hid, q, st);
}

// Nature forward on the plane path: torso and the fused hidden layer read f16 planes
// (gemm_p3.h); `wpl` are the planes of `prm`.
int nature_forward_p3(acme_dqn* l, const float* prm, uint16_t* wpl, const torso::Frames& frames,
                      int rows, const torso::Plane& x1, const torso::Plane& x2,
                      const torso::Plane& x3, float* hid, float* q, hipStream_t st,
                      float* slab = nullptr, int keep_x1 = -1, bool defer_head = false) {
  if (!slab) slab = l->slab;
  torso::PWeights w{WP(l, wpl, l->t_c1w), WP(l, wpl, l->t_c2w), WP(l, wpl, l->t_c3w),
                    P(l, prm, l->t_c1b), P(l, prm, l->t_c2b), P(l, prm, l->t_c3b)};
  int rc = torso::forward_p3(w, frames, rows, torso::PActs{x1, x2, x3}, st, keep_x1);
  if (rc != ACME_OK) return rc;
  {
    P3DenseFwd p;
    // Split-K 8: about one round of blocks (one block per CU at BK 32): the online forward's
    // 2B = 1024 rows on 256x128 tiles (4 x 8 x 8), the target's 512 rows on 128x128.  The
    // taller tile takes in 24 KB per k16 step for 768 MFMA cycles against 16 KB per 384
    // (per-CU L2 intake): fc_fwd 47.0 -> 45.3 us, step 0.5037 -> 0.5028 ms
    // over 200 steps and 0.5146 -> 0.5084 ms over 20-step windows (three alternating pairs,
    // round 4; it had split-K 4 on 128x128 tiles).
    // The target forward at the headline batch (512 rows) on 256x128 tiles too, at split-K 8
    // (2 x 8 x 8 = 128 blocks, half the CUs; its head sums 8 partials).  It runs on the side
    // stream with ~100 us of slack before the loss, beside the online conv1 / conv2 forward:
    // with half the blocks it leaves half the CUs to them and writes half the partial tile
    // bytes.  Round 6: step 0.4744 -> 0.4678 ms (six alternating 300-step pairs) and 0.4803
    // -> 0.4729 ms over the driver's 20-step window (three pairs) against split-K 16 (256
    // blocks; round 4 had measured 16 against 8 as equal on that schedule); split-K 4: 0.4709.
    const bool tall = rows > 512;
    const bool ttall = rows == 512 && !defer_head;
    const int splits = kFcFwdSplits;
    p.M = rows; p.N = 2 * kHidden; p.K = kFlat; p.k_chunk = chunk_for(kFlat, splits);
    p.a_src = SRC(x3, (int64_t)rows * kFlat); p.ldx = kFlat;
    p.b_src = SRC(WP(l, wpl, l->t_fcw), (int64_t)kFlat * 2 * kHidden); p.slab = slab;
    if (tall) p.stamps = l->stamps;
    // Producer / consumer waves with fragment reads one k16 step ahead (gemm_p3ws_kernel):
    // 65.2 -> 60.5 us against the single-role kernel, the same bits.
    // (Two f16 planes, measured on the step: 256x128 / 128x256 WS tiles, 256x128 single-role
    // tiles with split-K 8, and the LDS-DMA ring (3 or 4 stages) all slower or equal.)
    // (The target launch is its own profiler section: bench.py reports both launches as
    // fc_fwd and each one apart.)
    if (ttall && l->single_role) ACME_P3_GEMM("fc_fwd_target", 256, 128, 2, 2, 32, p, splits);  // tests
    else if (ttall) ACME_P3WS_GEMM("fc_fwd_target", 256, 128, 2, 2, 32, p, splits, true);
    else if (tall && l->single_role) ACME_P3_GEMM("fc_fwd", 256, 128, 2, 2, 32, p, splits);  // tests
    else if (tall) ACME_P3WS_GEMM("fc_fwd", 256, 128, 2, 2, 32, p, splits, true);
    else if (l->single_role) ACME_P3_GEMM("fc_fwd", 128, 128, 2, 2, 32, p, splits);  // tests
    else ACME_P3WS_GEMM("fc_fwd", 128, 128, 2, 2, 32, p, splits, true);
    // The online forward of a step: the head runs inside the loss launch (nature_backward).
    if (defer_head &&
        dqn_head_loss_dz_fusable(kHidden, l->cfg.num_actions, splits, P(l, prm, l->t_vw),
                                 P(l, prm, l->t_aw), P(l, prm, l->t_fcb))) {
      l->head_deferred = true;
      l->head_splits = splits;
      return ACME_OK;
    }
    ACME_PROF("fc_head_fwd", st, 0.0, 4.0 * (double)rows * 2 * kHidden * (splits + 1));
    return launch_fc_head_forward(slab, splits, rows, kHidden, P(l, prm, l->t_fcb),
                                  P(l, prm, l->t_vw), P(l, prm, l->t_vb), P(l, prm, l->t_aw),
                                  P(l, prm, l->t_ab), l->cfg.num_actions, hid, q, st);
  }
}

// ---------------------------------------------------------------- MLP forward
template <class In>
int mlp_layer(acme_dqn* l, const float* prm, const Layer& L, const void* a, const void* b,
              int split, int rows, float* y, hipStream_t st) {
  const bool vec = L.in % 4 == 0 && L.out % 4 == 0;
  if (vec) {
    DenseFwd<true, In> p;
    p.M = rows; p.N = L.out; p.K = L.in; p.k_chunk = L.in;
    p.x = static_cast<const typename In::T*>(a); p.x2 = static_cast<const typename In::T*>(b);
    p.split_b = split; p.ldx = L.in; p.w = P(l, prm, L.w); p.bias = P(l, prm, L.b); p.y = y;
    p.act = L.relu ? ACT_RELU : ACT_NONE;
    ACME_GEMM_N("mlp_fwd", 64, 64, 2, 2, p, 1);
  } else {
    DenseFwd<false, In> p;
    p.M = rows; p.N = L.out; p.K = L.in; p.k_chunk = L.in;
    p.x = static_cast<const typename In::T*>(a); p.x2 = static_cast<const typename In::T*>(b);
    p.split_b = split; p.ldx = L.in; p.w = P(l, prm, L.w); p.bias = P(l, prm, L.b); p.y = y;
    p.act = L.relu ? ACT_RELU : ACT_NONE;
    ACME_GEMM_N("mlp_fwd", 64, 64, 2, 2, p, 1);
  }
  return ACME_OK;
}

int mlp_forward(acme_dqn* l, const float* prm, const void* obs_a, const void* obs_b, int split,
                int rows, std::vector<float*>& act, float* q, hipStream_t st) {
  const int nl = (int)l->layers.size();
  for (int i = 0; i < nl; ++i) {
    const Layer& L = l->layers[i];
    float* y = i == nl - 1 ? q : act[i];
    int rc;
    if (i == 0) {
      rc = l->cfg.obs_dtype == ACME_OBS_U8_SCALED
               ? mlp_layer<InU8>(l, prm, L, obs_a, obs_b, split, rows, y, st)
               : mlp_layer<InF32>(l, prm, L, obs_a, obs_b, split, rows, y, st);
    } else {
      rc = mlp_layer<InF32>(l, prm, L, act[i - 1], act[i - 1], rows, rows, y, st);
    }
    if (rc != ACME_OK) return rc;
  }
  return ACME_OK;
}

// The step's transient rescale and skip decision (the guard's kRgStep): every plane of the
// online forward and the backward is written by now; the target forward's records have their
// own rescale.  defer_r: consumers may still read the planes on the second stream.
RescaleJob step_rescale_job(acme_dqn* l, bool defer_r) {
  RescaleJob j;
  j.s = l->scales;
  j.nt = j.n = kScTransient;
  j.overflow = l->overflow;
  j.skip_lo = kScT1;
  j.skip_hi = kScT3 + 1;
  j.defer_r = defer_r ? 1 : 0;
  j.rg.g = l->guard;
  j.rg.mode = kRgStep;
  j.rg.gate = step_gate(l);
  j.rg.host_skipped = l->host_skipped;
  j.rg.host_verdicts = l->host_verdicts;
  j.rg.seq = l->verdict_seq++;
  j.rg.sticky = l->sticky ? 1 : 0;
  return j;
}

// The step's priority write-back (acme_dqn_step_update), once, on `st`, with the step's
// rescale in an extra workgroup of its launch (one kernel boundary fewer on the step's
// critical path; the read scales are committed by Adam, after the second stream's weight
// gradients that still read the planes).
int priority_update_tail(void* ctx, hipStream_t st) {
  acme_dqn* l = static_cast<acme_dqn*>(ctx);
  acme_replay* r = l->upd_replay;
  if (!r || !l->upd_prio) return ACME_OK;
  l->upd_replay = nullptr;
  if (l->upd_after) ACME_HIP_TRY(hipStreamWaitEvent(st, l->upd_after, 0));
  // Gated: a step that overflowed writes no priority.
  const RescaleJob job = step_rescale_job(l, true);
  const int rc =
      replay_update_priorities_gated(r, l->upd_keys, l->upd_prio, l->upd_n, step_gate(l), st, &job);
  if (rc == ACME_OK) l->step_rescaled = true;
  return rc;
}

// join_dense: the caller's stream waits for the side stream's dense weight gradients
// before returning (stage 0 of a data-parallel step all-reduces them next); otherwise the
// torso backward's final join covers them.
int nature_backward(acme_dqn* l, const void* o_tm1, int B, hipStream_t st_main,
                    bool join_dense) {
  hipStream_t st = st_main;
  const float* prm = l->params;
  float* gr = l->grads;
  const int A = l->cfg.num_actions;
  const bool p3 = use_p3(l);
  int rc;
  // The fused kernel leaves the batch loss as per-block partials; their sum is the side
  // stream's first launch (off the critical path: folding it into the fused kernel's last
  // block to finish measured 14.6 -> 20.5 us on the critical path).
  bool loss_sum = false;
  const LossArgs la = l->pending_la;
  if (p3 && l->loss_pending && l->head_deferred) {  // online head + loss + head dZ, one launch
    l->loss_pending = l->head_deferred = false;
    loss_sum = true;
    l->loss_nparts = B;
    ACME_PROF("head_loss_dz", st, 0.0, 4.0 * (double)2 * B * 2 * kHidden * (l->head_splits + 1));
    rc = launch_dqn_head_loss_dz(la, l->slab, l->head_splits, kHidden, P(l, prm, l->t_fcb),
                                 P(l, prm, l->t_vw), P(l, prm, l->t_vb), P(l, prm, l->t_aw),
                                 P(l, prm, l->t_ab), l->hid, l->dzhp.p, l->dzhp.stride,
                                 l->dzhp.sc, st);
    if (rc != ACME_OK) return rc;
  } else if (p3 && l->loss_pending) {  // the loss and the head dZ planes, one launch
    l->loss_pending = false;
    loss_sum = la.loss_part != nullptr;
    l->loss_nparts = dqn_loss_head_dz_blocks(B, kHidden);
    ACME_PROF("loss_head_dz", st, 0.0, 0.0);
    rc = launch_dqn_loss_head_dz(la, l->hid, kHidden, P(l, prm, l->t_vw),
                                 P(l, prm, l->t_aw), l->dzhp.p, l->dzhp.stride, l->dzhp.sc, st);
    if (rc != ACME_OK) return rc;
  } else {  // Head: dZ of the fused hidden layer (masked by its ReLU).
    ACME_PROF("head_dz", st, 0.0, 0.0);
    rc = p3 ? launch_head_dz_planes(l->hid, l->g, l->a_cache, B, kHidden, A, P(l, prm, l->t_vw),
                                    P(l, prm, l->t_aw), l->dzhp.p, l->dzhp.stride, l->dzhp.sc, st)
            : launch_duel_head_dz(l->hid, l->g, l->a_cache, B, kHidden, A, P(l, prm, l->t_vw),
                                  P(l, prm, l->t_aw), l->dzh, st);
    if (rc != ACME_OK) return rc;
  }
  // Weight gradients (head, then FC) on the side stream beside the FC input gradient.
  const bool fork = p3 && side_stream(l);
  float* hslab = fork ? l->side_slab : l->slab;
  if (fork) {
    ACME_HIP_TRY(hipEventRecord(l->ev[2], st_main));
    ACME_HIP_TRY(hipStreamWaitEvent(l->side, l->ev[2], 0));
    st = l->side;
  }
  if (p3 && l->upd_replay && !l->calibrating) {
    l->upd_prio = la.prio;
    l->upd_n = B;
    // Issued at the end of the main stream's torso backward, before the join
    // (priority_update_tail); on the second stream right after the loss its backward ended
    // ~20 us after the main stream's.
  }
  // The batch loss is summed by the head-gradient scatter's extra block (below): a launch of
  // its own on the second stream measured 0.5107 -> 0.5235 ms per step.
  const bool sum_in_scatter = loss_sum;
  {  // Head weight / bias gradients: one skinny GEMM over the batch + scatter.  (One
     // launch without split-K, 64 units per block and the batch over 8 waves, took 38 us
     // against 9.3 + 6.7: 17 blocks cannot hide the row loads.)
    DuelHeadWgrad p;
    p.M = 2 * kHidden; p.N = A + 1; p.K = B; p.k_chunk = chunk_for(B, kHeadBwdSplits);
    p.A = A; p.h = l->hid; p.g = l->g; p.act = l->a_cache; p.slab = hslab;
    ACME_GEMM_N("head_wgrad", 64, 32, 2, 1, p, kHeadBwdSplits);
    ACME_PROF("head_wgrad_scatter", st, 0.0, 0.0);
    rc = launch_duel_head_grad_scatter(
        hslab, kHeadBwdSplits, kHidden, A, Pm(l, gr, l->t_vw), Pm(l, gr, l->t_vb),
        Pm(l, gr, l->t_aw), Pm(l, gr, l->t_ab), st, sum_in_scatter ? la.loss_part : nullptr,
        l->loss_nparts, la.mean_over, la.loss);
    if (rc != ACME_OK) return rc;
  }
  if (p3) {
    {  // FC weight + bias grad: [7744, 1024] = x3^T dZh (reduction over the batch).
      P3DenseWgrad p;
      p.M = kFlat; p.N = 2 * kHidden; p.K = B; p.k_chunk = B;
      p.a_src = SRC(l->x3p, (int64_t)B * kFlat); p.ldx = kFlat;
      p.b_src = SRC(l->dzhp, (int64_t)B * 2 * kHidden); p.out = Pm(l, gr, l->t_fcw);
      p.bias_out = Pm(l, gr, l->t_fcb);
      // (Producer / consumer waves measured slower here on the step: 0.698 -> 0.72-0.73 ms.)
      // (256x128 warp-specialised tiles: 29.1 -> 30.1 us, round 4.)
      ACME_P3_GEMM("fc_wgrad", 128, 128, 2, 2, 16, p, 1);
    }
    if (fork) {
      ACME_HIP_TRY(hipEventRecord(l->ev[3], l->side));
      st = st_main;
    }
    {  // FC input grad -> dZ3 planes (masked by conv3's ReLU).
      P3DenseDgrad p;
      p.M = B; p.N = kFlat; p.K = 2 * kHidden; p.k_chunk = p.K;
      p.a_src = SRC(l->dzhp, (int64_t)B * 2 * kHidden);
      p.b_src = SRC(WP(l, l->wpl, l->t_fcw), (int64_t)kFlat * 2 * kHidden); p.xprev = CP(l->x3p);
      p.ldx = kFlat; p.dx = PP(l->dz3p);
      // LDS-DMA staging (gemm_p3.h P3G) measured fastest for this shape.
      // Producer / consumer waves (gemm_p3ws_kernel): 51.4 -> 47.3 us against the LDS-DMA
      // ring, the same bits.
      if (l->single_role) ACME_P3G_GEMM("fc_dgrad", 128, 128, 2, 2, 32, 3, p, 1);  // tests
      else ACME_P3WS_GEMM("fc_dgrad", 128, 128, 2, 2, 32, p, 1, true);
    }
    if (fork && join_dense) ACME_HIP_TRY(hipStreamWaitEvent(st_main, l->ev[3], 0));
    l->dense_on_side = fork;
    return ACME_OK;
  }
  {  // FC weight + bias grad: [7744, 1024] = x3^T dZh (reduction over the batch).
    DenseWgrad<true> p;
    p.M = kFlat; p.N = 2 * kHidden; p.K = B; p.k_chunk = B;
    p.x = l->x3; p.ldx = kFlat; p.dz = l->dzh; p.out = Pm(l, gr, l->t_fcw);
    p.bias_out = Pm(l, gr, l->t_fcb);
    ACME_GEMM_N("fc_wgrad", 128, 128, 2, 2, p, 1);
  }
  {  // FC input grad -> dZ3 (masked by conv3's ReLU).
    DenseDgrad<true> p;
    p.M = B; p.N = kFlat; p.K = 2 * kHidden; p.k_chunk = p.K;
    p.dz = l->dzh; p.w = P(l, prm, l->t_fcw); p.xprev = l->x3; p.ldx = kFlat; p.dx = l->dz3;
    ACME_GEMM_NK("fc_dgrad", 64, 128, 2, 2, 16, p, 1);
  }
  return ACME_OK;  // the torso backward is stage 1 (acme_dqn_forward_backward_stage)
}

template <class In>
int mlp_wgrad(acme_dqn* l, const Layer& L, const void* x, const float* dz, int B, float* dw,
              float* db, hipStream_t st) {
  if (L.in % 4 == 0 && L.out % 4 == 0) {
    DenseWgrad<true, In> p;
    p.M = L.in; p.N = L.out; p.K = B; p.k_chunk = B;
    p.x = static_cast<const typename In::T*>(x); p.ldx = L.in; p.dz = dz; p.out = dw;
    p.bias_out = db;
    ACME_GEMM_N("mlp_wgrad", 64, 64, 2, 2, p, 1);
  } else {
    DenseWgrad<false, In> p;
    p.M = L.in; p.N = L.out; p.K = B; p.k_chunk = B;
    p.x = static_cast<const typename In::T*>(x); p.ldx = L.in; p.dz = dz; p.out = dw;
    p.bias_out = db;
    ACME_GEMM_N("mlp_wgrad", 64, 64, 2, 2, p, 1);
  }
  return ACME_OK;
}

int mlp_backward(acme_dqn* l, const void* o_tm1, int B, hipStream_t st) {
  const int nl = (int)l->layers.size();
  const float* prm = l->params;
  float* gr = l->grads;
  // dZ of the linear head: g_b at a_b.
  int rc = launch_onehot_dq(l->g, l->a_cache, B, l->cfg.num_actions, l->mlp_dz[nl - 1], st);
  if (rc != ACME_OK) return rc;
  for (int i = nl - 1; i >= 0; --i) {
    const Layer& L = l->layers[i];
    const float* dz = l->mlp_dz[i];
    if (i == 0) {
      rc = l->cfg.obs_dtype == ACME_OBS_U8_SCALED
               ? mlp_wgrad<InU8>(l, L, o_tm1, dz, B, Pm(l, gr, L.w), Pm(l, gr, L.b), st)
               : mlp_wgrad<InF32>(l, L, o_tm1, dz, B, Pm(l, gr, L.w), Pm(l, gr, L.b), st);
    } else {
      rc = mlp_wgrad<InF32>(l, L, l->mlp_act[i - 1], dz, B, Pm(l, gr, L.w), Pm(l, gr, L.b), st);
    }
    if (rc != ACME_OK) return rc;
    if (i > 0) {
      if (L.in % 4 == 0 && L.out % 4 == 0) {
        DenseDgrad<true> p;
        p.M = B; p.N = L.in; p.K = L.out; p.k_chunk = L.out;
        p.dz = dz; p.w = P(l, prm, L.w); p.xprev = l->mlp_act[i - 1]; p.ldx = L.in;
        p.dx = l->mlp_dz[i - 1];
        ACME_GEMM_N("mlp_dgrad", 64, 64, 2, 2, p, 1);
      } else {
        DenseDgrad<false> p;
        p.M = B; p.N = L.in; p.K = L.out; p.k_chunk = L.out;
        p.dz = dz; p.w = P(l, prm, L.w); p.xprev = l->mlp_act[i - 1]; p.ldx = L.in;
        p.dx = l->mlp_dz[i - 1];
        ACME_GEMM_N("mlp_dgrad", 64, 64, 2, 2, p, 1);
      }
    }
  }
  return ACME_OK;
}

// Refreshes the parameter planes from the f32 parameter buffers, each at a scale that suits
// its max (the current one when it does: after acme_dqn_set_scale_state the planes are the
// bits the checkpointed run's Adam wrote).
int sync_planes(acme_dqn* l, hipStream_t st) {
  if (!l->p3_capable || !l->planes_stale) return ACME_OK;
  int rc = launch_split_planes(l->params, l->flat, l->wpl, l->flat, l->scales + kScParams, st,
                               l->overflow, 1);
  if (rc == ACME_OK)
    rc = launch_split_planes(l->target, l->flat, l->tpl, l->flat, l->scales + kScTarget, st,
                             l->overflow, 1);
  if (rc == ACME_OK) l->planes_stale = false;
  return rc;
}

// Initial scale records: w = r = wi = 1, amax slots 0; each record's flag is the guard word
// of the tensors it covers (the online step's, the target forward's, the parameters').
int reset_scales(acme_dqn* l) {
  std::vector<gemm::PScale> init(kScCount);
  std::memset(init.data(), 0, init.size() * sizeof(gemm::PScale));
  for (auto& r : init) r.w = r.r = r.wi = r.rl = 1.f;
  for (int i = 0; i < kScCount; ++i)
    init[i].flag = i >= kScT1 && i <= kScT3 ? &l->guard->tt
                   : i >= kScTransient     ? &l->guard->prm
                                           : &l->guard->on;
  ACME_HIP_TRY(hipMemcpy(l->scales, init.data(), init.size() * sizeof(gemm::PScale),
                         hipMemcpyHostToDevice));
  ACME_HIP_TRY(hipMemset(l->overflow, 0, sizeof(int)));
  return ACME_OK;
}

}  // namespace

extern "C" {

int acme_dqn_create(const acme_dqn_config* cfg, acme_dqn** out) {
  ACME_CHECK_ARG(cfg && out, "null argument");
  ACME_CHECK_ARG(cfg->num_actions >= 1 && cfg->num_actions <= 63, "num_actions must be in [1, 63]");
  ACME_CHECK_ARG(cfg->max_batch >= 1 && cfg->max_batch <= 65536, "max_batch must be in [1, 65536]");
  ACME_CHECK_ARG(cfg->network == ACME_NET_NATURE_DQN || cfg->network == ACME_NET_MLP,
                 "unknown network kind %d", cfg->network);
  ACME_CHECK_ARG(cfg->obs_dtype == ACME_OBS_U8_SCALED || cfg->obs_dtype == ACME_OBS_F32,
                 "unknown observation dtype %d", cfg->obs_dtype);
  ACME_CHECK_ARG(cfg->huber_loss_parameter >= 0.f, "quadratic_linear_boundary must be >= 0.");
  ACME_CHECK_ARG(cfg->target_update_period >= 1, "target_update_period must be >= 1");
  ACME_CHECK_ARG(cfg->semantics == ACME_SEMANTICS_TF || cfg->semantics == ACME_SEMANTICS_JAX,
                 "unknown learner semantics %d", cfg->semantics);
  acme_dqn* l = new acme_dqn();
  l->cfg = *cfg;
  l->single_stream = tune_variant("SIDE") == 1;
  l->single_role = tune_variant("WSN") == 1;
  l->stamps_on = tune_variant("STAMPS") == 1;
  const int A = cfg->num_actions;
  const int B = cfg->max_batch;
  int rc = ACME_OK;
  auto fail = [&](int code) {
    acme_dqn_destroy(l);
    return code;
  };
  if ((rc = dev_alloc(l, &l->guard, 1)) != ACME_OK) return fail(rc);
  if (hipMemset(l->guard, 0, sizeof(StepGuard)) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&l->host_skipped), sizeof(int64_t),
                    hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&l->host_verdicts), kVerdictRing * sizeof(uint32_t),
                    hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
    return fail((set_error("step guard allocation failed"), ACME_ERR_HIP));
  *l->host_skipped = 0;
  for (int i = 0; i < kVerdictRing; ++i) l->host_verdicts[i] = 0xFFFFFFFFu;  // none decided
  if (cfg->network == ACME_NET_NATURE_DQN) {
    l->t_c1w = add_tensor(l, "atari_torso/conv2_d/w", {8, 8, 4, 32});
    l->t_c1b = add_tensor(l, "atari_torso/conv2_d/b", {32});
    l->t_c2w = add_tensor(l, "atari_torso/conv2_d_1/w", {4, 4, 32, 64});
    l->t_c2b = add_tensor(l, "atari_torso/conv2_d_1/b", {64});
    l->t_c3w = add_tensor(l, "atari_torso/conv2_d_2/w", {3, 3, 64, 64});
    l->t_c3b = add_tensor(l, "atari_torso/conv2_d_2/b", {64});
    // Fused [value_mlp/linear_0 | advantage_mlp/linear_0].
    l->t_fcw = add_tensor(l, "duelling_q_network/hidden/w", {kFlat, 2 * kHidden});
    l->t_fcb = add_tensor(l, "duelling_q_network/hidden/b", {2 * kHidden});
    l->t_vw = add_tensor(l, "duelling_q_network/mlp/linear_1/w", {kHidden, 1});
    l->t_vb = add_tensor(l, "duelling_q_network/mlp/linear_1/b", {1});
    l->t_aw = add_tensor(l, "duelling_q_network/mlp_1/linear_1/w", {kHidden, A});
    l->t_ab = add_tensor(l, "duelling_q_network/mlp_1/linear_1/b", {A});
    const int R2 = 2 * B;
    if ((rc = dev_alloc(l, &l->x1, (int64_t)R2 * G1::OPIX * G1::CO)) ||
        (rc = dev_alloc(l, &l->x2, (int64_t)R2 * kFlat)) ||
        (rc = dev_alloc(l, &l->x3, (int64_t)R2 * kFlat)) ||
        (rc = dev_alloc(l, &l->hid, (int64_t)R2 * 2 * kHidden)) ||
        (rc = dev_alloc(l, &l->t1, (int64_t)B * G1::OPIX * G1::CO)) ||
        (rc = dev_alloc(l, &l->t2, (int64_t)B * kFlat)) ||
        (rc = dev_alloc(l, &l->t3, (int64_t)B * kFlat)) ||
        (rc = dev_alloc(l, &l->thid, (int64_t)B * 2 * kHidden)) ||
        (rc = dev_alloc(l, &l->dzh, (int64_t)B * 2 * kHidden)) ||
        (rc = dev_alloc(l, &l->dz3, (int64_t)B * kFlat)) ||
        (rc = dev_alloc(l, &l->dz2, (int64_t)B * kFlat)) ||
        (rc = dev_alloc(l, &l->dz1, (int64_t)B * G1::OPIX * G1::CO)))
      return fail(rc);
    l->slab_floats = slab_floats_needed(B, A);
    // The plane kernels address each operand plane through a buffer descriptor with a
    // 31-bit byte range: the bf16 frame copy of [o_tm1; o_t] (2B x 56,448 B) bounds the batch
    // (B <= 19,000); larger batches run the f32 / x6 engines.
    if (cfg->obs_dtype == ACME_OBS_U8_SCALED && (int64_t)R2 * kObsBytes * 2 < (int64_t)INT32_MAX) {
      l->p3_capable = true;
      const int64_t fl = l->flat;
      if ((rc = dev_alloc(l, &l->scales, kScCount)) || (rc = dev_alloc(l, &l->overflow, 1)) ||
          (rc = reset_scales(l)) ||
          (rc = dev_alloc(l, &l->wpl, gemm::kPlanes * fl)) ||
          (rc = dev_alloc(l, &l->tpl, gemm::kPlanes * fl)) ||
          (rc = dev_alloc(l, &l->frames, (int64_t)R2 * kObsBytes)) ||
          (rc = plane_alloc(l, &l->x1p, (int64_t)R2 * torso::kX1, kScX1)) ||
          (rc = plane_alloc(l, &l->x2p, (int64_t)R2 * kFlat, kScX2)) ||
          (rc = plane_alloc(l, &l->x3p, (int64_t)R2 * kFlat, kScX3)) ||
          (rc = plane_alloc(l, &l->t1p, (int64_t)B * torso::kX1, kScT1)) ||
          (rc = plane_alloc(l, &l->t2p, (int64_t)B * kFlat, kScT2)) ||
          (rc = plane_alloc(l, &l->t3p, (int64_t)B * kFlat, kScT3)) ||
          (rc = plane_alloc(l, &l->dzhp, (int64_t)B * 2 * kHidden, kScDzh)) ||
          (rc = dev_alloc(l, &l->loss_part,
                          std::max<int64_t>(B, dqn_loss_head_dz_blocks(B, kHidden)))) ||
          (rc = plane_alloc(l, &l->dz3p, (int64_t)B * kFlat, kScDz3)) ||
          (rc = plane_alloc(l, &l->dz2p, (int64_t)B * kFlat, kScDz2)) ||
          (rc = plane_alloc(l, &l->dz1p, (int64_t)B * torso::kX1, kScDz1)))
        return fail(rc);
      l->slab_floats = std::max(l->slab_floats, torso::wgrad_slab_floats_p3());
      // ACME_V_SIDE=1 at creation: a single stream (tests of the schedule).
      if (!l->single_stream) {
        // The second stream at the default priority.  At the lowest priority (rounds 2-3:
        // 0.5308 -> 0.5260 ms per step then, so the dispatcher favoured the main stream's
        // critical path) the step time depended on the order the process created its
        // streams: two streams created before the learner's first step (a table's insert
        // path) left every main-stream kernel about 2x longer, 0.51 -> 1.10 ms per step
        // (profiles/r04/tools/insert_diag5.py); at the default priority 0.51 ms either way, and the same
        // step time as the lowest priority otherwise (profiles/r04/tools/ab_sprio.sh, round 4).
        hipError_t e = hipStreamCreateWithFlags(&l->side, hipStreamNonBlocking);
        for (auto& ev : l->ev)
          if (e == hipSuccess) e = make_order_event(&ev);
        if (e != hipSuccess)
          return fail((set_error("side stream: %s", hipGetErrorString(e)), ACME_ERR_HIP));
      }
      // The side stream's slab, and conv2's for the fused step's deferred reductions (also
      // with one stream: ACME_V_SIDE=1 profiles the same kernels).
      if ((rc = dev_alloc(l, &l->side_slab, l->slab_floats)) ||
          (rc = dev_alloc(l, &l->tslab, l->slab_floats)) ||
          (rc = dev_alloc(l, &l->slab2, torso::wgrad_slab_floats_p3())))
        return fail(rc);
    }
  } else {
    ACME_CHECK_ARG(cfg->obs_dim >= 1, "obs_dim must be >= 1");
    ACME_CHECK_ARG(cfg->num_hidden >= 0 && cfg->num_hidden <= ACME_MAX_MLP_LAYERS,
                   "num_hidden must be in [0, %d]", ACME_MAX_MLP_LAYERS);
    int in = cfg->obs_dim;
    char name[64];
    for (int i = 0; i <= cfg->num_hidden; ++i) {
      Layer L;
      L.in = in;
      L.out = i < cfg->num_hidden ? cfg->hidden[i] : A;
      L.relu = i < cfg->num_hidden;
      if (L.out < 1) return fail((set_error("hidden sizes must be >= 1"), ACME_ERR_INVALID));
      snprintf(name, sizeof(name), "mlp/linear_%d/w", i);
      L.w = add_tensor(l, name, {L.in, L.out});
      snprintf(name, sizeof(name), "mlp/linear_%d/b", i);
      L.b = add_tensor(l, name, {L.out});
      l->layers.push_back(L);
      in = L.out;
    }
    for (size_t i = 0; i < l->layers.size(); ++i) {
      float *a = nullptr, *ta = nullptr, *dz = nullptr;
      const int w = l->layers[i].out;
      if ((rc = dev_alloc(l, &a, (int64_t)2 * B * w)) || (rc = dev_alloc(l, &ta, (int64_t)B * w)) ||
          (rc = dev_alloc(l, &dz, (int64_t)B * w)))
        return fail(rc);
      l->mlp_act.push_back(a);
      l->mlp_tact.push_back(ta);
      l->mlp_dz.push_back(dz);
    }
    l->slab_floats = 1;
  }
  if (make_order_event(&l->ev_dense) != hipSuccess)
    return fail((set_error("event creation failed"), ACME_ERR_HIP));
  if ((rc = dev_alloc(l, &l->q_on, (int64_t)2 * B * A)) ||
      (rc = dev_alloc(l, &l->q_tg, (int64_t)B * A)) ||
      (rc = dev_alloc(l, &l->slab, l->slab_floats)) ||
      (rc = dev_alloc(l, &l->g, (int64_t)B)) || (rc = dev_alloc(l, &l->a_cache, (int64_t)B)) ||
      (rc = dev_alloc(l, &l->loss_tmp, 4)) || (rc = dev_alloc(l, &l->td_tmp, (int64_t)B)) ||
      (rc = dev_alloc(l, &l->prio_tmp, (int64_t)B)) ||
      (l->stamps_on && (rc = dev_alloc(l, &l->stamps, (int64_t)5 * 4096 * 8))))
    return fail(rc);
  if (l->stamps_on) {  // [fc_fwd, conv1, conv2, conv3, update][4096][8] (one learner at a time)
    for (int i = 0; i < 3; ++i) torso::g_stamps_conv[i] = l->stamps + (int64_t)(i + 1) * 4096 * 8;
    g_update_stamps = l->stamps + (int64_t)4 * 4096 * 8;
  }
  if (hipDeviceSynchronize() != hipSuccess)
    return fail((set_error("learner init failed"), ACME_ERR_HIP));
  *out = l;
  return ACME_OK;
}

int acme_dqn_destroy(acme_dqn* l) {
  if (!l) return ACME_OK;
  (void)hipDeviceSynchronize();
  if (l->stamps_on) {
    for (auto& p : torso::g_stamps_conv) p = nullptr;
    g_update_stamps = nullptr;
  }
  for (void* p : l->allocs) (void)hipFree(p);
  for (auto& e : l->ev)
    if (e) (void)hipEventDestroy(e);
  if (l->side) (void)hipStreamDestroy(l->side);
  if (l->ev_dense) (void)hipEventDestroy(l->ev_dense);
  for (auto& e : l->dp_ev)
    if (e) (void)hipEventDestroy(e);
  if (l->dp_stream) (void)hipStreamDestroy(l->dp_stream);
  if (l->host_skipped) (void)hipHostFree(l->host_skipped);
  if (l->host_verdicts) (void)hipHostFree(l->host_verdicts);
  delete l;
  return ACME_OK;
}

int64_t acme_dqn_num_params(const acme_dqn* l) { return l ? l->logical : 0; }
int64_t acme_dqn_flat_size(const acme_dqn* l) { return l ? l->flat : 0; }
int32_t acme_dqn_num_tensors(const acme_dqn* l) { return l ? (int32_t)l->tensors.size() : 0; }

int acme_dqn_tensor_info(const acme_dqn* l, int32_t i, int64_t* offset, int64_t* numel,
                         int32_t* ndim, int64_t* shape4, const char** name) {
  ACME_CHECK_ARG(l && i >= 0 && i < (int32_t)l->tensors.size(), "tensor index out of range");
  const Tensor& t = l->tensors[i];
  if (offset) *offset = t.offset;
  if (numel) *numel = t.numel;
  if (ndim) *ndim = t.ndim;
  if (shape4)
    for (int k = 0; k < 4; ++k) shape4[k] = t.shape[k];
  if (name) *name = t.name.c_str();
  return ACME_OK;
}

int acme_dqn_bind(acme_dqn* l, float* params, float* target, float* grads, float* adam_m,
                  float* adam_v) {
  ACME_CHECK_ARG(l && params && target && grads && adam_m && adam_v, "null buffer");
  for (const float* p : {params, target, grads, adam_m, adam_v})
    ACME_CHECK_ARG(reinterpret_cast<uintptr_t>(p) % 16 == 0, "buffers must be 16-byte aligned");
  l->params = params;
  l->target = target;
  l->grads = grads;
  l->m = adam_m;
  l->v = adam_v;
  l->planes_stale = true;
  l->scales_ok = false;
  return ACME_OK;
}

int acme_dqn_params_changed(acme_dqn* l) {
  ACME_CHECK_ARG(l, "null learner");
  l->planes_stale = true;
  l->scales_ok = false;  // new parameters: recalibrate (unless a scale state is restored)
  l->target_dirty = true;
  return ACME_OK;
}

// Scale state = (w, r, wi, rl) of every record, host floats.
int acme_dqn_scale_state(const acme_dqn* l, float* out, int32_t capacity, int32_t* count) {
  ACME_CHECK_ARG(l && count, "null argument");
  *count = l->scales ? 4 * kScCount : 0;
  if (!l->scales || !out) return ACME_OK;
  ACME_CHECK_ARG(capacity >= 4 * kScCount, "scale state needs %d floats", 4 * kScCount);
  ACME_HIP_TRY(hipDeviceSynchronize());
  for (int i = 0; i < kScCount; ++i)
    ACME_HIP_TRY(hipMemcpy(out + 4 * i, l->scales + i, 4 * sizeof(float), hipMemcpyDeviceToHost));
  return ACME_OK;
}

int acme_dqn_set_scale_state(acme_dqn* l, const float* in, int32_t count) {
  ACME_CHECK_ARG(l && in, "null argument");
  ACME_CHECK_ARG(l->scales && count == 4 * kScCount, "scale state of %d floats expected, got %d",
                 l->scales ? 4 * kScCount : 0, count);
  for (int i = 0; i < 4 * kScCount; ++i) {
    int e;
    const float m = std::frexp(in[i], &e);
    ACME_CHECK_ARG(m == 0.5f, "scale state entries must be powers of two");
  }
  ACME_HIP_TRY(hipDeviceSynchronize());
  for (int i = 0; i < kScCount; ++i)
    ACME_HIP_TRY(hipMemcpy(l->scales + i, in + 4 * i, 4 * sizeof(float), hipMemcpyHostToDevice));
  l->scales_ok = true;
  l->target_dirty = true;
  return ACME_OK;
}

int acme_dqn_plane_overflow(acme_dqn* l, int32_t* overflow, int32_t reset) {
  ACME_CHECK_ARG(l && overflow, "null argument");
  *overflow = 0;
  if (!l->overflow) return ACME_OK;
  ACME_HIP_TRY(hipDeviceSynchronize());
  int v = 0;
  ACME_HIP_TRY(hipMemcpy(&v, l->overflow, sizeof(int), hipMemcpyDeviceToHost));
  *overflow = v != 0;
  if (reset) ACME_HIP_TRY(hipMemset(l->overflow, 0, sizeof(int)));
  return ACME_OK;
}

int64_t acme_dqn_skipped_steps(const acme_dqn* l) {
  if (!l || !l->host_skipped) return 0;
  return *reinterpret_cast<volatile const int64_t*>(l->host_skipped);
}

int acme_dqn_guard_state(acme_dqn* l, int64_t* out4) {
  ACME_CHECK_ARG(l && out4 && l->guard, "null argument");
  ACME_HIP_TRY(hipDeviceSynchronize());
  StepGuard g;
  ACME_HIP_TRY(hipMemcpy(&g, l->guard, sizeof(g), hipMemcpyDeviceToHost));
  out4[0] = g.applied;
  out4[1] = g.skipped;
  out4[2] = g.last;
  out4[3] = g.qv;
  return ACME_OK;
}

int acme_dqn_verdict_timeouts(acme_dqn* l, int64_t* out) {
  ACME_CHECK_ARG(l && out, "null argument");
  *out = 0;
  if (!l->guard) return ACME_OK;
  ACME_HIP_TRY(hipDeviceSynchronize());
  StepGuard g;
  ACME_HIP_TRY(hipMemcpy(&g, l->guard, sizeof(g), hipMemcpyDeviceToHost));
  *out = g.vtimeout;
  return ACME_OK;
}

int acme_dqn_set_reissue(acme_dqn* l, int32_t enable) {
  ACME_CHECK_ARG(l, "null learner");
  l->sticky = enable != 0 && l->p3_capable;
  return ACME_OK;
}

int64_t acme_dqn_verdicts_issued(const acme_dqn* l) { return l ? (int64_t)l->verdict_seq : 0; }

int acme_dqn_step_verdict(const acme_dqn* l, int64_t seq, int32_t* state) {
  ACME_CHECK_ARG(l && state && seq >= 0, "bad argument");
  *state = -1;
  if (!l->host_verdicts || seq >= (int64_t)l->verdict_seq) return ACME_OK;  // not issued
  ACME_CHECK_ARG(seq + kVerdictRing >= (int64_t)l->verdict_seq,
                 "verdict %lld is older than the ring's %d", (long long)seq, kVerdictRing);
  const uint32_t v =
      __atomic_load_n(l->host_verdicts + (seq & (kVerdictRing - 1)), __ATOMIC_ACQUIRE);
  if ((v >> 1) == ((uint32_t)seq & 0x7fffffffu)) *state = (int32_t)(v & 1u);
  return ACME_OK;
}

int acme_dqn_set_applied_steps(acme_dqn* l, int64_t n) {
  ACME_CHECK_ARG(l && l->guard && n >= 0, "bad argument");
  ACME_HIP_TRY(hipDeviceSynchronize());
  ACME_HIP_TRY(hipMemcpy(&l->guard->applied, &n, sizeof(n), hipMemcpyHostToDevice));
  return ACME_OK;
}

int acme_dqn_skip_word(const acme_dqn* l, const uint32_t** out) {
  ACME_CHECK_ARG(l && out, "null argument");
  *out = l->p3_capable ? &l->guard->last : nullptr;
  return ACME_OK;
}

int acme_dqn_set_data_parallel_gate(acme_dqn* l, int32_t enable) {
  ACME_CHECK_ARG(l, "null learner");
  if (enable && l->cfg.network == ACME_NET_NATURE_DQN && l->p3_capable) {
    // conv1's bias (32 values) is padded to 64 floats: the first padding word of the torso
    // bucket [0, grad_split) carries the gate (zero on every step that is applied, so its
    // Adam update stays zero).
    const Tensor& t = l->tensors[l->t_c1b];
    ACME_CHECK_ARG(align64(t.offset + t.numel) > t.offset + t.numel, "no padding word for the gate");
    l->dp_gate_index = t.offset + t.numel;
    l->dp_gate = true;
  } else {
    l->dp_gate = false;
  }
  return ACME_OK;
}

int64_t acme_dqn_num_steps(const acme_dqn* l) { return l ? l->num_steps : 0; }
int acme_dqn_set_num_steps(acme_dqn* l, int64_t n) {
  ACME_CHECK_ARG(l && n >= 0, "bad argument");
  l->num_steps = n;
  return ACME_OK;
}

int acme_dqn_debug_buffer(const acme_dqn* l, const char* name, const float** out,
                          int64_t* count) {
  ACME_CHECK_ARG(l && name && out && count, "null argument");
  const int64_t B = l->cfg.max_batch;
  struct {
    const char* n;
    const float* p;
    int64_t c;
  } tab[] = {{"gemm_stamps", reinterpret_cast<const float*>(l->stamps), 2 * 5 * 4096 * 8},
             {"x1", l->x1, 2 * B * 441 * 32}, {"x2", l->x2, 2 * B * kFlat},
             {"x3", l->x3, 2 * B * kFlat},    {"hid", l->hid, 2 * B * 2 * kHidden},
             {"dzh", l->dzh, B * 2 * kHidden}, {"dz3", l->dz3, B * kFlat},
             {"dz2", l->dz2, B * kFlat},       {"dz1", l->dz1, B * 441 * 32},
             {"q_on", l->q_on, 2 * B * l->cfg.num_actions},
             {"q_tg", l->q_tg, B * l->cfg.num_actions}, {"g", l->g, B}};
  for (auto& e : tab)
    if (e.p && std::strcmp(e.n, name) == 0) {
      if (l->last_p3) {  // the plane path keeps these tensors as planes: join into f32
        struct {
          const char* n;
          torso::Plane pl;
        } ptab[] = {{"x1", l->x1p},   {"x2", l->x2p},   {"x3", l->x3p},  {"dzh", l->dzhp},
                    {"dz3", l->dz3p}, {"dz2", l->dz2p}, {"dz1", l->dz1p}};
        for (auto& q : ptab)
          if (std::strcmp(q.n, name) == 0) {
            int rc = launch_join_planes(q.pl.p, q.pl.stride, e.c, const_cast<float*>(e.p),
                                        q.pl.sc, 0);
            if (rc != ACME_OK) return rc;
            ACME_HIP_TRY(hipDeviceSynchronize());
          }
      }
      *out = e.p;
      *count = e.c;
      return ACME_OK;
    }
  for (size_t i = 0; i < l->mlp_act.size(); ++i) {  // MLP layer outputs "act<i>" (2B rows)
    char nm[16];
    snprintf(nm, sizeof(nm), "act%zu", i);
    if (std::strcmp(nm, name) == 0) {
      *out = l->mlp_act[i];
      *count = 2 * B * l->layers[i].out;
      return ACME_OK;
    }
  }
  set_error("unknown debug buffer '%s'", name);
  return ACME_ERR_INVALID;
}

int acme_dqn_q_values(acme_dqn* l, const void* obs, int64_t batch, int32_t use_target,
                      float* q_out, void* stream) {
  ACME_CHECK_ARG(l && obs && q_out && l->params, "null argument or unbound learner");
  ACME_CHECK_ARG(batch >= 1 && batch <= l->cfg.max_batch, "batch must be in [1, max_batch]");
  hipStream_t st = as_stream(stream);
  const float* prm = use_target ? l->target : l->params;
  const int B = (int)batch;
  if (l->cfg.network == ACME_NET_NATURE_DQN && use_p3(l)) {
    l->target_dirty = true;  // the target activations and their records, on this stream
    int rc = sync_planes(l, st);
    if (rc == ACME_OK) rc = convert_frames(l, obs, obs, B, B, st);
    // Uncalibrated scales: one forward to measure the activations, then the real one.
    // Each pass ends with the target records' rescale; the last one's flag lands in the
    // guard's qv word (acme_dqn_guard_state), so a caller can repeat an overflowed call.
    for (int pass = l->scales_ok ? 1 : 0; pass < 2 && rc == ACME_OK; ++pass) {
      rc = nature_forward_p3(l, prm, use_target ? l->tpl : l->wpl, torso::Frames{l->frames}, B,
                             l->t1p, l->t2p, l->t3p, l->thid, q_out, st);
      RescaleGuard rg;
      rg.g = l->guard;
      rg.mode = kRgQValues;
      if (rc == ACME_OK)
        rc = launch_plane_rescale(l->scales + kScT1, 3, 3, -1, -1, l->overflow, st, -1, -1, rg);
    }
    return rc;
  }
  if (l->cfg.network == ACME_NET_NATURE_DQN)
    return nature_forward(l, prm, obs, obs, B, B, l->t1, l->t2, l->t3, l->thid, q_out, st);
  return mlp_forward(l, prm, obs, obs, B, B, l->mlp_tact, q_out, st);
}

static int forward_backward_stage(acme_dqn* l, const acme_transition_batch* batch,
                                  const acme_dqn_outputs* out, int32_t stage, void* stream,
                                  bool join_dense);

int acme_dqn_forward_backward_stage(acme_dqn* l, const acme_transition_batch* batch,
                                    const acme_dqn_outputs* out, int32_t stage, void* stream) {
  return forward_backward_stage(l, batch, out, stage, stream, true);
}

static int loss_and_dense_backward(acme_dqn* l, const acme_transition_batch* batch,
                                   const acme_dqn_outputs* out, hipStream_t st, bool join_dense);

// Activation / gradient scales for new parameters (gemm_p3.h): kCalibrationPasses passes of
// the step's forward, loss and backward on this batch (local IS normaliser, outputs to
// scratch; no Adam, no target copy), each followed by a rescale of the transient records.
// A pass measures each tensor's maximum before its split, so it is accurate even where the
// planes are written at a poor scale; but a tensor computed from planes that underflowed to
// zero at their scale measures 0 and keeps its scale, and only the next pass, reading its
// input at a calibrated scale, measures it.  The input-gradient chain (head dZ -> dz3 ->
// dz2 -> dz1) is four tensors deep, so four passes calibrate every record whatever the
// gradients' magnitude (two left dz2 / dz1 at scale 1 when |TD| was ~1e-4: their planes
// read as zeros, tests/test_step_guard_gpu.py).  Writes nothing the real step does not
// overwrite.
constexpr int kCalibrationPasses = 4;
static int calibrate_scales(acme_dqn* l, const acme_transition_batch* batch, hipStream_t st) {
  acme_transition_batch cb = *batch;
  cb.global_min_probability = nullptr;
  l->calibrating = true;
  int rc = ACME_OK;
  for (int pass = 0; pass < kCalibrationPasses && rc == ACME_OK; ++pass) {
    rc = forward_backward_stage(l, &cb, nullptr, 2, st, false);
    if (rc == ACME_OK) rc = forward_backward_stage(l, &cb, nullptr, 3, st, false);
    if (rc == ACME_OK) rc = forward_backward_stage(l, &cb, nullptr, 1, st, false);
    if (rc == ACME_OK)
      rc = launch_plane_rescale(l->scales, kScTransient, kScTransient, -1, -1, l->overflow, st);
  }
  l->calibrating = false;
  if (rc != ACME_OK) return rc;
  // Overflows at the initial scales are expected and corrected by the passes.
  ACME_HIP_TRY(hipMemsetAsync(l->overflow, 0, sizeof(int), st));
  if ((rc = clear_guard_flags(l, st)) != ACME_OK) return rc;
  l->scales_ok = true;
  return ACME_OK;
}

static int forward_backward_stage(acme_dqn* l, const acme_transition_batch* batch,
                                  const acme_dqn_outputs* out, int32_t stage, void* stream,
                                  bool join_dense) {
  ACME_CHECK_ARG(l && batch && l->params, "null argument or unbound learner");
  ACME_CHECK_ARG(stage >= 0 && stage <= 4, "stage must be 0, 1, 2, 3 or 4");
  ACME_CHECK_ARG(batch->o_tm1 && batch->a_tm1 && batch->r_t && batch->d_t && batch->o_t &&
                     batch->probabilities,
                 "transition batch has null fields");
  ACME_CHECK_ARG(batch->batch >= 1 && batch->batch <= l->cfg.max_batch,
                 "batch %lld outside [1, max_batch=%d]", (long long)batch->batch, l->cfg.max_batch);
  hipStream_t st = as_stream(stream);
  const int B = (int)batch->batch;
  const bool nature = l->cfg.network == ACME_NET_NATURE_DQN;
  if (stage == 1) {
    // Torso weight gradients (the flat buffer's head, [0, grad_split)).  Every gradient
    // element is written by its kernel (no accumulation), so nothing is cleared.
    if (!nature) return ACME_OK;
    if (use_p3(l)) {
      torso::Grads g{Pm(l, l->grads, l->t_c1w), Pm(l, l->grads, l->t_c1b),
                     Pm(l, l->grads, l->t_c2w), Pm(l, l->grads, l->t_c2b),
                     Pm(l, l->grads, l->t_c3w), Pm(l, l->grads, l->t_c3b)};
      torso::PWeights w{WP(l, l->wpl, l->t_c1w), WP(l, l->wpl, l->t_c2w),
                        WP(l, l->wpl, l->t_c3w), P(l, l->params, l->t_c1b),
                        P(l, l->params, l->t_c2b), P(l, l->params, l->t_c3b)};
      torso::Side sd;
      sd.single_role = l->single_role;
      // conv1's weight gradient on the single-role kernel: its two 20-KB stages (40 KB of
      // LDS) fit beside the next step's fused target convolution (121 KB) that runs on the
      // side stream at the same time; the producer / consumer kernel's three stages (60 KB)
      // do not.  Step 0.4957 -> 0.4920 ms (three alternating 300-step pairs, round 6,
      // profiles/r06/schedule/ab_conv1_wgrad_single_role.log).
      sd.conv1_single = true;
      if (side_stream(l)) {
        sd.side = l->side;
        sd.slab = l->side_slab;
        for (int i = 0; i < 3; ++i) sd.e[i] = l->ev[i];
      }
      l->slabs_pending = false;
      if (l->upd_replay && l->upd_prio && !l->calibrating) {
        sd.tail = priority_update_tail;
        sd.tail_ctx = l;
      }
      if (l->fused_step && !l->calibrating && l->slab2) {
        sd.slab = l->side_slab;
        sd.slab2 = l->slab2;
        sd.defer = l->wslabs;
        l->slabs_pending = true;
      }
      int rc = torso::backward_p3(w, g, l->cur_frames, B,
                                  torso::PActs{l->x1p, l->x2p, l->x3p}, l->dz3p, l->dz2p, l->dz1p,
                                  l->slab, st, sd);
      // Data parallelism: this rank's skip decision into the torso bucket's padding word,
      // which the ranks' all-reduce combines before Adam reads it (step_gate).
      if (rc == ACME_OK && l->dp_gate && !l->calibrating) {
        Gate local = step_gate(l);
        local.dp = nullptr;
        rc = launch_gate_publish(local, l->grads + l->dp_gate_index, st, l->scales,
                                 kScTransient, kScT1, kScT3 + 1);
      }
      return rc;
    }
    torso::Grads g{Pm(l, l->grads, l->t_c1w), Pm(l, l->grads, l->t_c1b), Pm(l, l->grads, l->t_c2w),
                   Pm(l, l->grads, l->t_c2b), Pm(l, l->grads, l->t_c3w), Pm(l, l->grads, l->t_c3b)};
    return torso::backward(torso_weights(l, l->params), g,
                           l->cfg.obs_dtype == ACME_OBS_U8_SCALED, batch->o_tm1, B,
                           torso::Acts{l->x1, l->x2, l->x3}, l->dz3, l->dz2, l->dz1, l->slab, st);
  }
  const int A = l->cfg.num_actions;
  int rc;
  // Stage 0 = stage 2 (the forwards) + stage 3 (loss and the dense backward); a
  // data-parallel rank splits them to run the IS-normaliser all-reduce beside the forwards.
  if (stage == 3 || stage == 4) {
    ACME_CHECK_ARG(l->fwd_batch == (int64_t)B, "stage %d needs the stage-2 forward of this batch",
                   stage);
    l->fwd_batch = 0;
    return loss_and_dense_backward(l, batch, out, st, join_dense && stage == 3);
  }
  // Forward: online on [o_tm1; o_t] (q_tm1 rows 0..B-1, q_t_selector rows B..2B-1),
  // target on o_t (q_t_value).
  l->last_p3 = nature && use_p3(l);
  if (l->last_p3) {
    // conv1's input: the batch's uint8 frames themselves (conv1's kernels widen them exactly
    // as they stage them: half the bytes of an f16 copy, and no copy), or an f16 copy (the
    // dataset's obs_f16, else our own).
    const bool u8 = !batch->obs_f16 && l->frames_u8 &&
                    ((reinterpret_cast<uintptr_t>(batch->o_tm1) |
                      reinterpret_cast<uintptr_t>(batch->o_t)) & 15) == 0;
    // The caller's inputs event can stand for the fork only if nothing is enqueued here first.
    const bool quiet =
        !l->planes_stale && l->scales_ok && (batch->obs_f16 || u8) && !l->calibrating;
    if ((rc = sync_planes(l, st)) != ACME_OK) return rc;
    if (!l->scales_ok && !l->calibrating && (rc = calibrate_scales(l, batch, st)) != ACME_OK)
      return rc;
    l->last_p3 = true;
    hipStream_t tst = st;
    hipStream_t side = side_stream(l);
    // conv1's input: an f16 copy of [o_tm1; o_t] on the main stream for everything.  (Reading
    // the batch's uint8 frames in the kernels instead measured slower beside the side stream,
    // 0.746 -> 0.750 ms per step: the uint8 image kernel is slower there than the 16-bit one.)
    if (!batch->obs_f16 && !u8 &&
        (rc = convert_frames(l, batch->o_tm1, batch->o_t, B, 2 * B, st)) != ACME_OK)
      return rc;
    // The dataset's fused gather may hand over the f16 copy (acme_replay_sample_gather_frames).
    const torso::Frames fwd_frames =
        u8 ? torso::Frames{batch->o_tm1, true, batch->o_t, B}
           : torso::Frames{batch->obs_f16 ? static_cast<const void*>(batch->obs_f16)
                                          : static_cast<const void*>(l->frames)};
    l->cur_frames = fwd_frames;
    // Target forward (q_t_value) on the side stream, beside the online forward.
    if (side) {
      // Early start: the side stream's own order covers the previous step's target work
      // and T-record rescale; only the batch's inputs are waited for.
      if (quiet && batch->inputs_event && !l->target_dirty) {
        ACME_HIP_TRY(hipStreamWaitEvent(side, static_cast<hipEvent_t>(batch->inputs_event), 0));
      } else {
        ACME_HIP_TRY(hipEventRecord(l->ev[0], st));
        ACME_HIP_TRY(hipStreamWaitEvent(side, l->ev[0], 0));
      }
      l->target_dirty = l->calibrating;
      tst = side;
    } else {
      l->target_dirty = true;  // the target forward runs on the caller's stream
    }
    // The online forward (the critical path) is issued before the target forward, so after a
    // host wait (a timed window's first step) its kernels reach the GPU first (20-step
    // windows 0.5208 -> 0.5181 ms, three alternating runs each).  Either order gives the
    // same bits.
    const bool online_first = side != nullptr;
    l->head_deferred = false;
    if (online_first &&
        (rc = nature_forward_p3(l, l->params, l->wpl, fwd_frames, 2 * B, l->x1p, l->x2p, l->x3p,
                                l->hid, l->q_on, st, nullptr, B, true)) != ACME_OK)
      return rc;
    if ((rc = nature_forward_p3(l, l->target, l->tpl, fwd_frames.rows_from(B), B,
                                l->t1p, l->t2p, l->t3p, l->thid, l->q_tg, tst,
                                side ? l->tslab : l->slab, 0)) != ACME_OK)
      return rc;
    {  // the target records' scales, and their flag into the step's slot t[seq & 1]
      RescaleGuard rg;
      rg.g = l->guard;
      rg.mode = kRgTarget;
      rg.gate = step_gate(l);
      if ((rc = launch_plane_rescale(l->scales + kScT1, 3, 3, -1, -1, l->overflow, tst, -1, -1,
                                     rg)))
        return rc;
    }
    if (side) ACME_HIP_TRY(hipEventRecord(l->ev[1], side));
    if (!online_first &&
        (rc = nature_forward_p3(l, l->params, l->wpl, fwd_frames, 2 * B, l->x1p, l->x2p, l->x3p,
                                l->hid, l->q_on, st, nullptr, B, true)) != ACME_OK)
      return rc;
    if (side) ACME_HIP_TRY(hipStreamWaitEvent(st, l->ev[1], 0));
  } else if (nature) {
    if ((rc = nature_forward(l, l->params, batch->o_tm1, batch->o_t, B, 2 * B, l->x1, l->x2, l->x3,
                             l->hid, l->q_on, st)) != ACME_OK)
      return rc;
    if ((rc = nature_forward(l, l->target, batch->o_t, batch->o_t, B, B, l->t1, l->t2, l->t3,
                             l->thid, l->q_tg, st)) != ACME_OK)
      return rc;
  } else {
    if ((rc = mlp_forward(l, l->params, batch->o_tm1, batch->o_t, B, 2 * B, l->mlp_act, l->q_on,
                          st)) != ACME_OK)
      return rc;
    if ((rc = mlp_forward(l, l->target, batch->o_t, batch->o_t, B, B, l->mlp_tact, l->q_tg, st)) !=
        ACME_OK)
      return rc;
  }
  if (stage == 2) {
    l->fwd_batch = B;
    return ACME_OK;
  }
  return loss_and_dense_backward(l, batch, out, st, join_dense);
}

// Loss (fused into the head dZ on the plane path) and the dense layers' backward, after
// the forwards of the same batch.
static int loss_and_dense_backward(acme_dqn* l, const acme_transition_batch* batch,
                                   const acme_dqn_outputs* out, hipStream_t st, bool join_dense) {
  const int B = (int)batch->batch, A = l->cfg.num_actions;
  const bool nature = l->cfg.network == ACME_NET_NATURE_DQN;
  int rc;
  float* loss = out && out->loss ? out->loss : l->loss_tmp;
  float* td = out && out->td_error ? out->td_error : l->td_tmp;
  double* prio = out && out->priorities ? out->priorities : l->prio_tmp;
  LossArgs la;
  la.q_on = l->q_on;
  la.q_tg = l->q_tg;
  la.a = batch->a_tm1;
  la.r = batch->r_t;
  la.d = batch->d_t;
  la.probs = batch->probabilities;
  la.global_min_prob = batch->global_min_probability;
  la.B = B;
  la.A = A;
  la.mean_over = batch->mean_over > 0 ? (int)batch->mean_over : B;
  la.discount = l->cfg.discount;
  la.beta = l->cfg.importance_sampling_exponent;
  la.delta = l->cfg.huber_loss_parameter;
  la.max_abs_reward = l->cfg.max_abs_reward;
  la.jax = l->cfg.semantics == ACME_SEMANTICS_JAX;
  la.loss = loss;
  la.td = td;
  la.prio = prio;
  la.g = l->g;
  la.a_cache = l->a_cache;
  if (l->last_p3) {  // fused with the head dZ (nature_backward)
    la.loss_part = l->loss_part;
    l->pending_la = la;
    l->loss_pending = true;
  } else {
    ACME_PROF("loss", st, 0.0, 0.0);
    if ((rc = launch_dqn_loss(la, st)) != ACME_OK) return rc;
  }
  l->dense_on_side = false;
  rc = nature ? nature_backward(l, batch->o_tm1, B, st, join_dense)
              : mlp_backward(l, batch->o_tm1, B, st);
  if (rc != ACME_OK) return rc;
  // After the backward: on the plane path its first launch forms q_on (the online head).
  if (out && out->q_tm1)
    ACME_HIP_TRY(hipMemcpyAsync(out->q_tm1, l->q_on, (size_t)B * A * sizeof(float),
                                hipMemcpyDeviceToDevice, st));
  if (l->dense_on_side) {
    l->dense_ev = l->ev[3];
  } else {
    ACME_HIP_TRY(hipEventRecord(l->ev_dense, st));
    l->dense_ev = l->ev_dense;
  }
  return ACME_OK;
}

int acme_dqn_forward_backward(acme_dqn* l, const acme_transition_batch* batch,
                              const acme_dqn_outputs* out, void* stream) {
  int rc = forward_backward_stage(l, batch, out, 0, stream, false);
  if (rc != ACME_OK) return rc;
  return forward_backward_stage(l, batch, out, 1, stream, false);
}

int acme_dqn_grad_split(const acme_dqn* l, int64_t* split) {
  ACME_CHECK_ARG(l && split, "null argument");
  *split = l->cfg.network == ACME_NET_NATURE_DQN ? l->tensors[l->t_fcw].offset : 0;
  return ACME_OK;
}

// Adam (+ the parameter planes) and the periodic target copy; `copy` decided by the host.
static int apply_impl(acme_dqn* l, bool copy, hipStream_t st) {
  int rc = ACME_OK;
  Gate gate;  // Adam reads the step's skip decision, made by the step's rescale
  AdamTail tail;
  if (l->p3_capable) {
    // Every transient record's next scale from this step's maxima, and the step guard's
    // decision (guard->last): skip when a plane write overflowed, when a tensor's maximum
    // fell more than ~2^8-fold below its scale (its planes lost precision), or, with data
    // parallelism, when any rank skips.  Before Adam, after every plane this step writes
    // (the fused step's priority write-back already ran it, with deferred read scales); the
    // target forward's records were rescaled after it (on the side stream, which may
    // already run the next step's target forward).
    if (!l->step_rescaled) {
      ACME_PROF("plane_rescale", st, 0.0, 0.0);
      if ((rc = launch_rescale_job(step_rescale_job(l, false), st)) != ACME_OK) return rc;
    } else {
      tail.commit = l->scales;
      tail.ncommit = kScTransient;
      tail.skip_lo = kScT1;
      tail.skip_hi = kScT3 + 1;
    }
    l->step_rescaled = false;
    gate.g = l->guard;
    gate.use_last = 1;
    tail.clear = l->guard;
    tail.params = l->scales + kScParams;
    if (copy) tail.target = l->scales + kScTarget;
  }
  // Adam's algorithmic bytes: 28 per parameter (p, m, v read and written, g read), the
  // parameter planes it writes for the next forward (2 x 2 B), and on the fused step the conv
  // weight gradients' split-K slabs it reduces on its read (and their reduced gradients).
  const double adam_bytes = 28.0 * (double)l->logical + (l->p3_capable ? 4.0 * (double)l->flat : 0.0);
  if (l->slabs_pending) {  // the conv weight gradients reduced on Adam's read
    l->slabs_pending = false;
    double slab_bytes = 0.0;
    for (int k = 0; k < 3; ++k) {
      const double count4 = (double)((l->wslabs[k].wcount + l->wslabs[k].bcount) / 4);
      slab_bytes += 16.0 * count4 * (double)(l->wslabs[k].splits + 1);
    }
    ACME_PROF("adam", st, 0.0, adam_bytes + slab_bytes);
    const int ten[3][2] = {{l->t_c1w, l->t_c1b}, {l->t_c2w, l->t_c2b}, {l->t_c3w, l->t_c3b}};
    AdamSlabs a;
    for (int k = 0; k < 3; ++k) {
      const torso::WgradSlab& w = l->wslabs[k];
      const int64_t count4 = (w.wcount + w.bcount) / 4;
      for (int j = 0; j < 2; ++j) {
        const Tensor& t = l->tensors[ten[k][j]];
        a.seg[a.nseg++] = AdamSlabs::Seg{t.offset / 4, t.numel / 4, w.slab, w.splits, count4,
                                         j ? w.wcount / 4 : 0};
      }
    }
    a.dense_off4 = l->tensors[l->t_fcw].offset / 4;
    a.dense_n4 = (l->flat - l->tensors[l->t_fcw].offset) / 4;
    rc = launch_adam_slabs(l->params, l->grads, l->m, l->v, a, l->cfg.learning_rate,
                           l->cfg.adam_beta1, l->cfg.adam_beta2, l->cfg.adam_epsilon,
                           &l->guard->applied, l->wpl, l->flat, l->scales + kScParams,
                           l->cfg.semantics == ACME_SEMANTICS_JAX ? 1 : 0, gate, tail, st);
    if (rc != ACME_OK) return rc;
  } else {
    ACME_PROF("adam", st, 0.0, adam_bytes);
    if ((rc = adam_range(l, 0, l->flat, gate, tail, st)) != ACME_OK) return rc;
  }
  if (copy) {
    l->target_dirty = true;
    ACME_PROF("target_copy", st, 0.0, 8.0 * (double)l->logical);
    if (l->p3_capable) {  // a skipped step copies nothing (gated on its verdict, as Adam)
      if ((rc = launch_copy_gated(l->target, l->params, l->flat * sizeof(float), l->tpl, l->wpl,
                                  gemm::kPlanes * l->flat * sizeof(uint16_t), gate, st)))
        return rc;
    } else {
      ACME_HIP_TRY(hipMemcpyAsync(l->target, l->params, l->flat * sizeof(float),
                                  hipMemcpyDeviceToDevice, st));
    }
  }
  if (l->p3_capable && l->num_steps % kParamAmaxPeriod == 0) {
    // The parameter planes' write scale from their maximum every kParamAmaxPeriod steps
    // (Adam moves a parameter by about lr per step, far inside the 2^8 headroom of its
    // scale); the read scale stays that of the planes stored now (Adam's tail set it; the
    // next Adam pass writes at the new scale and moves it).
    {
      ACME_PROF("param_amax", st, 0.0, 4.0 * (double)l->flat);
      if ((rc = launch_param_amax(l->params, l->flat, l->scales + kScParams, st)) != ACME_OK)
        return rc;
    }
    ACME_PROF("param_rescale", st, 0.0, 0.0);
    rc = launch_plane_rescale(l->scales + kScParams, 0, 1, -1, -1, l->overflow, st);
  }
  return rc;
}

// TF: copy when num_steps % period == 0, then num_steps += 1 (tf/dqn/learning.py:157-161);
// JAX: steps + 1 first, copy when that is a multiple of the period (jax/dqn/learning.py:114-119).
static bool copies_target(const acme_dqn* l) {
  const int64_t at = l->cfg.semantics == ACME_SEMANTICS_JAX ? l->num_steps + 1 : l->num_steps;
  return at % l->cfg.target_update_period == 0;
}

int acme_dqn_apply(acme_dqn* l, void* stream) {
  ACME_CHECK_ARG(l && l->params, "unbound learner");
  int rc = apply_impl(l, copies_target(l), as_stream(stream));
  if (rc != ACME_OK) return rc;
  l->num_steps += 1;
  l->seq += 1;
  return ACME_OK;
}

static int step_impl(acme_dqn* l, const acme_transition_batch* batch, const acme_dqn_outputs* out,
                     bool copy, hipStream_t st) {
  int rc = forward_backward_stage(l, batch, out, 0, st, false);
  l->fused_step = true;
  if (rc == ACME_OK) rc = forward_backward_stage(l, batch, out, 1, st, false);
  l->fused_step = false;
  if (rc == ACME_OK) rc = apply_impl(l, copy, st);
  return rc;
}

int acme_dqn_dense_grads_ready(acme_dqn* l, void* stream) {
  ACME_CHECK_ARG(l && l->dense_ev, "no stage 3 / 4 has run");
  ACME_HIP_TRY(hipStreamWaitEvent(as_stream(stream), l->dense_ev, 0));
  return ACME_OK;
}

// ------------------------------------------------------------------ data parallelism
int acme_dqn_dp_init(acme_dqn* l, void* nccl_comm, int32_t world_size) {
  ACME_CHECK_ARG(l && nccl_comm && world_size >= 1, "bad data-parallel arguments");
  if (!acme::rccl::api()) return ACME_ERR_HIP;
  if (!l->dp_stream) {
    ACME_HIP_TRY(hipStreamCreateWithFlags(&l->dp_stream, hipStreamNonBlocking));
    for (auto& e : l->dp_ev) ACME_HIP_TRY(make_order_event(&e));
    int rc = dev_alloc(l, &l->dp_gmin, 1);
    if (rc != ACME_OK) return rc;
  }
  l->dp_comm = nccl_comm;
  l->dp_world = world_size;
  return acme_dqn_set_data_parallel_gate(l, 1);
}

// One data-parallel step (the order of DQNLearner's data_parallel path, itself that of the
// reference's only data-parallel learner, acme/agents/tf/crr/recurrent_learning.py:346-358):
// the batch minimum probability is all-reduced (MIN) on the collective stream beside the
// forwards; the loss and dense backward read the global minimum; the dense gradients
// (99% of the bytes) are all-reduced (AVG) beside the torso backward, as soon as the side
// stream has produced them; then the torso bucket; then Adam on the caller's stream.
int acme_dqn_dp_step(acme_dqn* l, const acme_transition_batch* batch, const acme_dqn_outputs* out,
                     void* stream) {
  ACME_CHECK_ARG(l && batch && l->params, "null argument or unbound learner");
  ACME_CHECK_ARG(l->dp_comm, "acme_dqn_dp_init must be called first");
  const acme::rccl::Api* r = acme::rccl::api();
  if (!r) return ACME_ERR_HIP;
  hipStream_t st = as_stream(stream), cs = l->dp_stream;
  ncclComm_t comm = static_cast<ncclComm_t>(l->dp_comm);
  auto nccl = [&](ncclResult_t e, const char* what) {
    if (e == ncclSuccess) return ACME_OK;
    set_error("%s: %s", what, r->GetErrorString(e));
    return ACME_ERR_HIP;
  };
  int rc = acme_min_f64(batch->probabilities, batch->batch, l->dp_gmin, st);
  if (rc != ACME_OK) return rc;
  ACME_HIP_TRY(hipEventRecord(l->dp_ev[0], st));
  ACME_HIP_TRY(hipStreamWaitEvent(cs, l->dp_ev[0], 0));
  if ((rc = nccl(r->AllReduce(l->dp_gmin, l->dp_gmin, 1, ncclFloat64, ncclMin, comm, cs),
                 "all-reduce (min probability)")))
    return rc;
  ACME_HIP_TRY(hipEventRecord(l->dp_ev[1], cs));
  acme_transition_batch b = *batch;
  b.global_min_probability = l->dp_gmin;
  if ((rc = forward_backward_stage(l, &b, out, 2, st, false))) return rc;
  ACME_HIP_TRY(hipStreamWaitEvent(st, l->dp_ev[1], 0));
  if ((rc = forward_backward_stage(l, &b, out, 4, st, false))) return rc;
  int64_t split = 0;
  if ((rc = acme_dqn_grad_split(l, &split))) return rc;
  ACME_HIP_TRY(hipStreamWaitEvent(cs, l->dense_ev, 0));
  const ncclRedOp_t avg = static_cast<ncclRedOp_t>(ncclAvg);
  if ((rc = nccl(r->AllReduce(l->grads + split, l->grads + split, (size_t)(l->flat - split),
                              ncclFloat32, avg, comm, cs),
                 "all-reduce (dense gradients)")))
    return rc;
  if ((rc = forward_backward_stage(l, &b, out, 1, st, false))) return rc;
  if (split > 0) {
    ACME_HIP_TRY(hipEventRecord(l->dp_ev[2], st));
    ACME_HIP_TRY(hipStreamWaitEvent(cs, l->dp_ev[2], 0));
    if ((rc = nccl(r->AllReduce(l->grads, l->grads, (size_t)split, ncclFloat32, avg, comm, cs),
                   "all-reduce (torso gradients)")))
      return rc;
  }
  ACME_HIP_TRY(hipEventRecord(l->dp_ev[3], cs));
  ACME_HIP_TRY(hipStreamWaitEvent(st, l->dp_ev[3], 0));
  if ((rc = apply_impl(l, copies_target(l), st))) return rc;
  l->num_steps += 1;
  l->seq += 1;
  return ACME_OK;
}

int acme_dqn_step_update(acme_dqn* l, const acme_transition_batch* batch,
                         const acme_dqn_outputs* out, acme_replay* replay, const uint64_t* keys,
                         void* after_event, void* stream) {
  ACME_CHECK_ARG(l && batch && l->params, "null argument or unbound learner");
  ACME_CHECK_ARG(replay && keys, "null replay or keys");
  const bool inside = use_p3(l) && l->cfg.network == ACME_NET_NATURE_DQN && !l->calibrating;
  l->upd_replay = inside ? replay : nullptr;
  l->upd_keys = keys;
  l->upd_prio = nullptr;
  l->upd_after = static_cast<hipEvent_t>(after_event);
  int rc = step_impl(l, batch, out, copies_target(l), as_stream(stream));
  const bool pending = l->upd_replay != nullptr || !inside;
  l->upd_replay = nullptr;
  if (rc != ACME_OK) return rc;
  l->num_steps += 1;
  l->seq += 1;
  if (pending) {  // not issued inside the step (other paths): after it, on the stream
    const double* prio = out && out->priorities ? out->priorities : l->prio_tmp;
    if (after_event)
      ACME_HIP_TRY(hipStreamWaitEvent(as_stream(stream), static_cast<hipEvent_t>(after_event), 0));
    Gate q;  // the plane path's step has ended: its skip decision is `last`
    if (l->p3_capable) {
      q.g = l->guard;
      q.use_last = 1;
    }
    return replay_update_priorities_gated(replay, keys, prio, batch->batch, q,
                                          as_stream(stream));
  }
  return ACME_OK;
}

int acme_dqn_step(acme_dqn* l, const acme_transition_batch* batch, const acme_dqn_outputs* out,
                  void* stream) {
  ACME_CHECK_ARG(l && batch && l->params, "null argument or unbound learner");
  const int rc = step_impl(l, batch, out, copies_target(l), as_stream(stream));
  if (rc != ACME_OK) return rc;
  l->num_steps += 1;
  l->seq += 1;
  return ACME_OK;
}

}  // extern "C"
