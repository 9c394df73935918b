// R2D2 learner step for MI355X: the replacement of R2D2Learner._step
// (acme/agents/tf/r2d2/learning.py:112-200) behind the C ABI (include/acme_hip.h), with
// R2D2AtariNetwork (acme/tf/networks/atari.py:72-112): OAREmbedding(AtariTorso) ->
// snt.LSTM(lstm_size) -> DuellingMLP(num_actions, [head_size]).
//
// One call = the whole step on one stream, no host synchronisation.  The learner works on
// TIME-MAJOR rows (row = t * B + b): the batch's frames and OAR inputs are permuted once at
// the start, so the burn-in prefix (t < burn_in) and the trained suffix are contiguous row
// ranges, every LSTM step reads and writes one contiguous block of B rows, and the backward
// (which stops at t = burn_in, learning.py:134-137: the burn-in is outside the tape) runs
// its GEMMs and the torso backward over the suffix rows only.
//   permute: frames [B, T] -> [T, B]; prev action / reward likewise
//   target network: torso over all T B frames, OAR projection, T LSTM steps from the
//     stored core state (the burn-in is the first burn_in of them), duelling head over
//     the suffix rows -> q_target
//   online network: the same, activations kept -> q
//   loss (one wave per sequence; learning.py:153-178, losses/r2d2.py:29-169): greedy
//     actions, h^-1 bootstrap, n-step targets, h(target), errors, 0.5 sum errors^2,
//     IS weights (1 / (N p))^beta / max, priorities eta max + (1 - eta) mean, d loss / d q
//   backward over the suffix: duelling head, hidden layer, BPTT (t = T-1 .. burn_in), W_h,
//     W_i (+ b), embedding -> conv3 dZ -> torso backward
//   snt.Adam(lr, epsilon); target <- online when num_steps % period == 0     (:78, :181-189)
// Engines: the Atari torso, the OAR projection and their backward on the two-plane f16 engine
// (csrc/gemm_p3.h, the DQN / IMPALA learners' f32-equivalent planes; frames as one exact
// f16 plane; per-tensor power-of-two scales rescaled at the end of every step from its maxima,
// the step guard skipping a step whose planes overflowed); the LSTM, the duelling head and the
// flat torso on f32 MFMA (gemm.h / gemm_x6.h).  ACME_V_R2P3=1 at creation: f32 throughout.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "conv.h"
#include "gemm.h"
#include "gemm_x6.h"
#include "gemm_p3.h"
#include "conv_p3.h"
#include "kernels.h"
#include "profiler.h"
#include "torso.h"
#include "lstm.h"

using namespace acme;
using namespace acme::conv;

namespace {

constexpr int kOarSplits = 8;       // split-K of the Atari OAR projection (K = 7744 + A + 1)
constexpr int kHeadFwdSplits = 16;  // duelling head [rows, A + 1] x K = 2 H2
constexpr int kHeadBwdSplits = 8;   // duelling head weights [2 H2 + 1, A + 1] x K = rows
constexpr int kMaxSeq = 256;        // sequence length bound (the loss kernel's LDS)
constexpr int kFwdLds = 160 * 1024; // LDS per workgroup on gfx950
constexpr int kHiddenWgradSplits = 4;  // split-K of the duelling hidden layer's weight gradient
constexpr int kWhWgradSplits = 2;      // split-K of the W_h weight gradient
constexpr int kOarSplitsP3 = 2;     // split-K of the plane-engine OAR projection (K = 7744)

// Scale records of the plane path: the transient activations / gradients (the target and
// online passes write the same activation planes: one record each, the maximum of both),
// then the online and the target parameter planes (split at the start of every pass).
enum { kScX1, kScX2, kScX3, kScDz3, kScDz2, kScDz1, kScDg, kScParams, kScTParams, kScCount };

struct Tensor {
  std::string name;
  int64_t offset = 0, numel = 0;
  int ndim = 0;
  int64_t shape[4] = {1, 1, 1, 1};
};

int64_t align64(int64_t x) { return (x + 63) & ~int64_t(63); }

}  // namespace

struct acme_r2d2 {
  acme_r2d2_config cfg;
  std::vector<Tensor> tensors;
  int64_t flat = 0;
  int F = 0, D = 0, H = 0, H2 = 0, A = 0;
  int t_c[6] = {-1, -1, -1, -1, -1, -1};
  int t_wi = -1, t_wh = -1, t_b = -1, t_hw = -1, t_hb = -1, t_vw = -1, t_vb = -1, t_aw = -1,
      t_ab = -1;
  float *params = nullptr, *target = nullptr, *grads = nullptr, *m = nullptr, *v = nullptr;
  int64_t num_steps = 0;
  std::vector<void*> allocs;
  // Time-major inputs (R = T B rows): frames (uint8 Atari / f32 flat), prev action / reward.
  void* obs_tm = nullptr;
  int32_t* pa_tm = nullptr;
  float* pr_tm = nullptr;
  float* zero_state = nullptr;  // [B][H] zeros (store_lstm_state = false)
  // Activations (all R rows; the target network's pass reuses them before the online one).
  float *x1 = nullptr, *x2 = nullptr, *x3 = nullptr;
  float *slab = nullptr, *gx = nullptr, *gates = nullptr, *h = nullptr, *c = nullptr;
  float *hid = nullptr, *q = nullptr, *tq = nullptr;  // suffix rows: L B
  // Backward (suffix rows).
  float *g = nullptr, *dzh = nullptr, *dh = nullptr, *dgates = nullptr, *dc = nullptr;
  int32_t* act = nullptr;
  float *dz1 = nullptr, *dz2 = nullptr, *dz3 = nullptr;
  double* loss_part = nullptr;
  float* err_tmp = nullptr;
  double* prio_tmp = nullptr;
  float* loss_tmp = nullptr;
  int bc = 0;        // batch rows per workgroup of the LSTM forward step
  size_t fwd_smem = 0;
  // Plane path (Atari torso): parameter planes of the torso + W_i prefix of the online and
  // the target network, f16 time-major frames, activation / gradient planes, scale records,
  // split-K slab; the step guard (kernels.h StepGuard: a step whose planes overflowed applies
  // no update; Adam's count is guard->applied).
  bool p3 = false;
  int64_t p3_prefix = 0;
  uint16_t *wpl = nullptr, *tpl = nullptr, *frames16 = nullptr;
  torso::Plane x1p{}, x2p{}, x3p{}, dz1p{}, dz2p{}, dz3p{}, dgp{};
  gemm::PScale* scales = nullptr;
  int* overflow = nullptr;
  bool scales_ok = false;
  float* pslab = nullptr;
  StepGuard* guard = nullptr;
  int64_t* host_skipped = nullptr;
  int64_t last_rows = 0;
  // One-launch LSTM unroll and BPTT (lstm.h lstm_fwd_rg_kernel / lstm_bwd_rg_kernel) for
  // H = 256 or 512 with at most 256 co-resident workgroups: the h / dh granule exchange
  // buffers, the launch epoch of their tags, the sticky spin-timeout word; lstm_steps: the
  // per-step kernels instead (acme_r2d2_set_lstm_unroll, tests).
  unsigned long long *xg = nullptr, *xb = nullptr;
  unsigned* tmo = nullptr;
  unsigned lstm_epoch = 0;
  bool lstm_steps = false;
  // ACME_V_RGTRACE=1 at creation: per-step timestamps of the last forward and BPTT launches
  // (debug_buffer "lstm_trace": [2][kMaxSeq][4] u64, forward then BPTT).
  unsigned long long* rg_trace = nullptr;
};

namespace {

// The one-launch unroll's shapes: H of 256 or 512 and ceil(B / 4) x H / 16 <= 256
// workgroups (B <= 32 at H = 512, the R2D2 Atari batch).
bool rg_shape(int H, int B) {
  return (H == 256 || H == 512) && (int64_t)ceil_div(B, kRgRows) * (H / kRgUnits) <= 256;
}
bool lstm_persistent(const acme_r2d2* l, int B) {
  return l->xg && !l->lstm_steps && rg_shape(l->H, B);
}
// The granule tags of the next one-launch unroll: tag0 + t (t < kMaxSeq = 256), tag0 = 256 x
// a per-learner launch count, so no launch can match a granule an earlier one left; the
// buffers are cleared once the count wraps.
unsigned next_lstm_tags(acme_r2d2* l, hipStream_t st) {
  if (++l->lstm_epoch >= (1u << 24)) {
    l->lstm_epoch = 1;
    const int B = l->cfg.max_batch, H = l->H;
    (void)hipMemsetAsync(l->xg, 0, (size_t)2 * B * H * 8, st);
    (void)hipMemsetAsync(l->xb, 0, (size_t)2 * (H / kRgUnits) * B * H * 8, st);
  }
  return l->lstm_epoch << 8;
}

int add_tensor(acme_r2d2* l, const std::string& name, std::initializer_list<int64_t> shape) {
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
  l->tensors.push_back(t);
  return (int)l->tensors.size() - 1;
}

template <class T>
int dev_alloc(acme_r2d2* l, T** p, int64_t count) {
  void* q = nullptr;
  if (hipMalloc(&q, std::max<int64_t>(count, 1) * sizeof(T)) != hipSuccess) {
    set_error("hipMalloc of %lld bytes failed", (long long)(count * sizeof(T)));
    return ACME_ERR_OOM;
  }
  l->allocs.push_back(q);
  *p = static_cast<T*>(q);
  return ACME_OK;
}

inline const float* P(const acme_r2d2* l, const float* base, int t) {
  return base + l->tensors[t].offset;
}
inline float* Pm(const acme_r2d2* l, float* base, int t) { return base + l->tensors[t].offset; }

bool atari(const acme_r2d2* l) { return l->cfg.torso == ACME_IMPALA_TORSO_ATARI; }

inline int chunk_for(int K, int splits) {
  int c = (int)ceil_div(K, splits);
  return (int)ceil_div(c, 32) * 32;
}

#define R2_GEMM(name, BM, BN, WM, WN, WK, prob, splits)                                         \
  do {                                                                                         \
    ACME_PROF_PEAK(name, st, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, 0.0,  \
                   (gemm::matmul_peak_tflops<WK, decltype(prob)>()));                             \
    hipError_t _e = gemm::launch_matmul<BM, BN, WM, WN, 16, WK>(prob, splits, st);              \
    if (_e != hipSuccess) {                                                                    \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__);  \
      return ACME_ERR_HIP;                                                                     \
    }                                                                                          \
  } while (0)

#define R2_CHECK() ACME_LAUNCH_CHECK()

#define R2_P3_GEMM(name, BM, BN, WM, WN, BKV, prob, splits)                                    \
  do {                                                                                         \
    ACME_PROF_PEAK(name, st, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, 0.0, \
                   gemm::p3_peak_tflops<decltype(prob)>());                                    \
    hipError_t _e = gemm::launch_gemm_p3<BM, BN, WM, WN, BKV>(prob, splits, st);              \
    if (_e != hipSuccess) {                                                                    \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                     \
    }                                                                                          \
  } while (0)
#define R2_P3WS_GEMM(name, BM, BN, WM, WN, BKV, prob, splits)                                  \
  do {                                                                                         \
    ACME_PROF_PEAK(name, st, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, 0.0, \
                   gemm::p3_peak_tflops<decltype(prob)>());                                    \
    hipError_t _e = gemm::launch_gemm_p3ws<BM, BN, WM, WN, BKV, true>(prob, splits, st);      \
    if (_e != hipSuccess) {                                                                    \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                     \
    }                                                                                          \
  } while (0)

// Plane views: tensor t of a parameter plane set (record rec), an activation's rows from `row`.
torso::Plane WP(const acme_r2d2* l, uint16_t* planes, int rec, int t) {
  return torso::Plane{planes + l->tensors[t].offset, l->flat, l->scales + rec};
}
torso::Plane rows_from(const torso::Plane& x, int64_t row, int64_t per_row) {
  return torso::Plane{x.p + row * per_row, x.stride, x.sc};
}
gemm::PlaneSrc SRC(const torso::Plane& x, int64_t elems) {
  return gemm::PlaneSrc{x.p, x.stride, (int32_t)(2 * elems), x.sc};
}
torso::PWeights torso_pw(const acme_r2d2* l, const float* prm, uint16_t* planes, int rec) {
  return torso::PWeights{WP(l, planes, rec, l->t_c[0]), WP(l, planes, rec, l->t_c[2]),
                         WP(l, planes, rec, l->t_c[4]), P(l, prm, l->t_c[1]),
                         P(l, prm, l->t_c[3]), P(l, prm, l->t_c[5])};
}

// uint8 frames [B][T] -> exact f16 frames [T][B] (integers 0..255 are exact in f16): 16 bytes
// in, 32 out per thread; the OAR side inputs ride in the same launch (the first B T threads).
__global__ void __launch_bounds__(256) r2d2_frames_f16_kernel(
    const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t units, int B, int T,
    const int32_t* __restrict__ pa, const float* __restrict__ pr, int32_t* __restrict__ pa_tm,
    float* __restrict__ pr_tm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t R = (int64_t)B * T;
  if (i < R) {
    const int b = (int)(i / T), t = (int)(i - (int64_t)b * T);
    pa_tm[(int64_t)t * B + b] = pa[i];
    pr_tm[(int64_t)t * B + b] = pr[i];
  }
  if (i >= R * units) return;
  const int64_t row = i / units, u = i - row * units;
  const int b = (int)(row / T), t = (int)(row - (int64_t)b * T);
  const uint4 v = src[i];
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t o[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint32_t lo = (w[q >> 1] >> (16 * (q & 1))) & 0xffu, hi = (w[q >> 1] >> (16 * (q & 1) + 8)) & 0xffu;
    const _Float16 a = (_Float16)(float)lo, c = (_Float16)(float)hi;
    o[q] = (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, c) << 16);
  }
  uint4* d = dst + (((int64_t)t * B + b) * units + u) * 2;
  d[0] = uint4{o[0], o[1], o[2], o[3]};
  d[1] = uint4{o[4], o[5], o[6], o[7]};
}

// ------------------------------------------------------------------ input permutation
// Batch-major rows (b * T + t) of `unit`-sized records to time-major rows (t * B + b),
// in 16-byte (V = uint4) or 4-byte units.  The OAR side inputs (prev action / reward) ride
// in the same launch (the first B T threads).
template <class V>
__global__ void __launch_bounds__(256) r2d2_permute_kernel(
    const V* __restrict__ src, V* __restrict__ dst, int64_t units, int B, int T,
    const int32_t* __restrict__ pa, const float* __restrict__ pr, int32_t* __restrict__ pa_tm,
    float* __restrict__ pr_tm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t R = (int64_t)B * T;
  if (i < R) {
    const int b = (int)(i / T), t = (int)(i - (int64_t)b * T);
    pa_tm[(int64_t)t * B + b] = pa[i];
    pr_tm[(int64_t)t * B + b] = pr[i];
  }
  if (i >= R * units) return;
  const int64_t row = i / units, u = i - row * units;  // source row b * T + t
  const int b = (int)(row / T), t = (int)(row - (int64_t)b * T);
  dst[((int64_t)t * B + b) * units + u] = src[i];
}

// ------------------------------------------------------------------ loss
// trfl-free restatement of losses/r2d2.py in f32 with TF's operation order (no
// contraction): one 64-thread workgroup per sequence b, lanes over time t of the
// Tm = L - 1 loss steps (L = T - burn_in).
struct R2Loss {
  const float* q;    // [L][B][A] online, suffix rows
  const float* tq;   // [L][B][A] target
  const int32_t* action;  // [B][T] batch-major (the batch's)
  const float *reward, *discount;
  const double* probs;    // [B]
  int B, T, BI, A, n;
  float gamma, eta, one_minus_eta;
  double beta;  // f64, as the reference's exponent of the f64 weights
  double n_replay;  // max_replay_size
  float* g;        // [L][B] d loss / d q[a] (row t * B + b)
  int32_t* act;    // [L][B]
  float* errors;   // [L - 1][B]
  double* prio;    // [B]
  double* loss_part;  // [B]: w_b * 0.5 sum_t errors^2
};

__device__ __forceinline__ float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : x); }

// IEEE (correctly rounded) f32 square root and quotient: evaluated in f64 and rounded once
// to f32, which is exact for both (53 >= 2 x 24 + 2 bits: the double rounding is innocuous).
// (__fsqrt_rn without OCML_BASIC_ROUNDED_OPERATIONS is the native approximation.)
__device__ __forceinline__ float sqrt_rn(float x) { return (float)__builtin_sqrt((double)x); }
__device__ __forceinline__ float div_rn(float x, float y) { return (float)((double)x / (double)y); }

// _signed_hyperbolic_tx (losses/r2d2.py:172-174): sign(x) (sqrt(|x| + 1) - 1) + eps x, in
// TF's f32 operation order, no contraction.
__device__ __forceinline__ float hyperbolic(float x) {
#pragma clang fp contract(off)
  const float s = sqrt_rn(fabsf(x) + 1.f) - 1.f;
  return sgnf(x) * s + 1e-3f * x;
}

// _signed_parabolic_tx (:177-180): z = sqrt(1 + 4 eps (eps + 1 + |x|)) / 2 / eps - 1 / 2 / eps
// (Python folds eps + 1 and 4 eps and 1 / 2 / eps into f32 constants); sign(x) (z^2 - 1).
__device__ __forceinline__ float parabolic(float x) {
#pragma clang fp contract(off)
  const float t = 0.004f * (1.001f + fabsf(x));
  const float z = div_rn(sqrt_rn(1.f + t) * 0.5f, 1e-3f) - 500.f;  // x / 2 exact as x * 0.5
  return sgnf(x) * (z * z - 1.f);
}

// tf.argmax (first maximal index) of online q row (t, b).
__device__ __forceinline__ int greedy(const R2Loss& a, int t, int b) {
  const float* r = a.q + ((size_t)t * a.B + b) * a.A;
  int best = 0;
  float bq = r[0];
  for (int j = 1; j < a.A; ++j)
    if (r[j] > bq) {
      bq = r[j];
      best = j;
    }
  return best;
}

// bootstrap_value[t] = sum_a one_hot(greedy(t + 1))[a] h^-1(target_q[t + 1][a]), summed in
// action order (a non-finite h^-1 anywhere in the row makes it NaN, as the reference's 0 x inf).
__device__ __forceinline__ float bootstrap(const R2Loss& a, int t, int b) {
#pragma clang fp contract(off)
  const int gsel = greedy(a, t + 1, b);
  const float* r = a.tq + ((size_t)(t + 1) * a.B + b) * a.A;
  float s = 0.f;
  for (int j = 0; j < a.A; ++j) s = s + (j == gsel ? 1.f : 0.f) * parabolic(r[j]);
  return s;
}

__global__ void __launch_bounds__(64) r2d2_loss_kernel(const R2Loss a) {
#pragma clang fp contract(off)
  __shared__ float errs[kMaxSeq];
  __shared__ double red[64];
  const int b = blockIdx.x, lane = threadIdx.x;
  const int B = a.B, T = a.T, BI = a.BI, L = T - BI, Tm = L - 1;
  // Importance weight of this sequence: (1 / (N p))^beta / max_b, f64, cast to f32.
  double wmx = 0.0;
  for (int i = lane; i < B; i += 64) wmx = fmax(wmx, pow(1.0 / (a.n_replay * a.probs[i]), a.beta));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wmx = fmax(wmx, __shfl_xor(wmx, o, 64));
  const float w = (float)(pow(1.0 / (a.n_replay * a.probs[b]), a.beta) / wmx);
  const float inv_b = div_rn(1.f, (float)B);
  double sq = 0.0;
  for (int t = lane; t < Tm; t += 64) {
    // n-step target (losses/r2d2.py:122-169): the bootstrap of step min(t + n - 1, Tm - 1),
    // then n folds target = r + pcont target over the padded rewards / pcontinues.
    float target = bootstrap(a, min(t + a.n - 1, Tm - 1), b);
    for (int i = a.n - 1; i >= 0; --i) {
      const int k = t + i;
      const float r = k < Tm ? a.reward[(size_t)b * T + BI + k] : 0.f;
      const float pc = k < Tm ? a.discount[(size_t)b * T + BI + k] * a.gamma : 1.f;
      target = r + pc * target;
    }
    const bool finite = isfinite(target);
    if (!finite) target = 0.f;
    const int at = a.action[(size_t)b * T + BI + t];
    const float qa = a.q[((size_t)t * B + b) * a.A + at];
    const float err = finite ? qa - hyperbolic(target) : 0.f;
    errs[t] = err;
    a.errors[(size_t)t * B + b] = err;
    sq += (double)err * (double)err;
    a.g[(size_t)t * B + b] = (w * err) * inv_b;
    a.act[(size_t)t * B + b] = at;
  }
  if (lane == 0) {  // the last suffix row carries no loss term
    a.g[(size_t)Tm * B + b] = 0.f;
    a.act[(size_t)Tm * B + b] = 0;
  }
  red[lane] = sq;
  __syncthreads();
  if (lane == 0) {
    double s = 0.0;
    for (int i = 0; i < 64; ++i) s += red[i];
    a.loss_part[b] = 0.5 * s * (double)w;
    // compute_priority (learning.py:230-236): f32 max and in-order f32 mean of |errors|.
    float mx = 0.f, sm = 0.f;
    for (int t = 0; t < Tm; ++t) {
      const float e = fabsf(errs[t]);
      mx = fmaxf(mx, e);
      sm = sm + e;
    }
    const float mean = div_rn(sm, (float)Tm);
    a.prio[b] = (double)(a.eta * mx + a.one_minus_eta * mean);
  }
}

// The batch loss; NaN when this step's one-launch LSTM forward timed out (tmo[0]).
__global__ void r2d2_loss_sum_kernel(const double* __restrict__ part, int B,
                                     float* __restrict__ loss, const unsigned* __restrict__ tmo) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int b = 0; b < B; ++b) s += part[b];
  loss[0] = tmo && *tmo ? NAN : (float)(s / (double)B);
}

// The f32 path's step verdict before Adam: skipped when this step's one-launch LSTM timed
// out (tmo[0], then cleared and counted in tmo[1]), else applied (Adam's t = applied).
__global__ void r2d2_guard_kernel(StepGuard* __restrict__ g, unsigned* __restrict__ tmo,
                                  int64_t* __restrict__ host_skipped) {
  if (threadIdx.x != 0) return;
  const bool skip = tmo && tmo[0] != 0u;
  g->last = skip ? 1u : 0u;
  if (skip) {
    tmo[0] = 0u;
    tmo[1] += 1u;
    const int64_t k = g->skipped + 1;
    g->skipped = k;
    if (host_skipped) *host_skipped = k;
  } else {
    g->applied += 1;
  }
}

// dW = X^T dZ over row-major X [rows][ldx] and dZ [rows][N] (M = Kin, N = Nout, K = rows),
// db = column sums of dZ: both operands read as 16-B row segments (conv.h DenseWgrad reads
// X as four scalar loads strided by a row: 137 us for the R2D2 hidden layer).
struct DenseWgradRC {
  static constexpr int A_MODE = gemm::RCONTIG, B_MODE = gemm::RCONTIG;
  static constexpr bool kColSum = true;
  int M, N, K, k_chunk;
  const float* x;
  int ldx;
  const float* dz;
  float* out;
  float* bias_out;
  float* slab;  // split-K partials [splits][M + 1][N] (row M: the column sums), or direct
  struct ARow {
    int i;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int i) const { return ARow{i}; }
  __device__ f32x4 a_load(const ARow& a, int m) const {
    if (a.i >= M || m >= K) return gemm::zero4();
    return load_row4<true>(x + (size_t)m * ldx, a.i, M);
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ f32x4 b_load(const BRow& b, int m) const {
    if (b.n >= N || m >= K) return gemm::zero4();
    return load_row4<true>(dz + (size_t)m * N, b.n, N);
  }
  __device__ void store(int i, int n, float v, int split) const {
    if (slab) slab[((size_t)split * (M + 1) + i) * N + n] = v;
    else out[(size_t)i * N + n] = v;
  }
  __device__ void store_colsum(int n, float v, int split) const {
    if (slab) slab[((size_t)split * (M + 1) + M) * N + n] = v;
    else bias_out[n] = v;
  }
};

// dW_h = h_prev^T dgates over the suffix rows (time-major): h_prev of row m (global row
// BI B + m) is h[m + BI B - B], or the core state h0 for t = 0 (burn_in = 0).
struct HPrevTM {
  static constexpr int A_MODE = gemm::RCONTIG, B_MODE = gemm::RCONTIG;
  int M, N, K, k_chunk;  // M = H, N = 4H, K = L B
  const float* h;        // [R][H]
  const float* h0;
  int64_t h0_stride;
  int B, BI;
  const float* dz;       // [L B][4H]
  float* out;
  float* slab;           // split-K partials [splits][M][N], or direct
  struct ARow {
    int i;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int i) const { return ARow{i}; }
  __device__ f32x4 a_load(const ARow& a, int m) const {
    if (m >= K || a.i >= M) return gemm::zero4();
    const int gr = BI * B + m;
    const float* p = gr < B ? h0 + (size_t)gr * h0_stride : h + (size_t)(gr - B) * M;
    return *reinterpret_cast<const f32x4*>(p + a.i);
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ f32x4 b_load(const BRow& b, int m) const {
    if (b.n >= N || m >= K) return gemm::zero4();
    return load_row4<true>(dz + (size_t)m * N, b.n, N);
  }
  __device__ void store(int i, int n, float v, int split) const {
    if (slab) slab[((size_t)split * M + i) * N + n] = v;
    else out[(size_t)i * N + n] = v;
  }
};

torso::Weights torso_w(const acme_r2d2* l, const float* prm) {
  return torso::Weights{P(l, prm, l->t_c[0]), P(l, prm, l->t_c[1]), P(l, prm, l->t_c[2]),
                        P(l, prm, l->t_c[3]), P(l, prm, l->t_c[4]), P(l, prm, l->t_c[5])};
}

// One network's unroll over all T steps (time-major rows) from the core state, and its
// duelling head over the suffix rows -> q_out [L B][A].
int network_forward(acme_r2d2* l, const float* prm, const acme_sequence_batch* bt, int B, int T,
                    float* q_out, hipStream_t st, uint16_t* planes, int rec, bool online) {
  const int R = B * T, H = l->H, A = l->A, H2 = l->H2, BI = l->cfg.burn_in_length;
  const int L = T - BI, RL = L * B;
  const float* feat = nullptr;
  if (l->p3) {
    // The network's torso + W_i planes at its record's scale, the plane torso (the target's
    // conv1 output stays in LDS: fused conv1 -> conv2), feat @ W_i[0:F] on the plane engine,
    // then the embedding tail (one-hot(prev a), tanh(prev r) rows of W_i) and the bias.
    int rc;
    {
      ACME_PROF("r2d2_planes", st, 0.0, 8.0 * (double)l->p3_prefix);
      rc = launch_split_planes_lagged(prm, l->p3_prefix, planes, l->flat, l->scales + rec, st);
      if (rc != ACME_OK) return rc;
    }
    rc = torso::forward_p3(torso_pw(l, prm, planes, rec), torso::Frames{l->frames16}, R,
                           torso::PActs{l->x1p, l->x2p, l->x3p}, st, online ? -1 : 0);
    if (rc != ACME_OK) return rc;
    const int F = l->F, N = 4 * H;
    P3DenseFwd p;
    // 256x128 tiles at split-K 4 (16 x 16 x 4 blocks at the bench shape): 433 -> 325 us,
    // the split-K reduction 63 -> 30 us, the step 5.16 -> 4.87 ms against 128x128 at split-K
    // 8 (two alternating pairs, round 4; DESIGN.md 4.1 on the per-CU intake).  Split-K 2:
    // 321 -> 301 us, the reduction 30 -> 20 us, the step 4.51 -> 4.44 ms; split-K 1 292 us
    // but the step 4.46 ms (two alternating runs each, profiles/r04/tools/ab_oars.sh).
    const int splits = kOarSplitsP3;
    p.M = R; p.N = N; p.K = F; p.k_chunk = chunk_for(F, splits);
    p.a_src = SRC(l->x3p, (int64_t)R * F); p.ldx = F;
    p.b_src = SRC(WP(l, planes, rec, l->t_wi), (int64_t)F * N); p.slab = l->pslab;
    R2_P3WS_GEMM("r2d2_oar_fwd", 256, 128, 2, 2, 32, p, splits);
    {
      ACME_PROF("r2d2_oar_reduce", st, 0.0, 4.0 * (splits + 1) * (double)R * N);
      const int64_t n4 = (int64_t)R * N / 4;
      oar_finish_kernel<<<(unsigned)ceil_div(n4, 256), 256, 0, st>>>(
          l->pslab, splits, R, N, P(l, prm, l->t_wi) + (size_t)F * N, P(l, prm, l->t_b),
          l->pa_tm, l->pr_tm, A, l->gx);
      R2_CHECK();
    }
  } else if (atari(l)) {
    int rc = torso::forward(torso_w(l, prm), true, l->obs_tm, l->obs_tm, R, R,
                            torso::Acts{l->x1, l->x2, l->x3}, st);
    if (rc != ACME_OK) return rc;
    feat = l->x3;
  } else {
    feat = static_cast<const float*>(l->obs_tm);
  }
  if (!l->p3) {
    OarFwd p;
    p.M = R; p.N = 4 * H; p.K = l->D;
    p.x = Oar{feat, l->F, A, l->pa_tm, l->pr_tm};
    p.w = P(l, prm, l->t_wi); p.bias = P(l, prm, l->t_b); p.y = l->gx;
    if (atari(l)) {
      p.k_chunk = chunk_for(p.K, kOarSplits);
      p.slab = l->slab;
      R2_GEMM("r2d2_oar_fwd", 64, 64, 2, 2, 1, p, kOarSplits);
      ACME_PROF("r2d2_oar_reduce", st, 0.0, 4.0 * (kOarSplits + 1) * (double)R * 4 * H);
      int rc = launch_slab_reduce(l->slab, kOarSplits, (int64_t)R * 4 * H, l->gx,
                                  (int64_t)R * 4 * H, nullptr, P(l, prm, l->t_b), 4 * H, 0, st);
      if (rc != ACME_OK) return rc;
    } else {
      p.k_chunk = p.K;
      p.slab = nullptr;
      R2_GEMM("r2d2_oar_fwd", 32, 32, 1, 1, 8, p, 1);
    }
  }
  {
    ACME_PROF("r2d2_lstm_fwd", st, 2.0 * R * (double)H * 4 * H, 0.0);
    const float* h0 = l->cfg.store_lstm_state ? bt->h0 : l->zero_state;
    const float* c0 = l->cfg.store_lstm_state ? bt->c0 : l->zero_state;
    const int64_t s0 = l->cfg.store_lstm_state ? bt->state_stride : H;
    if (lstm_persistent(l, B)) {  // one launch for the whole unroll, burn-in included
      const unsigned tag0 = next_lstm_tags(l, st);
      const unsigned nblk = (unsigned)(ceil_div(B, kRgRows) * (H / kRgUnits));
      if (H == 512)
        lstm_fwd_rg_kernel<512><<<nblk, 512, 0, st>>>(l->gx, P(l, prm, l->t_wh), h0, s0, c0, s0,
                                                      B, T, 1, B, l->gates, l->h, l->c, l->xg,
                                                      tag0, l->tmo, l->rg_trace);
      else
        lstm_fwd_rg_kernel<256><<<nblk, 256, 0, st>>>(l->gx, P(l, prm, l->t_wh), h0, s0, c0, s0,
                                                      B, T, 1, B, l->gates, l->h, l->c, l->xg,
                                                      tag0, l->tmo, l->rg_trace);
      R2_CHECK();
    } else {
    const dim3 grid((unsigned)(H / kFwdUnits), (unsigned)ceil_div(B, l->bc));
    for (int t = 0; t < T; ++t) {
      const float* hp = t == 0 ? h0 : l->h + (size_t)(t - 1) * B * H;
      const float* cp = t == 0 ? c0 : l->c + (size_t)(t - 1) * B * H;
      const int64_t hs = t == 0 ? s0 : H;
      lstm_fwd_step_kernel<<<grid, 256, l->fwd_smem, st>>>(
          l->gx, P(l, prm, l->t_wh), hp, hs, cp, hs, B, 1, B, t, H, l->gates, l->h, l->c, l->bc);
      R2_CHECK();
    }
    }
  }
  {  // DuellingMLP: the fused [value | advantage] hidden layer over the suffix rows
    DenseFwd<true> p;
    p.M = RL; p.N = 2 * H2; p.K = H; p.k_chunk = H;
    p.x = l->h + (size_t)BI * B * H; p.x2 = p.x; p.split_b = RL; p.ldx = H;
    p.w = P(l, prm, l->t_hw); p.bias = P(l, prm, l->t_hb); p.y = l->hid;
    p.act = ACT_RELU; p.slab = nullptr;
    R2_GEMM("r2d2_hidden_fwd", 64, 64, 2, 2, 1, p, 1);
  }
  {
    DuelHeadFwd p;
    p.M = RL; p.N = A + 1; p.K = 2 * H2; p.k_chunk = chunk_for(p.K, kHeadFwdSplits);
    p.H = H2; p.A = A; p.h = l->hid; p.wv = P(l, prm, l->t_vw); p.wa = P(l, prm, l->t_aw);
    p.slab = l->slab;
    R2_GEMM("r2d2_head_fwd", 64, 32, 2, 1, 1, p, kHeadFwdSplits);
    ACME_PROF("r2d2_head_finish", st, 0.0, 0.0);
    int rc = launch_duel_head_finish(l->slab, kHeadFwdSplits, RL, A, P(l, prm, l->t_vb),
                                     P(l, prm, l->t_ab), q_out, st);
    if (rc != ACME_OK) return rc;
  }
  return ACME_OK;
}

// apply = false: forward, loss and backward only (the plane-scale calibration passes).
int r2d2_step_impl(acme_r2d2* l, const acme_sequence_batch* bt, const double* probs,
                   const acme_r2d2_outputs* out, hipStream_t st, bool apply = true) {
  const int B = (int)bt->batch, T = (int)bt->sequence_length, R = B * T;
  const int H = l->H, A = l->A, H2 = l->H2, BI = l->cfg.burn_in_length;
  const int L = T - BI, RL = L * B;
  int rc;
  {  // time-major inputs
    ACME_PROF("r2d2_permute", st, 0.0,
              (l->p3 ? 3.0 : 2.0) * (double)R * (atari(l) ? torso::kObsBytes : 4 * l->F));
    if (l->p3) {
      const int64_t units = torso::kObsBytes / 16;
      r2d2_frames_f16_kernel<<<(unsigned)ceil_div((int64_t)R * units, 256), 256, 0, st>>>(
          static_cast<const uint4*>(bt->observation), reinterpret_cast<uint4*>(l->frames16),
          units, B, T, bt->prev_action, bt->prev_reward, l->pa_tm, l->pr_tm);
    } else if (atari(l)) {
      const int64_t units = torso::kObsBytes / 16;
      r2d2_permute_kernel<uint4><<<(unsigned)ceil_div((int64_t)R * units, 256), 256, 0, st>>>(
          static_cast<const uint4*>(bt->observation), static_cast<uint4*>(l->obs_tm), units, B, T,
          bt->prev_action, bt->prev_reward, l->pa_tm, l->pr_tm);
    } else {
      const int64_t units = l->F;
      r2d2_permute_kernel<uint32_t><<<(unsigned)ceil_div((int64_t)R * units, 256), 256, 0, st>>>(
          static_cast<const uint32_t*>(bt->observation), static_cast<uint32_t*>(l->obs_tm), units,
          B, T, bt->prev_action, bt->prev_reward, l->pa_tm, l->pr_tm);
    }
    R2_CHECK();
  }
  // Target network first (its activations are overwritten by the online pass).
  l->last_rows = R;
  if ((rc = network_forward(l, l->target, bt, B, T, l->tq, st, l->tpl, kScTParams, false)) !=
      ACME_OK)
    return rc;
  if ((rc = network_forward(l, l->params, bt, B, T, l->q, st, l->wpl, kScParams, true)) != ACME_OK)
    return rc;
  float* errors = out && out->errors ? out->errors : l->err_tmp;
  double* prio = out && out->priorities ? out->priorities : l->prio_tmp;
  float* loss = out && out->loss ? out->loss : l->loss_tmp;
  {
    ACME_PROF("r2d2_loss", st, 0.0, 0.0);
    R2Loss a;
    a.q = l->q; a.tq = l->tq; a.action = bt->action; a.reward = bt->reward;
    a.discount = bt->discount; a.probs = probs;
    a.B = B; a.T = T; a.BI = BI; a.A = A; a.n = l->cfg.n_step;
    a.gamma = l->cfg.discount; a.beta = l->cfg.importance_sampling_exponent;
    a.eta = (float)l->cfg.max_priority_weight;
    a.one_minus_eta = (float)(1.0 - l->cfg.max_priority_weight);
    a.n_replay = (double)l->cfg.max_replay_size;
    a.g = l->g; a.act = l->act; a.errors = errors; a.prio = prio; a.loss_part = l->loss_part;
    r2d2_loss_kernel<<<(unsigned)B, 64, 0, st>>>(a);
    R2_CHECK();
    r2d2_loss_sum_kernel<<<1, 64, 0, st>>>(l->loss_part, B, loss, l->tmo);
    R2_CHECK();
  }
  float* gr = l->grads;
  const float* prm = l->params;
  {  // duelling head: dZ of the hidden layer, the head's weight gradients
    {
      ACME_PROF("r2d2_head_dz", st, 0.0, 0.0);
      rc = launch_duel_head_dz(l->hid, l->g, l->act, RL, H2, A, P(l, prm, l->t_vw),
                               P(l, prm, l->t_aw), l->dzh, st);
      if (rc != ACME_OK) return rc;
    }
    DuelHeadWgrad p;
    p.M = 2 * H2; p.N = A + 1; p.K = RL; p.k_chunk = chunk_for(RL, kHeadBwdSplits);
    p.A = A; p.h = l->hid; p.g = l->g; p.act = l->act; p.slab = l->slab;
    R2_GEMM("r2d2_head_wgrad", 64, 32, 2, 1, 1, p, kHeadBwdSplits);
    ACME_PROF("r2d2_head_scatter", st, 0.0, 0.0);
    rc = launch_duel_head_grad_scatter(l->slab, kHeadBwdSplits, H2, A, Pm(l, gr, l->t_vw),
                                       Pm(l, gr, l->t_vb), Pm(l, gr, l->t_aw),
                                       Pm(l, gr, l->t_ab), st);
    if (rc != ACME_OK) return rc;
  }
  const float* hs = l->h + (size_t)BI * B * H;  // the suffix's LSTM outputs
  {  // hidden layer: weights over the suffix rows, and d h
    // Split-K 4 over the 2,592 rows (8 x 16 tiles x 4 = 512 blocks), reduced with the bias.
    DenseWgradRC w;
    w.M = H; w.N = 2 * H2; w.K = RL; w.k_chunk = chunk_for(RL, kHiddenWgradSplits);
    w.x = hs; w.ldx = H; w.dz = l->dzh; w.out = Pm(l, gr, l->t_hw); w.bias_out = Pm(l, gr, l->t_hb);
    w.slab = l->slab;
    R2_GEMM("r2d2_hidden_wgrad", 64, 64, 2, 2, 1, w, kHiddenWgradSplits);
    {
      ACME_PROF("r2d2_hidden_wgrad_reduce", st, 0.0,
                4.0 * (kHiddenWgradSplits + 1) * (double)(H + 1) * 2 * H2);
      rc = launch_slab_reduce(l->slab, kHiddenWgradSplits, (int64_t)(H + 1) * 2 * H2,
                              Pm(l, gr, l->t_hw), (int64_t)H * 2 * H2, Pm(l, gr, l->t_hb),
                              nullptr, 0, 0, st);
      if (rc != ACME_OK) return rc;
    }
    DenseDgrad<true> d;
    d.M = RL; d.N = H; d.K = 2 * H2; d.k_chunk = 2 * H2;
    d.dz = l->dzh; d.w = P(l, prm, l->t_hw); d.xprev = nullptr; d.ldx = H;
    d.dx = l->dh + (size_t)BI * B * H;
    R2_GEMM("r2d2_hidden_dgrad", 64, 64, 2, 2, 1, d, 1);
  }
  {  // BPTT over t = T-1 .. burn_in (the burn-in is outside the gradient tape)
    ACME_PROF("r2d2_lstm_bwd", st, 2.0 * RL * (double)H * 4 * H, 0.0);
    const float* c0 = l->cfg.store_lstm_state ? bt->c0 : l->zero_state;
    const int64_t s0 = l->cfg.store_lstm_state ? bt->state_stride : H;
    // dgates rows are those of the suffix: the kernel's row (t, b) = t B + b is offset by
    // -BI B so that t >= BI lands on dgates[(t - BI) B + b].
    float* dg = l->dgates - (ptrdiff_t)BI * B * 4 * H;
    if (lstm_persistent(l, B)) {  // one launch for the whole BPTT, stopping at the burn-in
      const unsigned tag0 = next_lstm_tags(l, st);
      const unsigned nblk = (unsigned)(ceil_div(B, kRgRows) * (H / kRgUnits));
      if (H == 512)
        lstm_bwd_rg_kernel<512><<<nblk, 512, 0, st>>>(l->dh, P(l, prm, l->t_wh), l->gates, l->c,
                                                      c0, s0, B, T, BI, 1, B, dg, l->xb, tag0,
                                                      l->tmo, l->rg_trace ? l->rg_trace + 4 * kMaxSeq : nullptr);
      else
        lstm_bwd_rg_kernel<256><<<nblk, 256, 0, st>>>(l->dh, P(l, prm, l->t_wh), l->gates, l->c,
                                                      c0, s0, B, T, BI, 1, B, dg, l->xb, tag0,
                                                      l->tmo, l->rg_trace ? l->rg_trace + 4 * kMaxSeq : nullptr);
      R2_CHECK();
    } else {
    ACME_HIP_TRY(hipMemsetAsync(l->dc, 0, (size_t)B * H * sizeof(float), st));
    const dim3 bgrid((unsigned)(H / kUnits), (unsigned)ceil_div(B, kRowChunk));
    for (int t = T - 1; t >= BI; --t) {
      lstm_bwd_step_kernel<<<bgrid, 256, 0, st>>>(l->dh, P(l, prm, l->t_wh), l->gates, l->c,
                                                       c0, s0, l->dc, dg, B, T, t, H, 1, B);
      R2_CHECK();
    }
    }
  }
  {  // W_h over h_prev of the suffix rows
    HPrevTM w;
    w.M = H; w.N = 4 * H; w.K = RL; w.k_chunk = RL;
    w.h = l->h; w.h0 = l->cfg.store_lstm_state ? bt->h0 : l->zero_state;
    w.h0_stride = l->cfg.store_lstm_state ? bt->state_stride : H;
    w.B = B; w.BI = BI; w.dz = l->dgates; w.out = Pm(l, gr, l->t_wh);
    // Split-K 2 (8 x 32 tiles x 2 = 512 blocks).
    w.k_chunk = chunk_for(RL, kWhWgradSplits);
    w.slab = l->slab;
    R2_GEMM("r2d2_wh_wgrad", 64, 64, 2, 2, 1, w, kWhWgradSplits);
    {
      ACME_PROF("r2d2_wh_wgrad_reduce", st, 0.0, 4.0 * (kWhWgradSplits + 1) * (double)H * 4 * H);
      rc = launch_slab_reduce(l->slab, kWhWgradSplits, (int64_t)H * 4 * H, Pm(l, gr, l->t_wh),
                              (int64_t)H * 4 * H, nullptr, nullptr, 0, 0, st);
      if (rc != ACME_OK) return rc;
    }
  }
  if (l->p3) {  // W_i, b and the embedding gradient on the plane engine, then the plane torso
    const int F = l->F, N = 4 * H;
    const int64_t off = (int64_t)BI * B;
    {
      ACME_PROF("r2d2_dgates_planes", st, 0.0, 8.0 * (double)RL * N);
      rc = launch_split_planes_lagged(l->dgates, (int64_t)RL * N, l->dgp.p, l->dgp.stride,
                                      l->dgp.sc, st);
      if (rc != ACME_OK) return rc;
    }
    const torso::Plane x3s = rows_from(l->x3p, off, F);
    {
      P3DenseWgrad w;
      w.M = F; w.N = N; w.K = RL; w.k_chunk = RL;
      w.a_src = SRC(x3s, (int64_t)RL * F); w.ldx = F;
      w.b_src = SRC(l->dgp, (int64_t)RL * N); w.out = Pm(l, gr, l->t_wi);
      w.bias_out = Pm(l, gr, l->t_b);
      // 256x128 warp-specialised tiles over the 2,592-row reduction: 233 -> 188 us against
      // 128x128 single-role at BK 16 (single-role 256x128: 257 us; round 4).
      R2_P3WS_GEMM("r2d2_wi_wgrad", 256, 128, 2, 2, 32, w, 1);
    }
    {
      ACME_PROF("r2d2_wi_wgrad_tail", st, 0.0, 4.0 * (double)RL * N);
      const int tw = tail_waves(A);
      oar_wgrad_tail_kernel<<<(unsigned)ceil_div(N, 64), 64 * tw,
                              (size_t)tw * (A + 1) * 64 * sizeof(float), st>>>(
          l->dgates, RL, N, l->pa_tm + off, l->pr_tm + off, A,
          Pm(l, gr, l->t_wi) + (size_t)F * N);
      R2_CHECK();
    }
    {
      P3DenseDgrad d;
      d.M = RL; d.N = F; d.K = N; d.k_chunk = N;
      d.a_src = SRC(l->dgp, (int64_t)RL * N);
      d.b_src = SRC(WP(l, l->wpl, kScParams, l->t_wi), (int64_t)F * N);
      d.xprev = CPlanes{x3s.p, x3s.stride, x3s.sc}; d.ldx = F;
      d.dx = Planes{l->dz3p.p, l->dz3p.stride, l->dz3p.sc};
      // 256x128 tiles (11 x 61 blocks): 311 -> 278 us against 128x128 (round 4).
      R2_P3WS_GEMM("r2d2_feat_dgrad", 256, 128, 2, 2, 32, d, 1);
    }
    torso::Grads g{Pm(l, gr, l->t_c[0]), Pm(l, gr, l->t_c[1]), Pm(l, gr, l->t_c[2]),
                   Pm(l, gr, l->t_c[3]), Pm(l, gr, l->t_c[4]), Pm(l, gr, l->t_c[5])};
    rc = torso::backward_p3(torso_pw(l, prm, l->wpl, kScParams), g,
                            torso::Frames{l->frames16 + off * torso::kObsBytes}, RL,
                            torso::PActs{rows_from(l->x1p, off, torso::kX1),
                                         rows_from(l->x2p, off, F), x3s},
                            l->dz3p, l->dz2p, l->dz1p, l->pslab, st);
    if (rc != ACME_OK) return rc;
    // Every record's next scale from this step's maxima; with apply, the guard's decision
    // for this step (kRgStep: skip when a plane write overflowed or underflowed) and its
    // counts, read by Adam's gate.
    RescaleGuard rg;
    if (apply) {
      rg.g = l->guard;
      rg.mode = kRgStep;
      rg.host_skipped = l->host_skipped;
      rg.tmo = l->tmo;
    }
    rc = launch_plane_rescale(l->scales, kScCount, kScCount, -1, -1, l->overflow, st, -1, -1, rg);
    if (rc != ACME_OK) return rc;
    if (!apply) return ACME_OK;
  }
  const float* feat = atari(l) ? l->x3 + (size_t)BI * B * l->F
                               : static_cast<const float*>(l->obs_tm) + (size_t)BI * B * l->F;
  if (!l->p3) {  // W_i (+ b) over the suffix's OAR embedding
    OarWgrad o;
    o.M = l->D; o.N = 4 * H; o.K = RL; o.k_chunk = RL;
    o.x = Oar{feat, l->F, A, l->pa_tm + (size_t)BI * B, l->pr_tm + (size_t)BI * B};
    o.dz = l->dgates; o.out = Pm(l, gr, l->t_wi); o.bias_out = Pm(l, gr, l->t_b);
    if (atari(l)) R2_GEMM("r2d2_wi_wgrad", 128, 128, 2, 2, 1, o, 1);
    else R2_GEMM("r2d2_wi_wgrad", 32, 32, 1, 1, 8, o, 1);
  }
  if (atari(l) && !l->p3) {  // embedding features -> conv3 dZ -> torso backward (suffix frames)
    DenseDgrad<true> d;
    d.M = RL; d.N = l->F; d.K = 4 * H; d.k_chunk = 4 * H;
    d.dz = l->dgates; d.w = P(l, prm, l->t_wi); d.xprev = feat; d.ldx = l->F;
    d.dx = l->dz3; d.act = ACT_RELU;
    R2_GEMM("r2d2_feat_dgrad", 64, 128, 2, 2, 1, d, 1);
    torso::Grads g{Pm(l, gr, l->t_c[0]), Pm(l, gr, l->t_c[1]), Pm(l, gr, l->t_c[2]),
                   Pm(l, gr, l->t_c[3]), Pm(l, gr, l->t_c[4]), Pm(l, gr, l->t_c[5])};
    const size_t off = (size_t)BI * B;
    rc = torso::backward(torso_w(l, prm), g, true,
                         static_cast<const uint8_t*>(l->obs_tm) + off * torso::kObsBytes, RL,
                         torso::Acts{l->x1 + off * torso::kX1, l->x2 + off * torso::kFlat,
                                     l->x3 + off * torso::kFlat},
                         l->dz3, l->dz2, l->dz1, l->slab, st);
    if (rc != ACME_OK) return rc;
  }
  if (!apply) return ACME_OK;
  {
    ACME_PROF("r2d2_adam", st, 0.0, 7.0 * 4.0 * (double)l->flat);
    if (l->p3) {  // gated: a skipped step leaves p, m and v; t = the applied updates
      Gate gate;
      gate.g = l->guard;
      gate.use_last = 1;
      AdamTail tail;
      tail.clear = l->guard;
      rc = launch_adam(l->params, gr, l->m, l->v, l->flat, l->cfg.learning_rate,
                       l->cfg.adam_beta1, l->cfg.adam_beta2, l->cfg.adam_epsilon, 0, nullptr, 0,
                       st, 0, &l->guard->applied, nullptr, gate, false, tail);
    } else {  // the same gate, decided here: only an LSTM timeout skips the f32 path
      r2d2_guard_kernel<<<1, 64, 0, st>>>(l->guard, l->tmo, l->host_skipped);
      R2_CHECK();
      Gate gate;
      gate.g = l->guard;
      gate.use_last = 1;
      rc = launch_adam(l->params, gr, l->m, l->v, l->flat, l->cfg.learning_rate,
                       l->cfg.adam_beta1, l->cfg.adam_beta2, l->cfg.adam_epsilon, 0, nullptr, 0,
                       st, 0, &l->guard->applied, nullptr, gate, false, AdamTail{});
    }
    if (rc != ACME_OK) return rc;
  }
  if (l->num_steps % l->cfg.target_update_period == 0) {  // learning.py:185-189, after the update
    // Gated on the step's verdict: a skipped step copies nothing (its parameters are the
    // pre-step ones).
    Gate gate;
    gate.g = l->guard;
    gate.use_last = 1;
    if ((rc = launch_copy_gated(l->target, l->params, (size_t)l->flat * sizeof(float), nullptr,
                                nullptr, 0, gate, st)) != ACME_OK)
      return rc;
  }
  return ACME_OK;
}

}  // namespace

extern "C" {

int acme_r2d2_destroy(acme_r2d2* l) {
  if (!l) return ACME_OK;
  (void)hipDeviceSynchronize();
  for (void* p : l->allocs) (void)hipFree(p);
  if (l->host_skipped) (void)hipHostFree(l->host_skipped);
  delete l;
  return ACME_OK;
}

int acme_r2d2_create(const acme_r2d2_config* cfg, acme_r2d2** out) {
  ACME_CHECK_ARG(cfg && out, "null argument");
  ACME_CHECK_ARG(cfg->torso == ACME_IMPALA_TORSO_ATARI || cfg->torso == ACME_IMPALA_TORSO_FLAT,
                 "unknown torso %d", cfg->torso);
  ACME_CHECK_ARG(cfg->torso == ACME_IMPALA_TORSO_ATARI || cfg->obs_dim >= 1,
                 "obs_dim must be >= 1 for the flat torso");
  ACME_CHECK_ARG(cfg->num_actions >= 1 && cfg->num_actions <= 1024, "num_actions must be in [1, 1024]");
  ACME_CHECK_ARG(cfg->max_batch >= 1 && cfg->max_batch <= 1024, "max_batch must be in [1, 1024]");
  ACME_CHECK_ARG(cfg->burn_in_length >= 0, "burn_in_length must be >= 0");
  ACME_CHECK_ARG(cfg->max_sequence_length >= cfg->burn_in_length + 2 &&
                     cfg->max_sequence_length <= kMaxSeq,
                 "max_sequence_length must be in [burn_in_length + 2, %d]", kMaxSeq);
  ACME_CHECK_ARG(cfg->lstm_size >= 8 && cfg->lstm_size % 8 == 0,
                 "lstm_size must be a positive multiple of 8");
  ACME_CHECK_ARG(cfg->head_size >= 8 && cfg->head_size % 8 == 0,
                 "head_size must be a positive multiple of 8");
  ACME_CHECK_ARG(cfg->n_step >= 1, "n_step must be >= 1");
  ACME_CHECK_ARG(cfg->target_update_period >= 1, "target_update_period must be >= 1");
  ACME_CHECK_ARG(cfg->max_replay_size >= 1, "max_replay_size must be >= 1");
  acme_r2d2* l = new acme_r2d2();
  l->cfg = *cfg;
  auto fail = [&](int code) {
    acme_r2d2_destroy(l);
    return code;
  };
  l->A = cfg->num_actions;
  l->H = cfg->lstm_size;
  l->H2 = cfg->head_size;
  l->F = cfg->torso == ACME_IMPALA_TORSO_ATARI ? torso::kFlat : cfg->obs_dim;
  l->D = l->F + l->A + 1;
  // Rows of the LSTM forward step per workgroup: h_prev of those rows and the workgroup's
  // W_h columns are staged in LDS (up to 160 KB on gfx950).
  const int H = l->H, A = l->A, H2 = l->H2, B = cfg->max_batch;
  // 16 rows (one mat-vec pass) per workgroup: the step's grid is H / 4 x B / 16 workgroups
  // (256 at H 512, B 32), each staging a sixteenth of the batch's h_prev.
  l->bc = std::min(B, 16);
  while (l->bc > 1 && lstm_fwd_smem(l->bc, H) > (size_t)kFwdLds) l->bc = (l->bc + 1) / 2;
  l->fwd_smem = lstm_fwd_smem(l->bc, H);
  ACME_CHECK_ARG(l->fwd_smem <= (size_t)kFwdLds, "lstm_size too large for the LSTM step kernel");
  if (l->fwd_smem > 65536 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(lstm_fwd_step_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)l->fwd_smem) != hipSuccess)
    return fail((set_error("LSTM step kernel: %zu B of LDS refused", l->fwd_smem), ACME_ERR_HIP));
  const std::string pre = "r2d2_atari_network/";
  if (cfg->torso == ACME_IMPALA_TORSO_ATARI) {
    l->t_c[0] = add_tensor(l, pre + "atari_torso/conv2_d/w", {8, 8, 4, 32});
    l->t_c[1] = add_tensor(l, pre + "atari_torso/conv2_d/b", {32});
    l->t_c[2] = add_tensor(l, pre + "atari_torso/conv2_d_1/w", {4, 4, 32, 64});
    l->t_c[3] = add_tensor(l, pre + "atari_torso/conv2_d_1/b", {64});
    l->t_c[4] = add_tensor(l, pre + "atari_torso/conv2_d_2/w", {3, 3, 64, 64});
    l->t_c[5] = add_tensor(l, pre + "atari_torso/conv2_d_2/b", {64});
  }
  l->t_wi = add_tensor(l, pre + "lstm/w_i", {l->D, 4 * H});
  l->t_wh = add_tensor(l, pre + "lstm/w_h", {H, 4 * H});
  l->t_b = add_tensor(l, pre + "lstm/b", {4 * H});
  // Fused [value_mlp/linear_0 | advantage_mlp/linear_0] as in the DQN learner.
  l->t_hw = add_tensor(l, pre + "duelling_q_network/hidden/w", {H, 2 * H2});
  l->t_hb = add_tensor(l, pre + "duelling_q_network/hidden/b", {2 * H2});
  l->t_vw = add_tensor(l, pre + "duelling_q_network/mlp/linear_1/w", {H2, 1});
  l->t_vb = add_tensor(l, pre + "duelling_q_network/mlp/linear_1/b", {1});
  l->t_aw = add_tensor(l, pre + "duelling_q_network/mlp_1/linear_1/w", {H2, A});
  l->t_ab = add_tensor(l, pre + "duelling_q_network/mlp_1/linear_1/b", {A});
  const int T = cfg->max_sequence_length;
  const int64_t R = (int64_t)B * T, RL = (int64_t)B * (T - cfg->burn_in_length);
  int rc;
  int64_t slab = std::max<int64_t>({(int64_t)kHeadFwdSplits * RL * (A + 1),
                                    (int64_t)kHeadBwdSplits * (2 * H2 + 1) * (A + 1),
                                    (int64_t)kHiddenWgradSplits * (H + 1) * 2 * H2,
                                    (int64_t)kWhWgradSplits * H * 4 * H, (int64_t)64});
  if (cfg->torso == ACME_IMPALA_TORSO_ATARI) {
    slab = std::max<int64_t>({slab, torso::wgrad_slab_floats(), (int64_t)kOarSplits * R * 4 * H});
    // (On the plane path x1..x3 serve the debug buffers only: the planes joined to f32.)
    if ((rc = dev_alloc(l, reinterpret_cast<uint8_t**>(&l->obs_tm), R * torso::kObsBytes)) ||
        (rc = dev_alloc(l, &l->x1, R * torso::kX1)) || (rc = dev_alloc(l, &l->x2, R * torso::kFlat)) ||
        (rc = dev_alloc(l, &l->x3, R * torso::kFlat)) || (rc = dev_alloc(l, &l->dz1, RL * torso::kX1)) ||
        (rc = dev_alloc(l, &l->dz2, RL * torso::kFlat)) || (rc = dev_alloc(l, &l->dz3, RL * torso::kFlat)))
      return fail(rc);
  } else if ((rc = dev_alloc(l, reinterpret_cast<float**>(&l->obs_tm), R * l->F))) {
    return fail(rc);
  }
  // Plane path for the Atari torso (each operand plane is addressed through a 31-bit byte
  // range: the f16 frames of one step bound the batch), unless ACME_V_R2P3=1.
  l->p3 = cfg->torso == ACME_IMPALA_TORSO_ATARI && R * torso::kObsBytes * 2 < (int64_t)INT32_MAX &&
          tune_variant("R2P3") != 1;
  if ((rc = dev_alloc(l, &l->guard, 1))) return fail(rc);
  if (hipMemset(l->guard, 0, sizeof(StepGuard)) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&l->host_skipped), sizeof(int64_t),
                    hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
    return fail((set_error("step guard allocation failed"), ACME_ERR_HIP));
  *l->host_skipped = 0;
  if (l->p3) {
    l->p3_prefix = align64(l->tensors[l->t_wi].offset + l->tensors[l->t_wi].numel);
    if ((rc = dev_alloc(l, &l->scales, kScCount)) || (rc = dev_alloc(l, &l->overflow, 1)))
      return fail(rc);
    std::vector<gemm::PScale> init(kScCount);
    std::memset(init.data(), 0, init.size() * sizeof(gemm::PScale));
    for (auto& r : init) {
      r.w = r.r = r.wi = r.rl = 1.f;
      r.flag = &l->guard->on;
    }
    if (hipMemcpy(l->scales, init.data(), init.size() * sizeof(gemm::PScale),
                  hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(l->overflow, 0, sizeof(int)) != hipSuccess)
      return fail((set_error("scale record init failed"), ACME_ERR_HIP));
    auto plane = [&](torso::Plane* x, int64_t count, int rec) {
      const int64_t stride = align64(count);
      uint16_t* q = nullptr;
      int r = dev_alloc(l, &q, gemm::kPlanes * stride);
      *x = torso::Plane{q, stride, l->scales + rec};
      return r;
    };
    const int64_t N = 4 * (int64_t)H;
    if ((rc = dev_alloc(l, &l->wpl, gemm::kPlanes * l->flat)) ||
        (rc = dev_alloc(l, &l->tpl, gemm::kPlanes * l->flat)) ||
        (rc = dev_alloc(l, &l->frames16, R * torso::kObsBytes)) ||
        (rc = plane(&l->x1p, R * torso::kX1, kScX1)) ||
        (rc = plane(&l->x2p, R * torso::kFlat, kScX2)) ||
        (rc = plane(&l->x3p, R * torso::kFlat, kScX3)) ||
        (rc = plane(&l->dz1p, RL * torso::kX1, kScDz1)) ||
        (rc = plane(&l->dz2p, RL * torso::kFlat, kScDz2)) ||
        (rc = plane(&l->dz3p, RL * torso::kFlat, kScDz3)) ||
        (rc = plane(&l->dgp, RL * N, kScDg)) ||
        (rc = dev_alloc(l, &l->pslab, std::max<int64_t>(torso::wgrad_slab_floats_p3(),
                                                        (int64_t)kOarSplitsP3 * R * N))))
      return fail(rc);
  }
  if ((rc = dev_alloc(l, &l->slab, slab)) || (rc = dev_alloc(l, &l->pa_tm, R)) ||
      (rc = dev_alloc(l, &l->pr_tm, R)) || (rc = dev_alloc(l, &l->zero_state, (int64_t)B * H)) ||
      (rc = dev_alloc(l, &l->gx, R * 4 * H)) || (rc = dev_alloc(l, &l->gates, R * 4 * H)) ||
      (rc = dev_alloc(l, &l->h, R * H)) || (rc = dev_alloc(l, &l->c, R * H)) ||
      (rc = dev_alloc(l, &l->hid, RL * 2 * H2)) || (rc = dev_alloc(l, &l->q, RL * A)) ||
      (rc = dev_alloc(l, &l->tq, RL * A)) || (rc = dev_alloc(l, &l->g, RL)) ||
      (rc = dev_alloc(l, &l->act, RL)) || (rc = dev_alloc(l, &l->dzh, RL * 2 * H2)) ||
      (rc = dev_alloc(l, &l->dh, R * H)) || (rc = dev_alloc(l, &l->dgates, RL * 4 * H)) ||
      (rc = dev_alloc(l, &l->dc, (int64_t)B * H)) || (rc = dev_alloc(l, &l->loss_part, B)) ||
      (rc = dev_alloc(l, &l->err_tmp, RL)) || (rc = dev_alloc(l, &l->prio_tmp, B)) ||
      (rc = dev_alloc(l, &l->loss_tmp, 1)))
    return fail(rc);
  if (rg_shape(H, B)) {  // the one-launch unroll's granule buffers (never cleared per launch)
    const int64_t G = H / kRgUnits;
    if ((rc = dev_alloc(l, &l->xg, (int64_t)2 * B * H)) ||
        (rc = dev_alloc(l, &l->xb, 2 * G * B * H)) || (rc = dev_alloc(l, &l->tmo, 4)) ||
        (tune_variant("RGTRACE") == 1 && (rc = dev_alloc(l, &l->rg_trace, 8 * kMaxSeq))))
      return fail(rc);
    if (hipMemset(l->xg, 0, (size_t)2 * B * H * 8) != hipSuccess ||
        hipMemset(l->xb, 0, (size_t)2 * G * B * H * 8) != hipSuccess ||
        hipMemset(l->tmo, 0, 4 * sizeof(unsigned)) != hipSuccess)
      return fail((set_error("hipMemset failed"), ACME_ERR_HIP));
  }
  if (hipMemset(l->zero_state, 0, (size_t)B * H * sizeof(float)) != hipSuccess)
    return fail((set_error("hipMemset failed"), ACME_ERR_HIP));
  *out = l;
  return ACME_OK;
}

int64_t acme_r2d2_flat_size(const acme_r2d2* l) { return l ? l->flat : 0; }
int32_t acme_r2d2_num_tensors(const acme_r2d2* l) { return l ? (int32_t)l->tensors.size() : 0; }

int acme_r2d2_tensor_info(const acme_r2d2* l, int32_t i, int64_t* offset, int64_t* numel,
                          int32_t* ndim, int64_t* shape4, const char** name) {
  ACME_CHECK_ARG(l, "null learner");
  ACME_CHECK_ARG(i >= 0 && i < (int32_t)l->tensors.size(), "tensor index %d out of range", i);
  const Tensor& t = l->tensors[i];
  if (offset) *offset = t.offset;
  if (numel) *numel = t.numel;
  if (ndim) *ndim = t.ndim;
  if (shape4)
    for (int k = 0; k < 4; ++k) shape4[k] = t.shape[k];
  if (name) *name = t.name.c_str();
  return ACME_OK;
}

int acme_r2d2_bind(acme_r2d2* l, float* params, float* target, float* grads, float* adam_m,
                   float* adam_v) {
  ACME_CHECK_ARG(l, "null learner");
  ACME_CHECK_ARG(params && target && grads && adam_m && adam_v, "null buffer");
  l->params = params;
  l->target = target;
  l->grads = grads;
  l->m = adam_m;
  l->v = adam_v;
  l->scales_ok = false;
  return ACME_OK;
}

int acme_r2d2_params_changed(acme_r2d2* l) {
  ACME_CHECK_ARG(l, "null learner");
  l->scales_ok = false;
  return ACME_OK;
}

int acme_r2d2_scale_state(const acme_r2d2* l, float* out, int32_t capacity, int32_t* count) {
  ACME_CHECK_ARG(l && count, "null argument");
  *count = l->scales ? 4 * kScCount : 0;
  if (!l->scales || !out) return ACME_OK;
  ACME_CHECK_ARG(capacity >= 4 * kScCount, "scale state needs %d floats", 4 * kScCount);
  ACME_HIP_TRY(hipDeviceSynchronize());
  for (int i = 0; i < kScCount; ++i)
    ACME_HIP_TRY(hipMemcpy(out + 4 * i, l->scales + i, 4 * sizeof(float), hipMemcpyDeviceToHost));
  return ACME_OK;
}

int acme_r2d2_set_scale_state(acme_r2d2* l, const float* in, int32_t count) {
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
  return ACME_OK;
}

int acme_r2d2_step(acme_r2d2* l, const acme_sequence_batch* b, const double* probabilities,
                   const acme_r2d2_outputs* out, void* stream) {
  ACME_CHECK_ARG(l && b && probabilities, "null argument");
  ACME_CHECK_ARG(l->params, "acme_r2d2_bind must be called first");
  ACME_CHECK_ARG(b->batch >= 1 && b->batch <= l->cfg.max_batch, "batch %lld outside [1, %d]",
                 (long long)b->batch, l->cfg.max_batch);
  ACME_CHECK_ARG(b->sequence_length >= l->cfg.burn_in_length + 2 &&
                     b->sequence_length <= l->cfg.max_sequence_length,
                 "sequence_length %lld outside [burn_in_length + 2 = %d, %d]",
                 (long long)b->sequence_length, l->cfg.burn_in_length + 2,
                 l->cfg.max_sequence_length);
  ACME_CHECK_ARG(b->observation && b->prev_action && b->prev_reward && b->action && b->reward &&
                     b->discount,
                 "null batch field");
  ACME_CHECK_ARG(!l->cfg.store_lstm_state ||
                     (b->h0 && b->c0 && b->state_stride >= l->H && b->state_stride % 4 == 0 &&
                      ((uintptr_t)b->h0 & 15) == 0 && ((uintptr_t)b->c0 & 15) == 0),
                 "core state rows must be 16-byte aligned with state_stride >= lstm_size");
  ACME_CHECK_ARG(!atari(l) || ((uintptr_t)b->observation & 15) == 0,
                 "frames must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  int rc = ACME_OK;
  if (l->p3 && !l->scales_ok) {
    // Plane scales for newly bound parameters: forward + backward passes without the update,
    // each ending with the rescale; four, for the input-gradient chain dgates -> dz3 -> dz2
    // -> dz1 (a tensor computed from planes that underflowed at their initial scale measures
    // 0 until its input is calibrated, as the DQN / IMPALA learners' calibration).
    for (int pass = 0; pass < 4 && rc == ACME_OK; ++pass)
      rc = r2d2_step_impl(l, b, probabilities, out, st, false);
    if (rc != ACME_OK) return rc;
    ACME_HIP_TRY(hipMemsetAsync(l->overflow, 0, sizeof(int), st));
    ACME_HIP_TRY(hipMemsetAsync(l->guard, 0, offsetof(StepGuard, applied), st));
    // A calibration pass's LSTM timeout is not the first step's (as IMPALA's calibration).
    if (l->tmo) ACME_HIP_TRY(hipMemsetAsync(l->tmo, 0, sizeof(unsigned), st));
    l->scales_ok = true;
  }
  rc = r2d2_step_impl(l, b, probabilities, out, st);
  if (rc != ACME_OK) return rc;
  l->num_steps += 1;
  return ACME_OK;
}

int acme_r2d2_set_lstm_unroll(acme_r2d2* l, int32_t mode) {
  ACME_CHECK_ARG(l && (mode == 0 || mode == 1), "mode must be 0 (one launch) or 1 (per step)");
  l->lstm_steps = mode == 1;
  return ACME_OK;
}

int64_t acme_r2d2_skipped_steps(const acme_r2d2* l) {
  if (!l || !l->host_skipped) return 0;
  return *reinterpret_cast<volatile const int64_t*>(l->host_skipped);
}

int acme_r2d2_guard_state(acme_r2d2* l, int64_t* out3) {
  ACME_CHECK_ARG(l && out3, "null argument");
  ACME_HIP_TRY(hipDeviceSynchronize());
  StepGuard g;
  ACME_HIP_TRY(hipMemcpy(&g, l->guard, sizeof(g), hipMemcpyDeviceToHost));
  out3[0] = g.applied;
  out3[1] = g.skipped;
  out3[2] = g.last;
  return ACME_OK;
}

int acme_r2d2_set_applied_steps(acme_r2d2* l, int64_t n) {
  ACME_CHECK_ARG(l && n >= 0, "bad argument");
  ACME_HIP_TRY(hipDeviceSynchronize());
  ACME_HIP_TRY(hipMemcpy(&l->guard->applied, &n, sizeof(n), hipMemcpyHostToDevice));
  return ACME_OK;
}

const uint32_t* acme_r2d2_skip_word(const acme_r2d2* l) { return l ? &l->guard->last : nullptr; }

int64_t acme_r2d2_num_steps(const acme_r2d2* l) { return l ? l->num_steps : 0; }

int acme_r2d2_set_num_steps(acme_r2d2* l, int64_t n) {
  ACME_CHECK_ARG(l && n >= 0, "bad argument");
  l->num_steps = n;
  ACME_HIP_TRY(hipDeviceSynchronize());
  ACME_HIP_TRY(hipMemcpy(&l->guard->applied, &n, sizeof(n), hipMemcpyHostToDevice));
  return ACME_OK;
}

int acme_r2d2_debug_buffer(const acme_r2d2* l, const char* name, const float** out,
                           int64_t* count) {
  ACME_CHECK_ARG(l && name && out && count, "null argument");
  const int64_t B = l->cfg.max_batch, T = l->cfg.max_sequence_length;
  const int64_t RL = B * (T - l->cfg.burn_in_length);
  const std::string n(name);
  if (n == "q") { *out = l->q; *count = RL * l->A; }
  else if (n == "target_q") { *out = l->tq; *count = RL * l->A; }
  else if (n == "h") { *out = l->h; *count = B * T * l->H; }
  else if (n == "g") { *out = l->g; *count = RL; }
  else if (n == "hid") { *out = l->hid; *count = RL * 2 * l->H2; }
  else if (n == "x1" || n == "x2" || n == "x3") {
    float* x = n == "x1" ? l->x1 : (n == "x2" ? l->x2 : l->x3);
    const int64_t per = n == "x1" ? torso::kX1 : torso::kFlat;
    *out = x;
    *count = x ? B * T * per : 0;
    if (x && l->p3) {  // the plane path keeps them as planes: join the last step's
      const torso::Plane& pl = n == "x1" ? l->x1p : (n == "x2" ? l->x2p : l->x3p);
      ACME_HIP_TRY(hipDeviceSynchronize());
      const int rc = launch_join_planes(pl.p, pl.stride, l->last_rows * per, x, pl.sc, 0);
      if (rc != ACME_OK) return rc;
      ACME_HIP_TRY(hipDeviceSynchronize());
    }
  }
  else if (n == "lstm_trace") {  // u64 words: count is in floats
    *out = reinterpret_cast<const float*>(l->rg_trace);
    *count = l->rg_trace ? 2 * 8 * kMaxSeq : 0;
  }
  else if (n == "lstm_timeout_step") {  // u32: this step's timeout word (tests set it)
    *out = reinterpret_cast<const float*>(l->tmo);
    *count = l->tmo ? 1 : 0;
  }
  else if (n == "lstm_timeout") {  // u32: one-launch unroll timeouts so far (skipped steps)
    *out = reinterpret_cast<const float*>(l->tmo ? l->tmo + 1 : nullptr);
    *count = l->tmo ? 1 : 0;
  }
  else ACME_CHECK_ARG(false, "unknown debug buffer '%s'", name);
  return ACME_OK;
}

}  // extern "C"
