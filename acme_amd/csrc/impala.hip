// IMPALA learner step for MI355X: the replacement of IMPALALearner._step
// (acme/agents/tf/impala/learning.py:97-169) behind the C ABI (include/acme_hip.h).
//
// One call = the whole step on one stream, no host synchronisation.  Rows are the B*T
// frames of the batch in the dataset's batch-major order (row = b * T + t):
//   AtariTorso over all B*T frames (torso.h; the FLAT torso uses the observation)
//   OAR embedding x GEMM: gx = [feat | one_hot(prev a) | tanh(prev r)] @ W_i + b, the
//     embedding synthesised by the GEMM loader (never materialised)       (embedding.py)
//   T launches of the LSTM cell: gates = gx_t + h_{t-1} @ W_h, (i, f, g, o), c, h
//   head: relu(h @ W1 + b1) @ W_pv + b_pv -> logits [A], value              (atari.py:130-134)
//   loss kernel (one wave per sequence): log-rhos, V-trace backward scan,
//     pg / baseline / entropy losses and d loss / d(logits, value)        (learning.py:121-155)
//   backward: head GEMMs, T launches of LSTM BPTT, W_h / W_i(+b) weight GEMMs over all
//     rows, embedding dgrad masked by conv3's ReLU into the torso backward
//   clip_by_global_norm(max_gradient_norm) + Adam                         (learning.py:158-160)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "conv.h"
#include "conv_p3.h"
#include "gemm.h"
#include "gemm_direct.h"
#include "gemm_p3.h"
#include "gemm_x6.h"
#include "kernels.h"
#include "profiler.h"
#include "torso.h"
#include "lstm.h"

using namespace acme;
using namespace acme::conv;
using acme::gemm::launch_gemm;

namespace {

constexpr int kNormBlocks = 256;
constexpr int kOarSplits = 8;    // split-K of the Atari OAR projection (K = 7744 + A + 1)
constexpr int kOarSplitsP3 = 8;  // split-K of the plane-engine OAR projection (K = 7744)
constexpr int kP3MinRows = 64;   // learner steps of at least this many frames use the planes

struct Tensor {
  std::string name;
  int64_t offset = 0, numel = 0;
  int ndim = 0;
  int64_t shape[4] = {1, 1, 1, 1};
};

}  // namespace

struct acme_impala {
  acme_impala_config cfg;
  std::vector<Tensor> tensors;
  int64_t flat = 0;
  int F = 0, D = 0, H = 0, H2 = 0, A = 0;  // features, embedding, lstm, head, actions
  int t_c[6] = {-1, -1, -1, -1, -1, -1};   // torso w1 b1 w2 b2 w3 b3
  int t_wi = -1, t_wh = -1, t_b = -1, t_w1 = -1, t_b1 = -1, t_wpv = -1, t_bpv = -1;
  float *params = nullptr, *grads = nullptr, *m = nullptr, *v = nullptr;
  int64_t num_steps = 0;
  std::vector<void*> allocs;
  // workspace (rows = max_batch * max_sequence_length)
  float *x1 = nullptr, *x2 = nullptr, *x3 = nullptr, *dz1 = nullptr, *dz2 = nullptr,
        *dz3 = nullptr;
  float* slab = nullptr;
  float *gx = nullptr, *gates = nullptr, *h = nullptr, *c = nullptr, *hh = nullptr, *pv = nullptr;
  float *dpv = nullptr, *dhh = nullptr, *dh = nullptr, *dgates = nullptr, *dc = nullptr;
  float *vs = nullptr, *pg_adv = nullptr, *lrho = nullptr, *lpa = nullptr, *ent = nullptr;
  double* norm_part = nullptr;
  int64_t* dev_step = nullptr;
  float* metrics_tmp = nullptr;
  float* norms = nullptr;
  // Persistent LSTM unroll (H = 256, B <= 64): the forward's h_t granules [2][B * H] and the
  // backward's partial-product granules [2][16][B * H] (8 B: tag | value bits), zeroed before
  // every launch; the spin-timeout word.  lstm_steps: per-step launches instead (tests).
  unsigned long long* xg = nullptr;
  unsigned long long* xb = nullptr;
  unsigned* tmo = nullptr;
  bool lstm_steps = false;
  // Policy steps of an actor-side network on the plane engine (acme_impala_set_policy_planes):
  // the torso and W_i on f16 planes, the records rescaled after every call.
  bool policy_planes = false;
  unsigned lstm_epoch = 0;
  // Plane path of the Atari learner step (the DQN kernels: scaled two-plane f16 MFMA):
  // parameter planes of the torso + W_i prefix of the flat buffer, refreshed at the start
  // of every plane step; f16 frames; activation / gradient planes; its own split-K slab.
  bool p3_capable = false;
  int64_t p3_prefix = 0;  // floats of the flat buffer split into planes (torso + W_i)
  uint16_t* wpl = nullptr;
  uint16_t* frames = nullptr;
  torso::Plane x1p{}, x2p{}, x3p{}, dz1p{}, dz2p{}, dz3p{}, dgp{};
  // Scale records (gemm_p3.h PScale): the transient torso activations / gradients first
  // (rescaled at the end of every plane step), then the parameter and dgates planes (set
  // from their exact maxima by every split); sticky overflow flag.
  gemm::PScale* scales = nullptr;
  int* overflow = nullptr;
  bool scales_ok = false;
  float* pslab = nullptr;
  bool last_p3 = false;  // the last learner step ran the plane path (debug buffers join planes)
  int64_t last_rows = 0;
  // Step guard (kernels.h): a step whose planes overflowed or whose LSTM unroll timed out
  // (tmo[0]; tmo[1] counts them, tmo[2] is the policy step's own timeout word) applies no
  // update.  grad_sumsq folds the flags; clip_adam reads guard->last.
  StepGuard* guard = nullptr;
  int64_t* host_skipped = nullptr;
};

namespace {

int64_t align64(int64_t x) { return (x + 63) & ~int64_t(63); }

// Every record is transient (written and read within a step, rescaled at its end from the
// step's maxima): the activations, their gradients, dgates and the parameter planes (split
// from the f32 parameters at the start of each forward).
enum { kScX1, kScX2, kScX3, kScDz3, kScDz2, kScDz1, kScDgates, kScParams, kScTransient,
       kScCount = kScTransient };

int add_tensor(acme_impala* l, const std::string& name, std::initializer_list<int64_t> shape) {
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
int dev_alloc(acme_impala* l, T** p, int64_t count) {
  void* q = nullptr;
  if (hipMalloc(&q, std::max<int64_t>(count, 1) * sizeof(T)) != hipSuccess) {
    set_error("hipMalloc of %lld bytes failed", (long long)(count * sizeof(T)));
    return ACME_ERR_OOM;
  }
  l->allocs.push_back(q);
  *p = static_cast<T*>(q);
  return ACME_OK;
}

inline const float* P(const acme_impala* l, const float* base, int t) {
  return base + l->tensors[t].offset;
}
inline float* Pm(const acme_impala* l, float* base, int t) { return base + l->tensors[t].offset; }

// dW_h = h_prev^T dgates: h_prev of row m = b*T + t is h[m - 1] (t > 0) or h0[b] (t = 0).
struct HPrevWgrad {
  static constexpr int A_MODE = gemm::RCONTIG, B_MODE = gemm::RCONTIG;
  int M, N, K, k_chunk;  // M = H, N = 4H, K = rows
  const float* h;        // [rows][H]
  const float* h0;
  int64_t h0_stride;
  int T;
  const float* dz;
  float* out;
  struct ARow {
    int i;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int i) const { return ARow{i}; }
  __device__ f32x4 a_load(const ARow& a, int m) const {
    if (m >= K || a.i >= M) return gemm::zero4();
    const int t = m % T;
    const float* p = t == 0 ? h0 + (size_t)(m / T) * h0_stride : h + (size_t)(m - 1) * M;
    return *reinterpret_cast<const f32x4*>(p + a.i);
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ f32x4 b_load(const BRow& b, int m) const {
    if (b.n >= N || m >= K) return gemm::zero4();
    return load_row4<true>(dz + (size_t)m * N, b.n, N);
  }
  __device__ void store(int i, int n, float v, int) const { out[(size_t)i * N + n] = v; }
};

// ---------------------------------------------------------------- persistent unroll
// The whole T-step LSTM forward and BPTT in one launch each (lstm.h lstm_fwd_rg_kernel /
// lstm_bwd_rg_kernel, H = 256 here: 4 rows x 16 units per workgroup, up to 64 rows).
constexpr int kRgH = 256;                       // hidden size of the persistent kernels
constexpr int kRgGroups = RgShape<kRgH>::G;     // workgroups per row group
constexpr int kRgMaxB = 64;                     // 16 row groups x 16 = 256 workgroups

// The persistent unroll's shape: H = 256 and at most 64 rows (256 co-resident workgroups).
bool lstm_persistent(const acme_impala* l, int B) {
  return l->H == kRgH && B <= kRgMaxB && l->xb && !l->lstm_steps;
}
// Two rows per row group while the grid stays within 256 co-resident workgroups (up to 32
// rows): twice the workgroups, half the mat-vec and hand-off per workgroup.  At B = 16 the
// forward 56.0 -> 48.7 us, the BPTT 48.3 -> 39.1 us, the step 0.508 -> 0.488 ms against
// four rows (three alternating pairs, round 4; the same bits: each row's sums keep their
// order).
bool rg_pairs(const acme_impala*, int B) { return ceil_div(B, 2) * kRgGroups <= 256; }
// One row per row group up to 16 rows (16 x 16 workgroups at the learner's B = 16):
// forward 48.5 -> 36.5 us, BPTT 39.5 -> 31.2 us, the step 0.491 -> 0.473 ms against two
// rows (three alternating pairs, round 4; scalar FMAs, the same per-row order and bits).
bool rg_single(const acme_impala*, int B) { return B * kRgGroups <= 256; }

// The granule tags of the next persistent launch: tag0 + t, tag0 = 128 x a per-learner launch
// count, so no launch can match a granule an earlier one left (the buffers are never cleared
// between launches); the buffers are cleared once the count wraps.
unsigned next_lstm_tags(acme_impala* l, hipStream_t st) {
  if (++l->lstm_epoch >= (1u << 24)) {
    l->lstm_epoch = 1;
    (void)hipMemsetAsync(l->xg, 0, (size_t)2 * l->cfg.max_batch * l->H * 8, st);
    (void)hipMemsetAsync(l->xb, 0, (size_t)2 * kRgGroups * l->cfg.max_batch * l->H * 8, st);
  }
  return l->lstm_epoch << 7;
}

// ------------------------------------------------------------------ loss
// Three launches over the B*T rows (row = b * T + t, t < T-1 carry the losses):
//   rowstats (one wave per row, lane = action): log pi, log mu -> log rho, log pi(a),
//     entropy H(pi)
//   vtrace (one thread per sequence): trfl.vtrace_from_importance_weights backward scan
//     (rho_bar = c_bar = 1) -> vs, pg advantages; the four logged means
//   grads (one wave per row): d loss / d logits = (-(onehot - pi) adv + c_e pi (log pi
//     + H)) / N, d loss / d value = -2 c_b (vs - v) / N; zero at t = T-1
struct LossArgs {
  const float* pv;  // [rows][A + 1]
  const int32_t* action;
  const float *reward, *discount, *mu;
  int B, T, A;
  float gamma, entropy_cost, baseline_cost, max_abs_reward;
  float* lrho;   // [rows] scratch
  float* lpa;    // [rows]
  float* ent;    // [rows]
  float* dpv;
  float *vs, *pg_adv;  // [(T-1) * B] time-major
  float* metrics;      // [4]
  const unsigned* lstm_timeout;  // sticky: a persistent LSTM launch timed out (logs NaN)
};

__global__ void __launch_bounds__(256) impala_rowstats_kernel(const LossArgs a) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.B * a.T || row % a.T == a.T - 1) return;
  const int A = a.A, W = A + 1;
  const bool on = lane < A;
  const float l = on ? a.pv[(size_t)row * W + lane] : -INFINITY;
  const float m = wave_max(l);
  const float e = on ? expf(l - m) : 0.f;
  const float s = wave_sum(e);
  const float logp = l - m - logf(s);
  const float mu = on ? a.mu[(size_t)row * A + lane] : -INFINITY;
  const float mm = wave_max(mu);
  const float me = on ? expf(mu - mm) : 0.f;
  const float logmu = mu - mm - logf(wave_sum(me));
  const int act = a.action[row];
  const float lpa = __shfl(logp, act, 64), lma = __shfl(logmu, act, 64);
  const float ent = -wave_sum(on ? (e / s) * logp : 0.f);
  if (lane == 0) {
    a.lrho[row] = lpa - lma;
    a.lpa[row] = lpa;
    a.ent[row] = ent;
  }
}

// The scan's inputs (value, reward, discount, log rho, log pi(a), entropy per row) are
// loaded by the whole block into LDS first, every load in one round, when they fit
// (kVtraceLdsRows); otherwise read from global memory inside the scan.  Threads 0..63 then
// scan: thread b takes sequences b, b + 64, ...  Same arithmetic either way.  (Loads inside the
// scan were ~19 dependent round trips per thread: 12.6 us.)
constexpr int kVtraceLdsRows = 2048;  // 6 x 4 B x rows of LDS

template <bool LDS>
__device__ __forceinline__ void vtrace_scan(const LossArgs& a, const float* sv, const float* sr,
                                            const float* sd, const float* sl, const float* sp,
                                            const float* se) {
  __shared__ float red[64][3];
  const int b = threadIdx.x;
  const int T = a.T, W = a.A + 1;
  auto V = [&](size_t row) { return LDS ? sv[row] : a.pv[row * W + a.A]; };
  auto R = [&](size_t row) { return LDS ? sr[row] : a.reward[row]; };
  auto D = [&](size_t row) { return LDS ? sd[row] : a.discount[row]; };
  auto LR = [&](size_t row) { return LDS ? sl[row] : a.lrho[row]; };
  auto LP = [&](size_t row) { return LDS ? sp[row] : a.lpa[row]; };
  auto EN = [&](size_t row) { return LDS ? se[row] : a.ent[row]; };
  float s_pg = 0.f, s_cr = 0.f, s_en = 0.f;
  for (int bb = b; b < 64 && bb < a.B; bb += 64) {
    const size_t base = (size_t)bb * T;
    const float boot = V(base + T - 1);
    float acc = 0.f, vs_next = boot, v1 = boot;
    for (int t = T - 2; t >= 0; --t) {
      const size_t row = base + t;
      const float v = V(row);
      float r = R(row);
      r = fminf(fmaxf(r, -a.max_abs_reward), a.max_abs_reward);
      const float g = a.gamma * D(row);
      const float cr = fminf(1.f, expf(LR(row)));
      acc = cr * (r + g * v1 - v) + g * cr * acc;
      const float vs = acc + v;
      const float adv = cr * (r + g * vs_next - v);
      a.vs[(size_t)t * a.B + bb] = vs;
      a.pg_adv[(size_t)t * a.B + bb] = adv;
      s_pg += -LP(row) * adv;
      s_cr += (vs - v) * (vs - v);
      s_en += -EN(row);
      vs_next = vs;
      v1 = v;
    }
  }
  if (b < 64) {
    red[b][0] = s_pg;
    red[b][1] = s_cr;
    red[b][2] = s_en;
  }
  __syncthreads();
  if (b == 0) {
    float pg = 0.f, cr = 0.f, en = 0.f;
    for (int i = 0; i < 64; ++i) {
      pg += red[i][0];
      cr += red[i][1];
      en += red[i][2];
    }
    const float invN = 1.f / (float)((T - 1) * a.B);
    pg *= invN;
    cr *= invN;
    en *= invN;
    const float bad = a.lstm_timeout && *a.lstm_timeout ? NAN : 0.f;
    a.metrics[0] = pg + a.baseline_cost * cr + a.entropy_cost * en + bad;
    a.metrics[1] = cr + bad;
    a.metrics[2] = en + bad;
    a.metrics[3] = pg + bad;
  }
}

__global__ void __launch_bounds__(256) impala_vtrace_kernel(const LossArgs a) {
  extern __shared__ float sh[];  // [6][rows] when rows <= kVtraceLdsRows
  const int rows = a.B * a.T, W = a.A + 1;
  if (rows <= kVtraceLdsRows) {
    float *sv = sh, *sr = sh + rows, *sd = sr + rows, *sl = sd + rows, *sp = sl + rows,
          *se = sp + rows;
    for (int i = threadIdx.x; i < rows; i += blockDim.x) {
      const float v = a.pv[(size_t)i * W + a.A], r = a.reward[i], d = a.discount[i];
      const float lr = a.lrho[i], lp = a.lpa[i], en = a.ent[i];
      sv[i] = v; sr[i] = r; sd[i] = d; sl[i] = lr; sp[i] = lp; se[i] = en;
    }
    __syncthreads();
    vtrace_scan<true>(a, sv, sr, sd, sl, sp, se);
  } else {
    vtrace_scan<false>(a, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
  }
}

__global__ void __launch_bounds__(256) impala_loss_grad_kernel(const LossArgs a) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.B * a.T) return;
  const int A = a.A, W = A + 1, T = a.T;
  const int b = row / T, t = row - b * T;
  if (t == T - 1) {
    if (lane < W) a.dpv[(size_t)row * W + lane] = 0.f;
    return;
  }
  const float invN = 1.f / (float)((T - 1) * a.B);
  const bool on = lane < A;
  const float l = on ? a.pv[(size_t)row * W + lane] : -INFINITY;
  const float m = wave_max(l);
  const float e = on ? expf(l - m) : 0.f;
  const float s = wave_sum(e);
  const float logp = l - m - logf(s);
  const float pi = e / s;
  const float adv = a.pg_adv[(size_t)t * a.B + b], vs = a.vs[(size_t)t * a.B + b];
  const float ent = a.ent[row];
  if (on) {
    const float oh = lane == a.action[row] ? 1.f : 0.f;
    a.dpv[(size_t)row * W + lane] = (-(oh - pi) * adv + a.entropy_cost * pi * (logp + ent)) * invN;
  }
  if (lane == A) {
    const float v = a.pv[(size_t)row * W + A];
    a.dpv[(size_t)row * W + A] = a.baseline_cost * (-2.f) * (vs - v) * invN;
  }
}

// ------------------------------------------------------------------ orchestration

#define IM_GEMM(name, BM, BN, WM, WN, WK, prob, splits)                                         \
  do {                                                                                         \
    ACME_PROF_PEAK(name, st, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, 0.0,  \
                   (gemm::matmul_peak_tflops<WK, decltype(prob)>()));                             \
    hipError_t _e = gemm::launch_matmul<BM, BN, WM, WN, 16, WK>(prob, splits, st);              \
    if (_e != hipSuccess) {                                                                    \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__);  \
      return ACME_ERR_HIP;                                                                     \
    }                                                                                          \
  } while (0)

// The small f32 layers after the LSTM (a few hundred rows): the register-operand engine
// (gemm_direct.h: each lane's k run in one burst, 8 waves per 32 x 32 tile; round 5: faster
// than the staged f32 engine, profiles/r05/ab/impala_direct_small_layers.log).
#define IM_DGEMM(name, prob)                                                                   \
  do {                                                                                         \
    ACME_PROF_PEAK(name, st, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, 0.0,  \
                   157.3);                                                                     \
    hipError_t _e = gemm::launch_direct(prob, 1, (prob).K, st);                                \
    if (_e != hipSuccess) {                                                                    \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__);  \
      return ACME_ERR_HIP;                                                                     \
    }                                                                                          \
  } while (0)

#define IM_CHECK()                                                                             \
  do {                                                                                         \
    hipError_t _e = hipGetLastError();                                                         \
    if (_e != hipSuccess) {                                                                    \
      set_error("kernel launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                     \
    }                                                                                          \
  } while (0)

inline int chunk_for(int K, int splits) {
  int c = (int)ceil_div(K, splits);
  return (int)ceil_div(c, 32) * 32;
}

bool atari(const acme_impala* l) { return l->cfg.torso == ACME_IMPALA_TORSO_ATARI; }

// ---- plane path helpers
#define IM_P3_GEMM(name, BM, BN, WM, WN, BKV, prob, splits)                                    \
  do {                                                                                         \
    ACME_PROF_PEAK(name, st, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, 0.0, \
                   gemm::p3_peak_tflops<decltype(prob)>());                                    \
    hipError_t _e = gemm::launch_gemm_p3<BM, BN, WM, WN, BKV>(prob, splits, st);              \
    if (_e != hipSuccess) {                                                                    \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                     \
    }                                                                                          \
  } while (0)
#define IM_P3WS_GEMM(name, BM, BN, WM, WN, BKV, prob, splits)                                  \
  do {                                                                                         \
    ACME_PROF_PEAK(name, st, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, 0.0, \
                   gemm::p3_peak_tflops<decltype(prob)>());                                    \
    hipError_t _e = gemm::launch_gemm_p3ws<BM, BN, WM, WN, BKV, true>(prob, splits, st);      \
    if (_e != hipSuccess) {                                                                    \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                     \
    }                                                                                          \
  } while (0)

// Plane view of parameter tensor t in the [2][flat] parameter planes.
torso::Plane WP(const acme_impala* l, int t) {
  return torso::Plane{l->wpl + l->tensors[t].offset, l->flat, l->scales + kScParams};
}
gemm::PlaneSrc SRC(const torso::Plane& x, int64_t elems) {
  return gemm::PlaneSrc{x.p, x.stride, (int32_t)(2 * elems), x.sc};
}
torso::PWeights torso_pw(const acme_impala* l) {
  return torso::PWeights{WP(l, l->t_c[0]), WP(l, l->t_c[2]), WP(l, l->t_c[4]),
                         P(l, l->params, l->t_c[1]), P(l, l->params, l->t_c[3]),
                         P(l, l->params, l->t_c[5])};
}
// The plane path runs the learner steps of the Atari torso with enough frames to fill the
// GEMMs (ACME_V_IMP3=1 at creation: the f32 engine throughout, for tests).
bool use_p3(const acme_impala* l, int rows) { return l->p3_capable && rows >= kP3MinRows; }

torso::Weights torso_w(const acme_impala* l) {
  return torso::Weights{P(l, l->params, l->t_c[0]), P(l, l->params, l->t_c[1]),
                        P(l, l->params, l->t_c[2]), P(l, l->params, l->t_c[3]),
                        P(l, l->params, l->t_c[4]), P(l, l->params, l->t_c[5])};
}

// Network forward over rows = B*T frames: features, OAR projection, T LSTM steps, head.
int network_forward(acme_impala* l, const void* obs, const int32_t* prev_a, const float* prev_r,
                    const float* h0, const float* c0, int64_t state_stride, int B, int T,
                    hipStream_t st, bool p3, unsigned* tmo) {
  const int rows = B * T, H = l->H, A = l->A;
  const float* feat;
  if (p3) {
    // Parameter planes of the torso + W_i (the only plane operands), the f16 frames,
    // the plane torso, then feat @ W_i[0:F] on the plane engine and the embedding tail.
    int rc;
    {
      ACME_PROF("impala_planes", st, 0.0, 8.0 * (double)l->p3_prefix);
      rc = launch_split_planes_lagged(l->params, l->p3_prefix, l->wpl, l->flat,
                                      l->scales + kScParams, st);
      if (rc != ACME_OK) return rc;
    }
    {
      ACME_PROF("impala_frames_f16", st, 0.0, 3.0 * (double)rows * torso::kObsBytes);
      rc = launch_frames_f16(static_cast<const uint8_t*>(obs), static_cast<const uint8_t*>(obs),
                              rows, rows, torso::kObsBytes, l->frames, st);
      if (rc != ACME_OK) return rc;
    }
    rc = torso::forward_p3(torso_pw(l), torso::Frames{l->frames}, rows,
                           torso::PActs{l->x1p, l->x2p, l->x3p}, st);
    if (rc != ACME_OK) return rc;
    const int F = l->F, N = 4 * H;
    P3DenseFwd p;
    p.M = rows; p.N = N; p.K = F; p.k_chunk = chunk_for(F, kOarSplitsP3);
    p.a_src = SRC(l->x3p, (int64_t)rows * F); p.ldx = F;
    p.b_src = SRC(WP(l, l->t_wi), (int64_t)F * N); p.slab = l->pslab;
    IM_P3WS_GEMM("impala_oar_fwd", 128, 128, 2, 2, 32, p, kOarSplitsP3);
    {
      ACME_PROF("impala_oar_reduce", st, 0.0, 4.0 * (kOarSplitsP3 + 1) * (double)rows * N);
      const int64_t n4 = (int64_t)rows * N / 4;
      oar_finish_kernel<<<(unsigned)ceil_div(n4, 256), 256, 0, st>>>(
          l->pslab, kOarSplitsP3, rows, N, P(l, l->params, l->t_wi) + (size_t)F * N,
          P(l, l->params, l->t_b), prev_a, prev_r, A, l->gx);
      IM_CHECK();
    }
  } else if (atari(l)) {
    int rc = torso::forward(torso_w(l), true, obs, obs, rows, rows,
                            torso::Acts{l->x1, l->x2, l->x3}, st);
    if (rc != ACME_OK) return rc;
    feat = l->x3;
  } else {
    feat = static_cast<const float*>(obs);
  }
  if (!p3) {
    OarFwd p;
    p.M = rows; p.N = 4 * H; p.K = l->D;
    p.x = Oar{feat, l->F, A, prev_a, prev_r};
    p.w = P(l, l->params, l->t_wi); p.bias = P(l, l->params, l->t_b); p.y = l->gx;
    if (atari(l)) {
      p.k_chunk = chunk_for(p.K, kOarSplits);
      p.slab = l->slab;
      IM_GEMM("impala_oar_fwd", 64, 64, 2, 2, 1, p, kOarSplits);
      ACME_PROF("impala_oar_reduce", st, 0.0, 4.0 * (kOarSplits + 1) * (double)rows * 4 * H);
      int rc = launch_slab_reduce(l->slab, kOarSplits, (int64_t)rows * 4 * H, l->gx,
                                  (int64_t)rows * 4 * H, nullptr, P(l, l->params, l->t_b), 4 * H,
                                  0, st);
      if (rc != ACME_OK) return rc;
    } else {
      p.k_chunk = p.K;
      p.slab = nullptr;
      IM_GEMM("impala_oar_fwd", 32, 32, 1, 1, 8, p, 1);
    }
  }
  {
    ACME_PROF("impala_lstm_fwd", st, 2.0 * rows * (double)H * 4 * H, 0.0);
    const size_t smem = lstm_fwd_smem(B, H);
    if (lstm_persistent(l, B)) {  // one launch for the whole unroll (lstm_fwd_rg_kernel)
      const unsigned tag0 = next_lstm_tags(l, st);
      if (rg_single(l, B))
        lstm_fwd_rg_kernel<kRgH, 1><<<(unsigned)(B * kRgGroups), 256, 0, st>>>(
            l->gx, P(l, l->params, l->t_wh), h0, state_stride, c0, state_stride, B, T, T, 1,
            l->gates, l->h, l->c, l->xg, tag0, tmo);
      else if (rg_pairs(l, B))
        lstm_fwd_rg_kernel<kRgH, 2><<<(unsigned)(ceil_div(B, 2) * kRgGroups), 256, 0, st>>>(
            l->gx, P(l, l->params, l->t_wh), h0, state_stride, c0, state_stride, B, T, T, 1,
            l->gates, l->h, l->c, l->xg, tag0, tmo);
      else
        lstm_fwd_rg_kernel<kRgH, 4><<<(unsigned)(ceil_div(B, 4) * kRgGroups), 256, 0, st>>>(
            l->gx, P(l, l->params, l->t_wh), h0, state_stride, c0, state_stride, B, T, T, 1,
            l->gates, l->h, l->c, l->xg, tag0, tmo);
      IM_CHECK();
    } else
    for (int t = 0; t < T; ++t) {
      const float* hp = t == 0 ? h0 : l->h + (size_t)(t - 1) * H;
      const float* cp = t == 0 ? c0 : l->c + (size_t)(t - 1) * H;
      const int64_t hs = t == 0 ? state_stride : (int64_t)T * H;
      lstm_fwd_step_kernel<<<H / kFwdUnits, 256, smem, st>>>(l->gx, P(l, l->params, l->t_wh), hp, hs,
                                                          cp, hs, B, T, 1, t, H, l->gates, l->h,
                                                          l->c, B);
      IM_CHECK();
    }
  }
  {
    DenseFwd<true> p;
    p.M = rows; p.N = l->H2; p.K = H; p.k_chunk = H;
    p.x = l->h; p.x2 = l->h; p.split_b = rows; p.ldx = H;
    p.w = P(l, l->params, l->t_w1); p.bias = P(l, l->params, l->t_b1); p.y = l->hh;
    p.act = ACT_RELU; p.slab = nullptr;
    IM_DGEMM("impala_head_fwd", p);
  }
  {
    DenseFwd<false> p;
    p.M = rows; p.N = A + 1; p.K = l->H2; p.k_chunk = l->H2;
    p.x = l->hh; p.x2 = l->hh; p.split_b = rows; p.ldx = l->H2;
    p.w = P(l, l->params, l->t_wpv); p.bias = P(l, l->params, l->t_bpv); p.y = l->pv;
    p.act = ACT_NONE; p.slab = nullptr;
    IM_DGEMM("impala_pv_fwd", p);
  }
  return ACME_OK;
}

// apply = false: the forward, loss and backward only (the plane-scale calibration passes).
int impala_step_impl(acme_impala* l, const acme_sequence_batch* bt, float* metrics,
                     hipStream_t st, bool apply = true) {
  const int B = (int)bt->batch, T = (int)bt->sequence_length, rows = B * T;
  const int H = l->H, A = l->A;
  const bool p3 = atari(l) && use_p3(l, rows);
  l->last_p3 = p3;
  l->last_rows = rows;
  int rc = network_forward(l, bt->observation, bt->prev_action, bt->prev_reward, bt->h0, bt->c0,
                           bt->state_stride, B, T, st, p3, l->tmo);
  if (rc != ACME_OK) return rc;
  {
    ACME_PROF("impala_loss", st, 0.0, 0.0);
    LossArgs a;
    a.pv = l->pv; a.action = bt->action; a.reward = bt->reward; a.discount = bt->discount;
    a.mu = bt->behaviour_logits; a.B = B; a.T = T; a.A = A;
    a.gamma = l->cfg.discount; a.entropy_cost = l->cfg.entropy_cost;
    a.baseline_cost = l->cfg.baseline_cost; a.max_abs_reward = l->cfg.max_abs_reward;
    a.dpv = l->dpv; a.vs = l->vs; a.pg_adv = l->pg_adv;
    a.lrho = l->lrho; a.lpa = l->lpa; a.ent = l->ent;
    a.metrics = metrics ? metrics : l->metrics_tmp;
    a.lstm_timeout = l->tmo;
    const unsigned rb = (unsigned)ceil_div(rows, 4);
    impala_rowstats_kernel<<<rb, 256, 0, st>>>(a);
    IM_CHECK();
    const int vrows = B * T;
    impala_vtrace_kernel<<<1, 256, vrows <= kVtraceLdsRows ? 6 * sizeof(float) * vrows : 0,
                           st>>>(a);
    IM_CHECK();
    impala_loss_grad_kernel<<<rb, 256, 0, st>>>(a);
    IM_CHECK();
  }
  float* gr = l->grads;
  {  // policy/value head
    DenseWgrad<false> w;
    w.M = l->H2; w.N = A + 1; w.K = rows; w.k_chunk = rows;
    w.x = l->hh; w.ldx = l->H2; w.dz = l->dpv; w.out = Pm(l, gr, l->t_wpv);
    w.bias_out = Pm(l, gr, l->t_bpv);
    IM_DGEMM("impala_pv_wgrad", w);
    DenseDgrad<false> d;
    d.M = rows; d.N = l->H2; d.K = A + 1; d.k_chunk = A + 1;
    d.dz = l->dpv; d.w = P(l, l->params, l->t_wpv); d.xprev = l->hh; d.ldx = l->H2; d.dx = l->dhh;
    d.act = ACT_RELU;
    IM_DGEMM("impala_pv_dgrad", d);
  }
  {  // Linear(256) after the LSTM
    DenseWgrad<true> w;
    w.M = H; w.N = l->H2; w.K = rows; w.k_chunk = rows;
    w.x = l->h; w.ldx = H; w.dz = l->dhh; w.out = Pm(l, gr, l->t_w1); w.bias_out = Pm(l, gr, l->t_b1);
    IM_DGEMM("impala_head_wgrad", w);
    DenseDgrad<true> d;
    d.M = rows; d.N = H; d.K = l->H2; d.k_chunk = l->H2;
    d.dz = l->dhh; d.w = P(l, l->params, l->t_w1); d.xprev = nullptr; d.ldx = H; d.dx = l->dh;
    IM_DGEMM("impala_head_dgrad", d);
  }
  {  // BPTT
    ACME_PROF("impala_lstm_bwd", st, 2.0 * rows * (double)H * 4 * H, 0.0);
    if (lstm_persistent(l, B)) {  // one launch for the whole BPTT (lstm_bwd_rg_kernel)
      const unsigned tag0 = next_lstm_tags(l, st);
      if (rg_single(l, B))
        lstm_bwd_rg_kernel<kRgH, 1><<<(unsigned)(B * kRgGroups), 256, 0, st>>>(
            l->dh, P(l, l->params, l->t_wh), l->gates, l->c, bt->c0, bt->state_stride, B, T, 0,
            T, 1, l->dgates, l->xb, tag0, l->tmo);
      else if (rg_pairs(l, B))
        lstm_bwd_rg_kernel<kRgH, 2><<<(unsigned)(ceil_div(B, 2) * kRgGroups), 256, 0, st>>>(
            l->dh, P(l, l->params, l->t_wh), l->gates, l->c, bt->c0, bt->state_stride, B, T, 0,
            T, 1, l->dgates, l->xb, tag0, l->tmo);
      else
        lstm_bwd_rg_kernel<kRgH, 4><<<(unsigned)(ceil_div(B, 4) * kRgGroups), 256, 0, st>>>(
            l->dh, P(l, l->params, l->t_wh), l->gates, l->c, bt->c0, bt->state_stride, B, T, 0,
            T, 1, l->dgates, l->xb, tag0, l->tmo);
      IM_CHECK();
    } else {
    ACME_HIP_TRY(hipMemsetAsync(l->dc, 0, (size_t)B * H * sizeof(float), st));
    for (int t = T - 1; t >= 0; --t) {
      lstm_bwd_step_kernel<<<H / kUnits, 256, 0, st>>>(l->dh, P(l, l->params, l->t_wh), l->gates,
                                                       l->c, bt->c0, bt->state_stride, l->dc,
                                                       l->dgates, B, T, t, H, T, 1);
      IM_CHECK();
    }
    }
  }
  {  // LSTM weights: W_h over h_prev, W_i (+ b via colsum) over the OAR embedding
    HPrevWgrad w;
    w.M = H; w.N = 4 * H; w.K = rows; w.k_chunk = rows;
    w.h = l->h; w.h0 = bt->h0; w.h0_stride = bt->state_stride; w.T = T; w.dz = l->dgates;
    w.out = Pm(l, gr, l->t_wh);
    IM_GEMM("impala_wh_wgrad", 32, 32, 1, 1, 8, w, 1);
  }
  if (p3) {  // W_i, b and the embedding gradient on the plane engine, then the plane torso
    const int F = l->F, N = 4 * H;
    {
      ACME_PROF("impala_dgates_planes", st, 0.0, 8.0 * (double)rows * N);
      rc = launch_split_planes_lagged(l->dgates, (int64_t)rows * N, l->dgp.p, l->dgp.stride,
                                      l->dgp.sc, st);
      if (rc != ACME_OK) return rc;
    }
    {
      P3DenseWgrad p;
      p.M = F; p.N = N; p.K = rows; p.k_chunk = rows;
      p.a_src = SRC(l->x3p, (int64_t)rows * F); p.ldx = F;
      p.b_src = SRC(l->dgp, (int64_t)rows * N); p.out = Pm(l, gr, l->t_wi);
      p.bias_out = Pm(l, gr, l->t_b);
      // (256x128 warp-specialised tiles: 24.7 -> 26.6 us, round 4.)
      IM_P3_GEMM("impala_wi_wgrad", 128, 128, 2, 2, 16, p, 1);
    }
    {
      ACME_PROF("impala_wi_wgrad_tail", st, 0.0, 4.0 * (double)rows * N);
      const int tw = tail_waves(A);
      oar_wgrad_tail_kernel<<<(unsigned)ceil_div(N, 64), 64 * tw,
                              (size_t)tw * (A + 1) * 64 * sizeof(float), st>>>(
          l->dgates, rows, N, bt->prev_action, bt->prev_reward, A,
          Pm(l, gr, l->t_wi) + (size_t)F * N);
      IM_CHECK();
    }
    {
      P3DenseDgrad p;
      p.M = rows; p.N = F; p.K = N; p.k_chunk = N;
      p.a_src = SRC(l->dgp, (int64_t)rows * N);
      p.b_src = SRC(WP(l, l->t_wi), (int64_t)F * N);
      p.xprev = CPlanes{l->x3p.p, l->x3p.stride, l->x3p.sc}; p.ldx = F;
      p.dx = Planes{l->dz3p.p, l->dz3p.stride, l->dz3p.sc};
      IM_P3WS_GEMM("impala_feat_dgrad", 128, 128, 2, 2, 32, p, 1);
    }
    torso::Grads g{Pm(l, gr, l->t_c[0]), Pm(l, gr, l->t_c[1]), Pm(l, gr, l->t_c[2]),
                   Pm(l, gr, l->t_c[3]), Pm(l, gr, l->t_c[4]), Pm(l, gr, l->t_c[5])};
    rc = torso::backward_p3(torso_pw(l), g, torso::Frames{l->frames}, rows,
                            torso::PActs{l->x1p, l->x2p, l->x3p}, l->dz3p, l->dz2p, l->dz1p,
                            l->pslab, st);
    if (rc != ACME_OK) return rc;
    // The next plane step's activation / gradient scales from this step's maxima.
    RescaleGuard rg;  // an overflowed or underflowed record skips the step (grad_sumsq)
    rg.g = l->guard;
    rg.mode = kRgFlag;
    rc = launch_plane_rescale(l->scales, kScTransient, kScTransient, -1, -1, l->overflow, st, -1,
                              -1, rg);
    if (rc != ACME_OK) return rc;
  } else {
    const float* feat = atari(l) ? l->x3 : static_cast<const float*>(bt->observation);
    OarWgrad o;
    o.M = l->D; o.N = 4 * H; o.K = rows; o.k_chunk = rows;
    o.x = Oar{feat, l->F, A, bt->prev_action, bt->prev_reward};
    o.dz = l->dgates; o.out = Pm(l, gr, l->t_wi); o.bias_out = Pm(l, gr, l->t_b);
    if (atari(l)) IM_GEMM("impala_wi_wgrad", 128, 128, 2, 2, 1, o, 1);
    else IM_GEMM("impala_wi_wgrad", 32, 32, 1, 1, 8, o, 1);
  }
  if (!p3 && atari(l)) {  // embedding features -> conv3 dZ -> torso backward
    DenseDgrad<true> d;
    d.M = rows; d.N = l->F; d.K = 4 * H; d.k_chunk = 4 * H;
    d.dz = l->dgates; d.w = P(l, l->params, l->t_wi); d.xprev = l->x3; d.ldx = l->F;
    d.dx = l->dz3; d.act = ACT_RELU;
    IM_GEMM("impala_feat_dgrad", 64, 128, 2, 2, 1, d, 1);
    torso::Grads g{Pm(l, gr, l->t_c[0]), Pm(l, gr, l->t_c[1]), Pm(l, gr, l->t_c[2]),
                   Pm(l, gr, l->t_c[3]), Pm(l, gr, l->t_c[4]), Pm(l, gr, l->t_c[5])};
    rc = torso::backward(torso_w(l), g, true, bt->observation, rows,
                         torso::Acts{l->x1, l->x2, l->x3}, l->dz3, l->dz2, l->dz1, l->slab, st);
    if (rc != ACME_OK) return rc;
  }
  if (!apply) return ACME_OK;
  {
    ACME_PROF("impala_adam", st, 0.0, 7.0 * 4.0 * (double)l->flat);
    const int64_t n4 = l->flat / 4;
    rc = launch_grad_sumsq(gr, n4, n4, l->norm_part, kNormBlocks, l->dev_step, st, l->guard,
                           l->tmo, l->host_skipped);
    if (rc != ACME_OK) return rc;
    ClipAdamArgs a;
    a.p = l->params; a.m = l->m; a.v = l->v; a.g = gr; a.n4 = n4; a.group0_4 = n4;
    a.part = l->norm_part; a.nparts = kNormBlocks; a.clipping = 1;
    a.clip_norm = l->cfg.max_gradient_norm;
    a.optix = l->cfg.semantics == ACME_SEMANTICS_JAX;
    a.lr0 = a.lr1 = l->cfg.learning_rate;
    a.b1 = l->cfg.adam_beta1; a.b2 = l->cfg.adam_beta2; a.eps = l->cfg.adam_epsilon;
    a.dev_step = l->dev_step; a.norms = l->norms;
    a.gate.g = l->guard;
    a.gate.use_last = 1;
    rc = launch_clip_adam(a, st);
    if (rc != ACME_OK) return rc;
  }
  return ACME_OK;
}

}  // namespace

extern "C" {

int acme_impala_destroy(acme_impala* l) {
  if (!l) return ACME_OK;
  // Work of this learner may still be queued on a caller's stream (an actor network dropped
  // right after its last step): drain it before the buffers go.
  (void)hipDeviceSynchronize();
  for (void* p : l->allocs) (void)hipFree(p);
  if (l->host_skipped) (void)hipHostFree(l->host_skipped);
  delete l;
  return ACME_OK;
}

int acme_impala_create(const acme_impala_config* cfg, acme_impala** out) {
  ACME_CHECK_ARG(cfg && out, "null argument");
  ACME_CHECK_ARG(cfg->torso == ACME_IMPALA_TORSO_ATARI || cfg->torso == ACME_IMPALA_TORSO_FLAT,
                 "unknown torso %d", cfg->torso);
  ACME_CHECK_ARG(cfg->torso == ACME_IMPALA_TORSO_ATARI || cfg->obs_dim >= 1,
                 "obs_dim must be >= 1 for the flat torso");
  ACME_CHECK_ARG(cfg->num_actions >= 1 && cfg->num_actions <= 63, "num_actions must be in [1, 63]");
  ACME_CHECK_ARG(cfg->semantics == ACME_SEMANTICS_TF || cfg->semantics == ACME_SEMANTICS_JAX,
                 "unknown learner semantics %d", cfg->semantics);
  ACME_CHECK_ARG(cfg->max_batch >= 1 && cfg->max_batch <= 1024, "max_batch must be in [1, 1024]");
  ACME_CHECK_ARG(cfg->max_sequence_length >= 2 && cfg->max_sequence_length <= 64,
                 "max_sequence_length must be in [2, 64]");
  ACME_CHECK_ARG(cfg->lstm_size >= 8 && cfg->lstm_size % 8 == 0,
                 "lstm_size must be a positive multiple of 8");
  // The per-step forward stages h_prev of every row in LDS; the one-launch unroll (lstm_size
  // 256, at most 64 sequences) does not.
  ACME_CHECK_ARG(lstm_fwd_smem(cfg->max_batch, cfg->lstm_size) <= 65536 ||
                     (cfg->lstm_size == kRgH && cfg->max_batch <= kRgMaxB),
                 "max_batch * lstm_size + 16 * lstm_size must stay within 64 KB of LDS");
  ACME_CHECK_ARG(cfg->head_size >= 4 && cfg->head_size % 4 == 0,
                 "head_size must be a positive multiple of 4");
  acme_impala* l = new acme_impala();
  l->cfg = *cfg;
  auto fail = [&](int code) {
    acme_impala_destroy(l);
    return code;
  };
  l->A = cfg->num_actions;
  l->H = cfg->lstm_size;
  l->H2 = cfg->head_size;
  l->F = cfg->torso == ACME_IMPALA_TORSO_ATARI ? torso::kFlat : cfg->obs_dim;
  l->D = l->F + l->A + 1;
  const std::string pre = "impala_atari_network/";
  if (cfg->torso == ACME_IMPALA_TORSO_ATARI) {
    l->t_c[0] = add_tensor(l, pre + "atari_torso/conv2_d/w", {8, 8, 4, 32});
    l->t_c[1] = add_tensor(l, pre + "atari_torso/conv2_d/b", {32});
    l->t_c[2] = add_tensor(l, pre + "atari_torso/conv2_d_1/w", {4, 4, 32, 64});
    l->t_c[3] = add_tensor(l, pre + "atari_torso/conv2_d_1/b", {64});
    l->t_c[4] = add_tensor(l, pre + "atari_torso/conv2_d_2/w", {3, 3, 64, 64});
    l->t_c[5] = add_tensor(l, pre + "atari_torso/conv2_d_2/b", {64});
  }
  const int H = l->H, A = l->A, H2 = l->H2;
  l->t_wi = add_tensor(l, pre + "lstm/w_i", {l->D, 4 * H});
  l->t_wh = add_tensor(l, pre + "lstm/w_h", {H, 4 * H});
  l->t_b = add_tensor(l, pre + "lstm/b", {4 * H});
  l->t_w1 = add_tensor(l, pre + "linear/w", {H, H2});
  l->t_b1 = add_tensor(l, pre + "linear/b", {H2});
  l->t_wpv = add_tensor(l, pre + "policy_value/w", {H2, A + 1});
  l->t_bpv = add_tensor(l, pre + "policy_value/b", {A + 1});
  const int64_t R = (int64_t)cfg->max_batch * cfg->max_sequence_length;
  const int B = cfg->max_batch;
  int rc;
  int64_t slab = 1;
  if (cfg->torso == ACME_IMPALA_TORSO_ATARI) {
    slab = std::max<int64_t>(torso::wgrad_slab_floats(), (int64_t)kOarSplits * R * 4 * H);
    if ((rc = dev_alloc(l, &l->x1, R * torso::kX1)) || (rc = dev_alloc(l, &l->x2, R * torso::kFlat)) ||
        (rc = dev_alloc(l, &l->x3, R * torso::kFlat)) || (rc = dev_alloc(l, &l->dz1, R * torso::kX1)) ||
        (rc = dev_alloc(l, &l->dz2, R * torso::kFlat)) || (rc = dev_alloc(l, &l->dz3, R * torso::kFlat)))
      return fail(rc);
  }
  if ((rc = dev_alloc(l, &l->slab, slab)) || (rc = dev_alloc(l, &l->gx, R * 4 * H)) ||
      (rc = dev_alloc(l, &l->gates, R * 4 * H)) || (rc = dev_alloc(l, &l->h, R * H)) ||
      (rc = dev_alloc(l, &l->c, R * H)) || (rc = dev_alloc(l, &l->hh, R * H2)) ||
      (rc = dev_alloc(l, &l->pv, R * (A + 1))) || (rc = dev_alloc(l, &l->dpv, R * (A + 1))) ||
      (rc = dev_alloc(l, &l->dhh, R * H2)) || (rc = dev_alloc(l, &l->dh, R * H)) ||
      (rc = dev_alloc(l, &l->dgates, R * 4 * H)) || (rc = dev_alloc(l, &l->dc, (int64_t)B * H)) ||
      (rc = dev_alloc(l, &l->vs, R)) || (rc = dev_alloc(l, &l->pg_adv, R)) ||
      (rc = dev_alloc(l, &l->lrho, R)) || (rc = dev_alloc(l, &l->lpa, R)) ||
      (rc = dev_alloc(l, &l->ent, R)) ||
      (rc = dev_alloc(l, &l->norm_part, 2 * kNormBlocks)) || (rc = dev_alloc(l, &l->dev_step, 1)) ||
      (rc = dev_alloc(l, &l->metrics_tmp, 4)) || (rc = dev_alloc(l, &l->norms, 2)) ||
      (rc = dev_alloc(l, &l->xg, (int64_t)2 * B * H)) || (rc = dev_alloc(l, &l->tmo, 4)) ||
      (rc = dev_alloc(l, &l->guard, 1)))
    return fail(rc);
  if (hipMemset(l->guard, 0, sizeof(StepGuard)) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&l->host_skipped), sizeof(int64_t),
                    hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
    return fail((set_error("step guard allocation failed"), ACME_ERR_HIP));
  *l->host_skipped = 0;
  if (H == kRgH && B <= kRgMaxB &&
      (rc = dev_alloc(l, &l->xb, (int64_t)2 * kRgGroups * B * H)))
    return fail(rc);
  // Plane path (Atari torso): each operand plane is addressed through a 31-bit byte range,
  // so the f16 frames of one step bound it (R < 38,000 frames); larger unrolls stay f32.
  if (cfg->torso == ACME_IMPALA_TORSO_ATARI && R * torso::kObsBytes * 2 < (int64_t)INT32_MAX &&
      R >= kP3MinRows && tune_variant("IMP3") != 1) {
    l->p3_capable = true;
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
    if ((rc = dev_alloc(l, &l->wpl, gemm::kPlanes * l->flat)) ||
        (rc = dev_alloc(l, &l->frames, R * torso::kObsBytes)) ||
        (rc = plane(&l->x1p, R * torso::kX1, kScX1)) ||
        (rc = plane(&l->x2p, R * torso::kFlat, kScX2)) ||
        (rc = plane(&l->x3p, R * torso::kFlat, kScX3)) ||
        (rc = plane(&l->dz1p, R * torso::kX1, kScDz1)) ||
        (rc = plane(&l->dz2p, R * torso::kFlat, kScDz2)) ||
        (rc = plane(&l->dz3p, R * torso::kFlat, kScDz3)) ||
        (rc = plane(&l->dgp, R * 4 * H, kScDgates)) ||
        (rc = dev_alloc(l, &l->pslab, std::max<int64_t>(torso::wgrad_slab_floats_p3(),
                                                        (int64_t)kOarSplitsP3 * R * 4 * H))))
      return fail(rc);
  }
  if (hipMemset(l->dev_step, 0, sizeof(int64_t)) != hipSuccess ||
      hipMemset(l->tmo, 0, 4 * sizeof(unsigned)) != hipSuccess ||
      (l->xg && hipMemset(l->xg, 0, (size_t)2 * B * H * 8) != hipSuccess) ||
      (l->xb && hipMemset(l->xb, 0, (size_t)2 * kRgGroups * B * H * 8) != hipSuccess))
    return fail((set_error("hipMemset failed"), ACME_ERR_HIP));
  *out = l;
  return ACME_OK;
}

int64_t acme_impala_flat_size(const acme_impala* l) { return l ? l->flat : 0; }

int acme_impala_set_lstm_unroll(acme_impala* l, int32_t mode) {
  ACME_CHECK_ARG(l && (mode == 0 || mode == 1), "mode must be 0 (auto) or 1 (per-step)");
  ACME_CHECK_ARG(mode == 0 || lstm_fwd_smem(l->cfg.max_batch, l->H) <= 65536,
                 "per-step launches need max_batch * lstm_size within 64 KB of LDS");
  l->lstm_steps = mode == 1;
  return ACME_OK;
}
int32_t acme_impala_num_tensors(const acme_impala* l) { return l ? (int32_t)l->tensors.size() : 0; }

int acme_impala_tensor_info(const acme_impala* l, int32_t i, int64_t* offset, int64_t* numel,
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

int acme_impala_bind(acme_impala* l, float* params, float* grads, float* adam_m, float* adam_v) {
  ACME_CHECK_ARG(l, "null learner");
  ACME_CHECK_ARG(params && grads && adam_m && adam_v, "null buffer");
  l->params = params;
  l->grads = grads;
  l->m = adam_m;
  l->v = adam_v;
  l->scales_ok = false;
  return ACME_OK;
}

int acme_impala_params_changed(acme_impala* l) {
  ACME_CHECK_ARG(l, "null learner");
  l->scales_ok = false;
  return ACME_OK;
}

int acme_impala_step(acme_impala* l, const acme_sequence_batch* b, float* metrics, void* stream) {
  ACME_CHECK_ARG(l && b, "null argument");
  ACME_CHECK_ARG(l->params, "acme_impala_bind must be called first");
  ACME_CHECK_ARG(b->batch >= 1 && b->batch <= l->cfg.max_batch, "batch %lld outside [1, %d]",
                 (long long)b->batch, l->cfg.max_batch);
  ACME_CHECK_ARG(b->sequence_length >= 2 && b->sequence_length <= l->cfg.max_sequence_length,
                 "sequence_length %lld outside [2, %d]", (long long)b->sequence_length,
                 l->cfg.max_sequence_length);
  ACME_CHECK_ARG(b->observation && b->prev_action && b->prev_reward && b->action && b->reward &&
                     b->discount && b->behaviour_logits && b->h0 && b->c0,
                 "null batch field");
  ACME_CHECK_ARG(b->state_stride >= l->H && b->state_stride % 4 == 0 &&
                     ((uintptr_t)b->h0 & 15) == 0,
                 "core state rows must be 16-byte aligned with state_stride >= lstm_size");
  hipStream_t st = as_stream(stream);
  int rc = ACME_OK;
  if (atari(l) && use_p3(l, (int)(b->batch * b->sequence_length)) && !l->scales_ok) {
    // Plane scales for newly bound parameters: forward + backward passes without the
    // update (the first at the current scales, whose maxima are measured before the split;
    // each ends with the rescale), then the step.  Overflows at the initial scales are
    // expected and cleared.
    // Four passes: the input-gradient chain dgates -> dz3 -> dz2 -> dz1 is four tensors
    // deep, and a tensor computed from planes that underflowed at their initial scale
    // measures 0 until its input is calibrated (as the DQN learner's calibrate_scales).
    for (int pass = 0; pass < 4 && rc == ACME_OK; ++pass) rc = impala_step_impl(l, b, nullptr, st, false);
    if (rc != ACME_OK) return rc;
    ACME_HIP_TRY(hipMemsetAsync(l->overflow, 0, sizeof(int), st));
    ACME_HIP_TRY(hipMemsetAsync(l->guard, 0, offsetof(StepGuard, applied), st));
    ACME_HIP_TRY(hipMemsetAsync(l->tmo, 0, sizeof(unsigned), st));
    l->scales_ok = true;
  }
  rc = impala_step_impl(l, b, metrics, st);
  if (rc != ACME_OK) return rc;
  l->num_steps += 1;
  return ACME_OK;
}

int acme_impala_plane_overflow(acme_impala* l, int32_t* overflow, int32_t reset) {
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

int acme_impala_policy_step(acme_impala* l, const void* obs, const int32_t* prev_action,
                            const float* prev_reward, const float* h, const float* c,
                            int64_t rows, float* logits, float* values, float* h_out,
                            float* c_out, void* stream) {
  ACME_CHECK_ARG(l && obs && prev_action && prev_reward && h && c, "null argument");
  ACME_CHECK_ARG(l->params, "acme_impala_bind must be called first");
  ACME_CHECK_ARG(rows >= 1 && rows <= l->cfg.max_batch,
                 "rows must be in [1, max_batch=%d]", l->cfg.max_batch);
  hipStream_t st = as_stream(stream);
  const int H = l->H, A = l->A;
  const bool p3 = l->policy_planes && atari(l) && use_p3(l, (int)rows);
  auto forward = [&]() {
    // The policy's unroll has its own timeout word (a learner step is not skipped for it).
    int rc = network_forward(l, obs, prev_action, prev_reward, h, c, H, (int)rows, 1, st, p3,
                             l->tmo + 2);
    if (rc != ACME_OK || !p3) return rc;
    // The next call's scales from this call's maxima (lagged, 2^8 of headroom); a plane
    // write that overflowed shows in acme_impala_plane_overflow.
    RescaleGuard rg;
    return launch_plane_rescale(l->scales, kScTransient, kScTransient, -1, -1, l->overflow, st,
                                -1, -1, rg);
  };
  int rc;
  if (p3 && !l->scales_ok) {
    // First call (or new parameters): three passes set the chain frames -> x1 -> x2 -> x3
    // (and the parameter planes) from real maxima before the call whose outputs count.
    for (int pass = 0; pass < 3; ++pass)
      if ((rc = forward()) != ACME_OK) return rc;
    ACME_HIP_TRY(hipMemsetAsync(l->overflow, 0, sizeof(int), st));
    l->scales_ok = true;
  }
  if ((rc = forward()) != ACME_OK) return rc;
  // Outputs are rows of the T = 1 unroll.
  if (logits)
    ACME_HIP_TRY(hipMemcpy2DAsync(logits, A * sizeof(float), l->pv, (A + 1) * sizeof(float),
                                  A * sizeof(float), rows, hipMemcpyDeviceToDevice, st));
  if (values)
    ACME_HIP_TRY(hipMemcpy2DAsync(values, sizeof(float), l->pv + A, (A + 1) * sizeof(float),
                                  sizeof(float), rows, hipMemcpyDeviceToDevice, st));
  if (h_out)
    ACME_HIP_TRY(hipMemcpyAsync(h_out, l->h, rows * H * sizeof(float), hipMemcpyDeviceToDevice, st));
  if (c_out)
    ACME_HIP_TRY(hipMemcpyAsync(c_out, l->c, rows * H * sizeof(float), hipMemcpyDeviceToDevice, st));
  return ACME_OK;
}

int acme_impala_set_policy_planes(acme_impala* l, int32_t on) {
  ACME_CHECK_ARG(l, "null learner");
  l->policy_planes = on != 0;
  l->scales_ok = false;
  return ACME_OK;
}

int64_t acme_impala_num_steps(const acme_impala* l) { return l ? l->num_steps : 0; }

int acme_impala_set_applied_steps(acme_impala* l, int64_t n) {
  ACME_CHECK_ARG(l && n >= 0, "bad argument");
  ACME_HIP_TRY(hipDeviceSynchronize());
  ACME_HIP_TRY(hipMemcpy(l->dev_step, &n, sizeof(n), hipMemcpyHostToDevice));
  ACME_HIP_TRY(hipMemcpy(&l->guard->applied, &n, sizeof(n), hipMemcpyHostToDevice));
  return ACME_OK;
}

// Scale state = (w, r, wi, rl) of every record (as acme_dqn_scale_state).
int acme_impala_scale_state(const acme_impala* l, float* out, int32_t capacity, int32_t* count) {
  ACME_CHECK_ARG(l && count, "null argument");
  *count = l->scales ? 4 * kScCount : 0;
  if (!l->scales || !out) return ACME_OK;
  ACME_CHECK_ARG(capacity >= 4 * kScCount, "scale state needs %d floats", 4 * kScCount);
  ACME_HIP_TRY(hipDeviceSynchronize());
  for (int i = 0; i < kScCount; ++i)
    ACME_HIP_TRY(hipMemcpy(out + 4 * i, l->scales + i, 4 * sizeof(float), hipMemcpyDeviceToHost));
  return ACME_OK;
}

int acme_impala_set_scale_state(acme_impala* l, const float* in, int32_t count) {
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

int64_t acme_impala_skipped_steps(const acme_impala* l) {
  if (!l || !l->host_skipped) return 0;
  return *reinterpret_cast<volatile const int64_t*>(l->host_skipped);
}

int acme_impala_guard_state(acme_impala* l, int64_t* out4) {
  ACME_CHECK_ARG(l && out4 && l->guard, "null argument");
  ACME_HIP_TRY(hipDeviceSynchronize());
  StepGuard g;
  unsigned t[4];
  ACME_HIP_TRY(hipMemcpy(&g, l->guard, sizeof(g), hipMemcpyDeviceToHost));
  ACME_HIP_TRY(hipMemcpy(t, l->tmo, sizeof(t), hipMemcpyDeviceToHost));
  out4[0] = g.applied;
  out4[1] = g.skipped;
  out4[2] = g.last;
  out4[3] = t[1];
  return ACME_OK;
}

int acme_impala_set_num_steps(acme_impala* l, int64_t n) {
  ACME_CHECK_ARG(l && n >= 0, "bad argument");
  ACME_HIP_TRY(hipDeviceSynchronize());
  ACME_HIP_TRY(hipMemcpy(l->dev_step, &n, sizeof(n), hipMemcpyHostToDevice));
  l->num_steps = n;
  return ACME_OK;
}

int acme_impala_debug_buffer(const acme_impala* l, const char* name, const float** out,
                             int64_t* count) {
  ACME_CHECK_ARG(l && name && out && count, "null argument");
  const int64_t R = (int64_t)l->cfg.max_batch * l->cfg.max_sequence_length;
  struct Item {
    const char* n;
    const float* p;
    int64_t c;
  } items[] = {
      {"pv", l->pv, R * (l->A + 1)}, {"vs", l->vs, R},        {"pg_adv", l->pg_adv, R},
      {"h", l->h, R * l->H},         {"c", l->c, R * l->H},   {"dpv", l->dpv, R * (l->A + 1)},
      {"dgates", l->dgates, R * 4 * l->H}, {"grad_norm", l->norms, 1},
      {"lstm_timeout", reinterpret_cast<const float*>(l->tmo + 1), 1},
      {"lstm_timeout_step", reinterpret_cast<const float*>(l->tmo), 1},
      {"policy_lstm_timeout", reinterpret_cast<const float*>(l->tmo + 2), 1},
      {"hh", l->hh, R * l->H2},      {"x1", l->x1, l->x1 ? R * torso::kX1 : 0},
      {"x2", l->x2, l->x2 ? R * torso::kFlat : 0}, {"x3", l->x3, l->x3 ? R * torso::kFlat : 0},
  };
  for (const Item& it : items)
    if (it.p && strcmp(it.n, name) == 0) {
      if (l->last_p3) {  // the plane path keeps the torso activations as planes: join them
        const struct {
          const char* n;
          torso::Plane pl;
          int64_t per_row;
        } ptab[] = {{"x1", l->x1p, torso::kX1}, {"x2", l->x2p, torso::kFlat},
                    {"x3", l->x3p, torso::kFlat}};
        for (const auto& q : ptab)
          if (strcmp(q.n, name) == 0) {
            ACME_HIP_TRY(hipDeviceSynchronize());
            int rc = launch_join_planes(q.pl.p, q.pl.stride, l->last_rows * q.per_row,
                                        const_cast<float*>(it.p), q.pl.sc, 0);
            if (rc != ACME_OK) return rc;
            ACME_HIP_TRY(hipDeviceSynchronize());
          }
      }
      *out = it.p;
      *count = it.c;
      return ACME_OK;
    }
  set_error("unknown debug buffer '%s'", name);
  return ACME_ERR_INVALID;
}

}  // extern "C"
