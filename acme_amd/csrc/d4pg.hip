// D4PG learner step for MI355X: the replacement of D4PGLearner._step
// (acme/agents/tf/d4pg/learning.py:156-247) behind the C ABI (include/acme_hip.h).
//
// One call = the whole step on one stream, no host synchronisation:
//   target <- online when num_steps % period == 0 (at the start)          (:171-175)
//   online policy on o_t (dpg actions), target policy on o_t              (:199, :206)
//   online critic on [o_tm1, a_tm1 ; o_t, dpg_a] as ONE 2B-row pass        (:198, :207)
//   target critic on (o_t, target actions)                                (:199)
//   fused loss kernel: categorical L2 projection + softmax cross-entropy   (:202-203)
//     for rows < B, d mean(q) / d logits for the dpg rows                  (:208)
//   critic backward over 2B rows (weight gradients from the first B rows
//     only); the LayerNorm backward of the dpg rows also forms dq/da,
//     tf.clip_by_norm(., 1) and dloss/da = -dqda / B                      (:211-218, dpg.py)
//   policy backward; clip_by_global_norm(40) per network; two Adams       (:221-241)
//
// Networks (examples/control_suite/run_d4pg.py:60-81): LayerNormMLP
// (acme/tf/networks/continuous.py:37-68) = Linear -> LayerNorm -> tanh -> MLP(elu,
// activate_final); policy head NearZeroInitializedLinear + TanhToSpec
// (rescaling.py:55-74); critic head DiscreteValuedHead (distributional.py:36-67).
//
// Small-batch regime (B = 256, widths <= 512): the step is ~1.5 GFLOP, so it is latency
// bound.  Dense layers go through the fp32 MFMA GEMM engine with fused bias/activation
// epilogues and masked dgrads; the row-wise work (LayerNorm+tanh, TanhToSpec head,
// projection loss, LayerNorm backward + dpg) are one-kernel-per-stage row kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "conv.h"
#include "gemm.h"
#include "gemm_direct.h"
#include "kernels.h"
#include "profiler.h"


using namespace acme;
using namespace acme::conv;

namespace {

constexpr int kRows = 4;      // rows per block of the LayerNorm row kernels
constexpr int kMaxWidth = 1024;
constexpr int kMaxIn = 64;    // obs_dim + act_dim
constexpr int kNormBlocks = 256;

struct Tensor {
  std::string name;
  int64_t offset = 0, numel = 0;
  int ndim = 0;
  int64_t shape[4] = {1, 1, 1, 1};
};

// Tensor indices of one LayerNormMLP + output layer.
struct NetDesc {
  int din = 0, nl = 0, nout = 0;
  int sizes[ACME_D4PG_MAX_LAYERS] = {};
  int w1 = -1, b1 = -1, scale = -1, offset = -1;
  int w[ACME_D4PG_MAX_LAYERS] = {}, b[ACME_D4PG_MAX_LAYERS] = {};  // mlp linear_{i-1}, i >= 1
  int ow = -1, ob = -1;                                            // output layer
};

// Activations of one evaluation of a network over `rows` rows.
struct Acts {
  float* z1 = nullptr;    // [rows][H0] first linear output (pre-LayerNorm)
  float* mean = nullptr;  // [rows]
  float* rstd = nullptr;  // [rows]
  float* h[ACME_D4PG_MAX_LAYERS] = {};  // h[0] = tanh(LN(z1)), h[i] = elu(...)
  float* out = nullptr;   // policy: actions [rows][act]; critic: logits [rows][atoms]
  float* t = nullptr;     // policy: tanh of the head [rows][act]
};

}  // namespace

struct acme_d4pg {
  acme_d4pg_config cfg;
  std::vector<Tensor> tensors;
  int64_t flat = 0, policy_flat = 0;
  float *params = nullptr, *target = nullptr, *grads = nullptr, *m = nullptr, *v = nullptr;
  int64_t num_steps = 0;
  NetDesc pol, cri;
  std::vector<void*> allocs;
  Acts pon, ptg, con, ctg;
  float* cdz[ACME_D4PG_MAX_LAYERS] = {};  // critic pre-activation grads [2B][C_i]
  float* pdz[ACME_D4PG_MAX_LAYERS] = {};  // policy [B][P_i]
  float* dlogits = nullptr;               // [2B][atoms]
  float* du = nullptr;                    // [B][act] dloss/d(policy head pre-tanh)
  float* dqda = nullptr;                  // [B][act] clipped dq/da
  float* values = nullptr;                // [atoms] support
  float* act_lo = nullptr;                // [act]
  float* act_scale = nullptr;             // [act]
  float* lnslab = nullptr;                // LayerNorm parameter-gradient partials (critic)
  float* lnslab2 = nullptr;               // (policy: both are reduced after the backward)
  float* ploss_part = nullptr;            // per-block dpg loss partials
  double* norm_part = nullptr;            // [2][kNormBlocks]
  float* norms = nullptr;                 // [2] global norms (policy, critic)
  float* loss_tmp = nullptr;              // [2] critic / policy loss
  float* ce = nullptr;                    // [B] per-row cross-entropy
  int64_t* dev_step = nullptr;            // device mirror of num_steps (Adam t)
  // Captured step graphs, keyed by the batch / output pointers, B and the target copy.
  struct Graph {
    const void* key[7];
    int64_t B;
    bool copy;
    hipGraphExec_t exec;
  };
  std::vector<Graph> graphs;
  hipStream_t capture = nullptr;
};

namespace {

int64_t align64(int64_t x) { return (x + 63) & ~int64_t(63); }

int add_tensor(acme_d4pg* l, const std::string& name, std::initializer_list<int64_t> shape) {
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
int dev_alloc(acme_d4pg* l, T** p, int64_t count) {
  void* q = nullptr;
  if (hipMalloc(&q, std::max<int64_t>(count, 1) * sizeof(T)) != hipSuccess) {
    set_error("hipMalloc of %lld bytes failed", (long long)(count * sizeof(T)));
    return ACME_ERR_OOM;
  }
  l->allocs.push_back(q);
  *p = static_cast<T*>(q);
  return ACME_OK;
}

void add_net(acme_d4pg* l, NetDesc& d, const char* prefix, int din, int nl, const int32_t* sizes,
             int nout, const char* head) {
  d.din = din;
  d.nl = nl;
  d.nout = nout;
  for (int i = 0; i < nl; ++i) d.sizes[i] = sizes[i];
  const std::string p = std::string(prefix) + "/layer_norm_mlp";
  d.w1 = add_tensor(l, p + "/linear/w", {din, sizes[0]});
  d.b1 = add_tensor(l, p + "/linear/b", {sizes[0]});
  d.scale = add_tensor(l, p + "/layer_norm/scale", {sizes[0]});
  d.offset = add_tensor(l, p + "/layer_norm/offset", {sizes[0]});
  for (int i = 1; i < nl; ++i) {
    const std::string q = p + "/mlp/linear_" + std::to_string(i - 1);
    d.w[i] = add_tensor(l, q + "/w", {sizes[i - 1], sizes[i]});
    d.b[i] = add_tensor(l, q + "/b", {sizes[i]});
  }
  const std::string h = std::string(prefix) + "/" + head;
  d.ow = add_tensor(l, h + "/w", {sizes[nl - 1], nout});
  d.ob = add_tensor(l, h + "/b", {nout});
}

int alloc_acts(acme_d4pg* l, Acts& a, const NetDesc& d, int rows, bool policy) {
  int rc;
  if ((rc = dev_alloc(l, &a.z1, (int64_t)rows * d.sizes[0])) ||
      (rc = dev_alloc(l, &a.mean, rows)) || (rc = dev_alloc(l, &a.rstd, rows)) ||
      (rc = dev_alloc(l, &a.out, (int64_t)rows * d.nout)))
    return rc;
  for (int i = 0; i < d.nl; ++i)
    if ((rc = dev_alloc(l, &a.h[i], (int64_t)rows * d.sizes[i]))) return rc;
  if (policy && (rc = dev_alloc(l, &a.t, (int64_t)rows * d.nout))) return rc;
  return ACME_OK;
}

inline const float* P(const acme_d4pg* l, const float* base, int t) {
  return base + l->tensors[t].offset;
}
inline float* Pm(const acme_d4pg* l, float* base, int t) { return base + l->tensors[t].offset; }

// ------------------------------------------------------------------ device helpers

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Sums N per-thread values over a 256-thread block; every thread gets the totals.
template <int N>
__device__ __forceinline__ void block_sum256(float (&v)[N], float (*red)[N]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = wave_sum(v[i]);
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < N; ++i) red[wave][i] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
}

// ------------------------------------------------------------------ LayerNorm first layer
// h = tanh(LayerNorm(concat(xa, xb) @ W + b)) for kRows rows per 256-thread block.
// Rows < split read (xa0, xb0), the others (xa1, xb1) at row - split.
// The policy head in front of the critic: part p's xb (the actions) computed in the block from
// the policy's last hidden layer when head[p].h is set (and written to head[p].t / .a as
// policy_head_kernel would), instead of read from xb.
struct PolHeadSrc {
  const float* h;  // [rows of the part][Hp], null: xb is given
  float *t, *a;    // tanh outputs, actions
};
struct LnFirstArgs {
  const float *xa0, *xb0, *xa1, *xb1;
  int split, rows, da, db, H;
  const float *w, *b, *scale, *offset;
  float eps;
  float *z, *mean, *rstd, *h;
  PolHeadSrc head[2];
  const float *hw, *hb;  // the policy head of this evaluation's network
};

// Two evaluations in one launch (the online and target networks): blockIdx.y picks the
// argument set; blocks past that set's rows leave at once.
struct LnFirstPair {
  LnFirstArgs a[2];
  const float *lo, *scale;  // TanhToSpec range of the fused policy heads
  int Hp;                   // policy hidden width
};

// One row of the policy head, lane j < A: u_j = h_row . W[:, j] (lane-strided partial sums,
// then the butterfly sum) and the TanhToSpec action; policy_head_kernel and the fused head
// of ln_first_kernel share it, so both give the same bits.
__device__ __forceinline__ void policy_head_row(const float* __restrict__ h, const float* __restrict__ w,
                                                const float* __restrict__ b, const float* __restrict__ lo,
                                                const float* __restrict__ scale, int H, int A,
                                                int lane, float& t, float& act) {
  float acc[ACME_D4PG_MAX_ACT];
#pragma unroll
  for (int j = 0; j < ACME_D4PG_MAX_ACT; ++j) acc[j] = 0.f;
  // Four k steps per chunk with their loads issued together (the sums still run k by k).
  for (int k0 = lane; k0 < H; k0 += 4 * 64) {
    float hv[4], wv[4][ACME_D4PG_MAX_ACT];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = min(k0 + 64 * u, H - 1);
      hv[u] = h[k];
#pragma unroll
      for (int j = 0; j < ACME_D4PG_MAX_ACT; ++j) wv[u][j] = j < A ? w[(size_t)k * A + j] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (k0 + 64 * u >= H) break;
#pragma unroll
      for (int j = 0; j < ACME_D4PG_MAX_ACT; ++j)
        if (j < A) acc[j] = fmaf(hv[u], wv[u][j], acc[j]);
    }
  }
  float mine = 0.f;
#pragma unroll
  for (int j = 0; j < ACME_D4PG_MAX_ACT; ++j) {
    if (j >= A) break;
    const float s = wave_sum(acc[j]);
    if (lane == j) mine = s;
  }
  t = 0.f;
  act = 0.f;
  if (lane < A) {
    t = tanhf(mine + b[lane]);
    act = (0.5f * (t + 1.f)) * scale[lane] + lo[lane];
  }
}

template <int C>  // feature columns per thread: H <= 256 C
__global__ void __launch_bounds__(256) ln_first_kernel(const LnFirstPair pair) {
  __shared__ float xs[kRows][kMaxIn];
  __shared__ float red[4][kRows];
  const LnFirstArgs& a = pair.a[blockIdx.y];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * kRows;
  if (r0 >= a.rows) return;  // uniform per block
  const int din = a.da + a.db;
  // Loads that depend on nothing go out first: the bias / LayerNorm parameters of this
  // thread's columns and the first KU input rows of their weights (clamped indices; the
  // products below still run in k order).
  constexpr int KU = 32;
  float bj[C], scj[C], ofj[C], wk[C][KU];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int j = min(tid + 256 * c, a.H - 1);
    bj[c] = a.b[j];
    scj[c] = a.scale[j];
    ofj[c] = a.offset[j];
#pragma unroll
    for (int u = 0; u < KU; ++u) wk[c][u] = a.w[(size_t)min(u, din - 1) * a.H + j];
  }
  for (int i = tid; i < kRows * din; i += 256) {
    const int r = i / din, k = i - r * din, row = r0 + r;
    float v = 0.f;
    if (row < a.rows) {
      const bool second = row >= a.split;
      const int rr = second ? row - a.split : row;
      if (k >= a.da && a.head[second].h) continue;  // the fused head writes it
      v = k < a.da ? (second ? a.xa1 : a.xa0)[(size_t)rr * a.da + k]
                   : (second ? a.xb1 : a.xb0)[(size_t)rr * a.db + (k - a.da)];
    }
    xs[r][k] = v;
  }
  {
    // Fused policy head: wave r computes row r0 + r's actions.
    static_assert(kRows == 4, "one wave per row of the block");
    const int r = tid >> 6, lane = tid & 63, row = r0 + r;
    const bool second = row >= a.split;
    const PolHeadSrc hs = a.head[second];
    if (row < a.rows && hs.h) {  // uniform per wave
      const int rr = second ? row - a.split : row;
      float t, act;
      policy_head_row(hs.h + (size_t)rr * pair.Hp, a.hw, a.hb, pair.lo, pair.scale, pair.Hp,
                      a.db, lane, t, act);
      if (lane < a.db) {
        if (hs.t) hs.t[(size_t)rr * a.db + lane] = t;
        hs.a[(size_t)rr * a.db + lane] = act;
        xs[r][a.da + lane] = act;
      }
    }
  }
  __syncthreads();
  float acc[kRows][C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int j = tid + 256 * c;
#pragma unroll
    for (int r = 0; r < kRows; ++r) acc[r][c] = 0.f;
    if (j < a.H) {
      for (int k0 = 0; k0 < din; k0 += KU) {
        if (k0 > 0) {
#pragma unroll
          for (int u = 0; u < KU; ++u)
            wk[c][u] = k0 + u < din ? a.w[(size_t)(k0 + u) * a.H + j] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < KU; ++u) {
          if (k0 + u >= din) break;
#pragma unroll
          for (int r = 0; r < kRows; ++r) acc[r][c] = fmaf(xs[r][k0 + u], wk[c][u], acc[r][c]);
        }
      }
#pragma unroll
      for (int r = 0; r < kRows; ++r) acc[r][c] += bj[c];
    }
  }
  // tf.nn.moments over the feature axis: mean, then mean of squared deviations.
  float s[kRows];
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    s[r] = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c)
      if (tid + 256 * c < a.H) s[r] += acc[r][c];
  }
  block_sum256<kRows>(s, red);
  const float invH = 1.f / (float)a.H;
  float mean[kRows], q[kRows];
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    mean[r] = s[r] * invH;
    q[r] = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c)
      if (tid + 256 * c < a.H) {
        const float dv = acc[r][c] - mean[r];
        q[r] = fmaf(dv, dv, q[r]);
      }
  }
  block_sum256<kRows>(q, red);
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    const int row = r0 + r;
    if (row >= a.rows) continue;
    const float rs = 1.f / sqrtf(q[r] * invH + a.eps);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int j = tid + 256 * c;
      if (j >= a.H) continue;
      const size_t idx = (size_t)row * a.H + j;
      a.z[idx] = acc[r][c];
      const float y = (acc[r][c] - mean[r]) * rs * scj[c] + ofj[c];
      a.h[idx] = tanhf(y);
    }
    if (tid == 0) {
      a.mean[row] = mean[r];
      a.rstd[row] = rs;
    }
  }
}

// ------------------------------------------------------------------ policy head
// One wave per row: u = h @ W + b (A <= 16 outputs), t = tanh(u),
// a = (0.5 (t + 1)) * (max - min) + min  (TanhToSpec, rescaling.py:70-73).
struct PolicyHeadArgs {
  const float *h, *w, *b;
  int rows;
  float *t_out, *a_out;
};
struct PolicyHeadPair {
  PolicyHeadArgs a[2];  // blockIdx.y
  const float *lo, *scale;
  int H, A;
};

__global__ void __launch_bounds__(256) policy_head_kernel(const PolicyHeadPair pr) {
  const PolicyHeadArgs& pa = pr.a[blockIdx.y];
  const float* __restrict__ h = pa.h;
  const float* __restrict__ w = pa.w;
  const float* __restrict__ b = pa.b;
  const float* __restrict__ lo = pr.lo;
  const float* __restrict__ scale = pr.scale;
  const int rows = pa.rows, H = pr.H, A = pr.A;
  float* __restrict__ t_out = pa.t_out;
  float* __restrict__ a_out = pa.a_out;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float t, act;
  policy_head_row(h + (size_t)row * H, w, b, lo, scale, H, A, lane, t, act);
  if (lane < A) {
    if (t_out) t_out[(size_t)row * A + lane] = t;
    a_out[(size_t)row * A + lane] = act;
  }
}

// ------------------------------------------------------------------ loss
// One wave per row (4 rows per 256-thread block); lane i = atom i.
//   rows < B  : categorical TD loss (distributional.py:22-41) with the L2 projection
//               written exactly as l2_project (:44-83); dlogits = (softmax - target) / B,
//               ce[row] = cross-entropy (summed into the loss by adam_clip_kernel).
//   rows >= B : dpg rows; q = sum softmax * values, dq/dlogits = (values - q) * softmax.
// The loss math of one row from its logits in registers (ql: the online critic's, tl: the
// target critic's, lane = atom, -inf past K).
__device__ __forceinline__ void loss_row(float ql, float tl, int row, int lane,
                                         const float* __restrict__ r, const float* __restrict__ d,
                                         const float* __restrict__ values, int B, int K,
                                         float discount, float* __restrict__ dlogits,
                                         float* __restrict__ ce_out) {
  const bool on = lane < K;
  const float vi = on ? values[lane] : 0.f;
  const float m2 = wave_max(ql);
  const float e2 = on ? expf(ql - m2) : 0.f;
  const float s2 = wave_sum(e2);
  const float sm = e2 / s2;
  if (row >= B) {
    const float q = wave_sum(on ? sm * vi : 0.f);
    if (on) dlogits[(size_t)row * K + lane] = (vi - q) * sm;
    return;
  }
  const float vmin = values[0], vmax = values[K - 1];
  // Support spacings of l2_project: d_pos = Zq[i+1] - Zq[i] (wrapping to vmin), d_neg =
  // Zq[i] - Zq[i-1] (wrapping to vmax).
  const float dpos = on ? ((lane + 1 < K ? values[lane + 1] : vmin) - vi) : 1.f;
  const float dneg = on ? (vi - (lane > 0 ? values[lane - 1] : vmax)) : 1.f;
  const float mx = wave_max(tl);
  const float e = on ? expf(tl - mx) : 0.f;
  const float pj = e / wave_sum(e);
  const float gd = discount * d[row];
  const float zc = fminf(fmaxf(r[row] + gd * vi, vmin), vmax);
  // delta_hat = (sg dq) / d_pos - ((1 - sg) dq) / d_neg with sg = (dq >= 0): one of the two
  // terms is an exact zero, so delta_hat = |dq| / (sg ? d_pos : d_neg), the same bits with
  // one division.  Source atom j's values come from lane j by readlane (j is uniform).
  float tgt = 0.f;
  for (int j = 0; j < K; ++j) {
    const float zcj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(zc), j));
    const float pjj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pj), j));
    const float dq = zcj - vi;
    const float dh = fabsf(dq) / (dq >= 0.f ? dpos : dneg);
    tgt += fminf(fmaxf(1.f - dh, 0.f), 1.f) * pjj;
  }
  const float logp = ql - m2 - logf(s2);
  const float ce = wave_sum(on ? -tgt * logp : 0.f);
  if (on) dlogits[(size_t)row * K + lane] = (1.f / (float)B) * (sm - tgt);
  if (lane == 0) ce_out[row] = ce;
}

__global__ void __launch_bounds__(256) d4pg_loss_kernel(
    const float* __restrict__ c_logits, const float* __restrict__ t_logits,
    const float* __restrict__ r, const float* __restrict__ d, const float* __restrict__ values,
    int B, int K, float discount, float* __restrict__ dlogits, float* __restrict__ ce_out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= 2 * B) return;
  const bool on = lane < K;
  const float ql = on ? c_logits[(size_t)row * K + lane] : -INFINITY;
  const float tl = on && row < B ? t_logits[(size_t)row * K + lane] : -INFINITY;
  loss_row(ql, tl, row, lane, r, d, values, B, K, discount, dlogits, ce_out);
}

// ------------------------------------------------------------------ LayerNorm backward
// Per row (kRows rows per block): dy = dLoss/d(LayerNorm output) (tanh' already
// applied), xhat = (z - mean) * rstd, g = dy * scale,
//   dz = rstd * (g - mean(g) - xhat * mean(g * xhat))
// Rows < ce_rows: dz is written in place over dy and (dy * xhat, dy) are summed into
// per-block column partials (LayerNorm scale / offset gradients).
// Rows >= ce_rows (the critic's dpg rows): dqda = dz @ W1[act rows]^T, clipped to norm
// <= clip (tf.clip_by_norm; clip <= 0 disables), du = -dqda / B * 0.5 * scale_a * (1-t^2)
// (through TanhToSpec), and 0.5 |dqda|^2 summed into ploss_part[block].
struct LnBwdArgs {
  float* dy;  // [rows][H], overwritten with dz for rows < ce_rows
  const float *z, *mean, *rstd, *scale;
  int rows, ce_rows, H;
  float* colslab;  // [gridDim.x][2][H]
  // dpg
  const float* w1;  // [din][H]
  int act_off, A;
  float clip, invB;
  const float *t, *act_scale;  // [B][A], [A] (policy head tanh, TanhToSpec range)
  float *du, *dqda, *ploss_part;
};

// C: feature columns per thread (H <= 256 C); AM: action slots (A <= AM).  Both sized per
// launch: the widest instantiation (C = 4, AM = 16) spills at H = 512, A = 6.
template <int C, int AM>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const LnBwdArgs a) {
  __shared__ float red[4][2 * kRows];
  __shared__ float redq[4][kRows * AM];
  __shared__ float dq_s[kRows][AM];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * kRows;
  const float invH = 1.f / (float)a.H;
  float g[kRows][C], xh[kRows][C], dyv[kRows][C];
  float s[2 * kRows];
  // Every load of the block is issued before the first use: clamped addresses and selects
  // instead of branches around the loads (a branch per load serialises them).  Invalid
  // entries contribute exact zeros to the sums.
  const int last = a.rows - 1;
  const bool has_dpg = r0 + kRows - 1 >= a.ce_rows && r0 < a.rows;  // uniform per block
  float w1v[C][AM];
  if (has_dpg) {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int k = 0; k < AM; ++k)
        w1v[c][k] = a.w1[(size_t)(a.act_off + min(k, a.A - 1)) * a.H + min(tid + 256 * c, a.H - 1)];
  }
  float sc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) sc[c] = a.scale[min(tid + 256 * c, a.H - 1)];
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    const int row = r0 + r;
    const bool ok = row < a.rows;
    const float mu0 = a.mean[min(row, last)], rs0 = a.rstd[min(row, last)];
    const float mu = ok ? mu0 : 0.f, rs = ok ? rs0 : 0.f;
    s[2 * r] = s[2 * r + 1] = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int j = tid + 256 * c;
      const bool v = ok && j < a.H;
      const size_t idx = (size_t)min(row, last) * a.H + min(j, a.H - 1);
      const float dy = a.dy[idx], z = a.z[idx];
      dyv[r][c] = v ? dy : 0.f;
      xh[r][c] = v ? (z - mu) * rs : 0.f;
      g[r][c] = v ? dy * sc[c] : 0.f;
      s[2 * r] += g[r][c];
      s[2 * r + 1] = fmaf(g[r][c], xh[r][c], s[2 * r + 1]);
    }
  }
  block_sum256<2 * kRows>(s, red);
  float cs_x[C], cs_1[C];
#pragma unroll
  for (int c = 0; c < C; ++c) cs_x[c] = cs_1[c] = 0.f;
  float dqp[kRows][AM];
#pragma unroll
  for (int r = 0; r < kRows; ++r)
#pragma unroll
    for (int k = 0; k < AM; ++k) dqp[r][k] = 0.f;
  bool any_dpg = false;
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    const int row = r0 + r;
    if (row >= a.rows) continue;
    const float rs = a.rstd[row];
    const float m1 = s[2 * r] * invH, m2 = s[2 * r + 1] * invH;
    const bool ce = row < a.ce_rows;
    any_dpg |= !ce;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int j = tid + 256 * c;
      if (j >= a.H) continue;
      const float dz = rs * (g[r][c] - m1 - xh[r][c] * m2);
      if (ce) {
        a.dy[(size_t)row * a.H + j] = dz;
        cs_x[c] = fmaf(dyv[r][c], xh[r][c], cs_x[c]);
        cs_1[c] += dyv[r][c];
      } else {
#pragma unroll
        for (int k = 0; k < AM; ++k)
          dqp[r][k] = k < a.A ? fmaf(dz, w1v[c][k], dqp[r][k]) : dqp[r][k];
      }
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int j = tid + 256 * c;
    if (j < a.H) {
      a.colslab[((size_t)blockIdx.x * 2 + 0) * a.H + j] = cs_x[c];
      a.colslab[((size_t)blockIdx.x * 2 + 1) * a.H + j] = cs_1[c];
    }
  }
  if (!any_dpg) {  // uniform per block: rows are contiguous
    if (tid == 0 && a.ploss_part) a.ploss_part[blockIdx.x] = 0.f;
    return;
  }
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int r = 0; r < kRows; ++r)
#pragma unroll
    for (int k = 0; k < AM; ++k) {
      if (k >= a.A) break;
      const float v = wave_sum(dqp[r][k]);
      if (lane == 0) redq[wave][r * AM + k] = v;
    }
  __syncthreads();
  if (tid < kRows * AM) {
    const int r = tid / AM, k = tid % AM;
    dq_s[r][k] = ((redq[0][tid] + redq[1][tid]) + redq[2][tid]) + redq[3][tid];
  }
  __syncthreads();
  if (tid < kRows) {
    const int row = r0 + tid;
    float pl = 0.f;
    if (row < a.rows && row >= a.ce_rows) {
      const int b = row - a.ce_rows;
      float n2 = 0.f;
      for (int k = 0; k < a.A; ++k) n2 = fmaf(dq_s[tid][k], dq_s[tid][k], n2);
      // tf.clip_by_norm(t, c): t * c / max(|t|, c), |t| = 0 kept as is.
      const float nrm = n2 > 0.f ? sqrtf(n2) : 0.f;
      const float den = a.clip > 0.f ? fmaxf(nrm, a.clip) : 1.f;
      const float cm = a.clip > 0.f ? a.clip : 1.f;
      for (int k = 0; k < a.A; ++k) {
        const float dq = (dq_s[tid][k] * cm) / den;
        a.dqda[(size_t)b * a.A + k] = dq;
        pl = fmaf(0.5f * dq, dq, pl);
        const float tk = a.t[(size_t)b * a.A + k];
        const float da = -dq * a.invB;
        a.du[(size_t)b * a.A + k] = da * a.act_scale[k] * 0.5f * (1.f - tk * tk);
      }
    }
    // Sum the kRows partials of this block.
    pl += __shfl_down(pl, 2, 64);
    pl += __shfl_down(pl, 1, 64);
    if (tid == 0) a.ploss_part[blockIdx.x] = pl;
  }
}

// ------------------------------------------------------------------ orchestration

// Small GEMMs: 32x32 output tiles, 8 waves per block splitting the reduction, so a
// 512 x 512 x 512 layer runs 2048 waves: the register-operand engine (gemm_direct.h, one
// load burst per wave; round 5: 0.196 -> 0.164 ms per step against the staged f32 engine of
// gemm.h, profiles/r05/ab/d4pg_direct_*.log).
#define D4_LAUNCH(prob, nz) gemm::launch_direct(prob, nz, (prob).K, st)
#define D4_GEMM(name, prob)                                                                   \
  do {                                                                                        \
    ACME_PROF_PEAK(name, st, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, 0.0, 157.3);       \
    hipError_t _e = D4_LAUNCH(prob, 1);                                                       \
    if (_e != hipSuccess) {                                                                   \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                    \
    }                                                                                         \
  } while (0)

#define D4_CHECK()                                                                            \
  do {                                                                                        \
    hipError_t _e = hipGetLastError();                                                        \
    if (_e != hipSuccess) {                                                                   \
      set_error("kernel launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                    \
    }                                                                                         \
  } while (0)

// Dense layer forward y = act(x @ W + b) over `rows` rows.
int dense_fwd(const char* name, const float* x, int rows, int K, const float* w, const float* b,
              int N, int act, float* y, hipStream_t st) {
  if (K % 4 == 0 && N % 4 == 0) {
    DenseFwd<true> p;
    p.M = rows; p.N = N; p.K = K; p.k_chunk = K;
    p.x = x; p.x2 = x; p.split_b = rows; p.ldx = K;
    p.w = w; p.bias = b; p.y = y; p.act = act; p.slab = nullptr;
    D4_GEMM(name, p);
  } else {
    DenseFwd<false> p;
    p.M = rows; p.N = N; p.K = K; p.k_chunk = K;
    p.x = x; p.x2 = x; p.split_b = rows; p.ldx = K;
    p.w = w; p.bias = b; p.y = y; p.act = act; p.slab = nullptr;
    D4_GEMM(name, p);
  }
  return ACME_OK;
}

// The same layer of two evaluations (rows0 / rows1 rows, weights w0 / w1) in one launch.
int dense_fwd_pair(const char* name, const float* x0, int rows0, const float* w0,
                   const float* b0, float* y0, const float* x1, int rows1, const float* w1,
                   const float* b1, float* y1, int K, int N, int act, hipStream_t st) {
  if (rows1 == 0) return dense_fwd(name, x0, rows0, K, w0, b0, N, act, y0, st);
  // The direct engine reads W by columns whatever N is; only the x rows' vector loads need
  // K % 4 == 0.
  if (K % 4 != 0) {
    int rc = dense_fwd(name, x0, rows0, K, w0, b0, N, act, y0, st);
    return rc != ACME_OK ? rc : dense_fwd(name, x1, rows1, K, w1, b1, N, act, y1, st);
  }
  DenseFwd<true> q[2];
  const float* xs[2] = {x0, x1};
  const float* ws[2] = {w0, w1};
  const float* bs[2] = {b0, b1};
  float* ys[2] = {y0, y1};
  const int rs[2] = {rows0, rows1};
  for (int i = 0; i < 2; ++i) {
    q[i].M = rs[i]; q[i].N = N; q[i].K = K; q[i].k_chunk = K;
    q[i].x = xs[i]; q[i].x2 = xs[i]; q[i].split_b = rs[i]; q[i].ldx = K;
    q[i].w = ws[i]; q[i].bias = bs[i]; q[i].y = ys[i]; q[i].act = act; q[i].slab = nullptr;
  }
  auto p = gemm::make_zset(q);
  ACME_PROF_PEAK(name, st, 2.0 * (double)(rows0 + rows1) * N * K, 0.0, 157.3);
  hipError_t e = D4_LAUNCH(p, 2);
  if (e != hipSuccess) {
    set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(e), __FILE__, __LINE__);
    return ACME_ERR_HIP;
  }
  return ACME_OK;
}

// One input set of a LayerNormMLP evaluation: rows of concat(xa, xb), the second source
// from row `split` (xa1, xb1), parameters from `prm`, activations into `acts`.
struct NetIn {
  const float* prm;
  const float *xa0, *xb0, *xa1, *xb1;
  int split, rows;
  Acts* acts;
  PolHeadSrc head[2] = {};  // critic inputs: policy heads fused into the first layer
  const float* head_prm = nullptr;  // parameters holding that policy head
};

// Two evaluations of one LayerNormMLP (the online and the target network) in one launch
// per layer: the LayerNorm first layer, the ELU layers.
int lnmlp_forward_pair(acme_d4pg* l, const NetDesc& d, const NetIn (&in)[2], int da, int db,
                       const char* tag, hipStream_t st) {
  {
    ACME_PROF(tag, st, 2.0 * (in[0].rows + in[1].rows) * (double)(da + db) * d.sizes[0], 0.0);
    LnFirstPair f;
    for (int i = 0; i < 2; ++i) {
      LnFirstArgs& g = f.a[i];
      g.xa0 = in[i].xa0; g.xb0 = in[i].xb0; g.xa1 = in[i].xa1; g.xb1 = in[i].xb1;
      g.split = in[i].split; g.rows = in[i].rows; g.da = da; g.db = db; g.H = d.sizes[0];
      g.w = P(l, in[i].prm, d.w1); g.b = P(l, in[i].prm, d.b1);
      g.scale = P(l, in[i].prm, d.scale); g.offset = P(l, in[i].prm, d.offset);
      g.eps = l->cfg.layer_norm_epsilon;
      Acts& a = *in[i].acts;
      g.z = a.z1; g.mean = a.mean; g.rstd = a.rstd; g.h = a.h[0];
      g.head[0] = in[i].head[0];
      g.head[1] = in[i].head[1];
      g.hw = in[i].head_prm ? P(l, in[i].head_prm, l->pol.ow) : nullptr;
      g.hb = in[i].head_prm ? P(l, in[i].head_prm, l->pol.ob) : nullptr;
    }
    f.lo = l->act_lo; f.scale = l->act_scale; f.Hp = l->pol.sizes[l->pol.nl - 1];
    const int rows = std::max(in[0].rows, in[1].rows);
    const int H = d.sizes[0];
    auto k = H <= 256 ? ln_first_kernel<1> : H <= 512 ? ln_first_kernel<2> : ln_first_kernel<4>;
    k<<<dim3((unsigned)ceil_div(rows, kRows), in[1].rows > 0 ? 2 : 1), 256, 0, st>>>(f);
    D4_CHECK();
  }
  for (int i = 1; i < d.nl; ++i) {
    Acts &a0 = *in[0].acts, &a1 = *in[1].acts;
    int rc = dense_fwd_pair("d4pg_mlp_fwd", a0.h[i - 1], in[0].rows, P(l, in[0].prm, d.w[i]),
                            P(l, in[0].prm, d.b[i]), a0.h[i], a1.h[i - 1], in[1].rows,
                            P(l, in[1].prm, d.w[i]), P(l, in[1].prm, d.b[i]), a1.h[i],
                            d.sizes[i - 1], d.sizes[i], ACT_ELU, st);
    if (rc != ACME_OK) return rc;
  }
  return ACME_OK;
}

// Up to two policy evaluations (TanhToSpec actions into out[i]); in[1].rows = 0: one.
int policy_forward_pair(acme_d4pg* l, const NetIn (&in)[2], float* const (&out)[2],
                        hipStream_t st) {
  const NetDesc& d = l->pol;
  int rc = lnmlp_forward_pair(l, d, in, l->cfg.obs_dim, 0, "d4pg_policy_ln", st);
  if (rc != ACME_OK) return rc;
  const int rows = std::max(in[0].rows, in[1].rows);
  ACME_PROF("d4pg_policy_head", st,
            2.0 * (in[0].rows + in[1].rows) * (double)d.sizes[d.nl - 1] * d.nout, 0.0);
  PolicyHeadPair h;
  for (int i = 0; i < 2; ++i) {
    h.a[i].h = in[i].acts->h[d.nl - 1];
    h.a[i].w = P(l, in[i].prm, d.ow);
    h.a[i].b = P(l, in[i].prm, d.ob);
    h.a[i].rows = in[i].rows;
    h.a[i].t_out = in[i].acts->t;
    h.a[i].a_out = out[i];
  }
  h.lo = l->act_lo; h.scale = l->act_scale; h.H = d.sizes[d.nl - 1]; h.A = d.nout;
  policy_head_kernel<<<dim3((unsigned)ceil_div(rows, 4), in[1].rows > 0 ? 2 : 1), 256, 0,
                       st>>>(h);
  D4_CHECK();
  return ACME_OK;
}

// The online critic (2B rows: [o_tm1, a_tm1 ; o_t, dpg actions]) and the target critic
// (B rows: [o_t, target actions]).
int critic_forward_pair(acme_d4pg* l, const NetIn (&in)[2], hipStream_t st) {
  const NetDesc& d = l->cri;
  int rc = lnmlp_forward_pair(l, d, in, l->cfg.obs_dim, l->cfg.act_dim, "d4pg_critic_ln", st);
  if (rc != ACME_OK) return rc;
  Acts &a0 = *in[0].acts, &a1 = *in[1].acts;
  return dense_fwd_pair("d4pg_critic_head", a0.h[d.nl - 1], in[0].rows, P(l, in[0].prm, d.ow),
                        P(l, in[0].prm, d.ob), a0.out, a1.h[d.nl - 1], in[1].rows,
                        P(l, in[1].prm, d.ow), P(l, in[1].prm, d.ob), a1.out,
                        d.sizes[d.nl - 1], d.nout, ACT_NONE, st);
}

inline int act_of_layer(int i) { return i == 0 ? ACT_TANH : ACT_ELU; }

// One backward launch (gemm::ZMulti): a layer's input gradient together with the weight
// gradients whose dZ is already written (the same layer's, the previous LayerNorm's first
// layer).  The problems read finished tensors and write disjoint outputs, so the weight
// gradients fill CUs the input gradient leaves idle instead of running as launches of
// their own.
struct BwdGroup {
  std::vector<DenseDgrad<true>> dg;
  std::vector<DenseDgrad<false>> dgn;  // widths not a multiple of 4 (the heads)
  std::vector<DenseWgrad<true>> wg;
  std::vector<DenseWgrad<false>> wgn;
};

// dW = X^T dZ over `rows` rows, db = column sums of dZ.
void add_wgrad(BwdGroup& g, const float* x, int rows, int Nin, const float* dz, int Nout,
               float* dw, float* db) {
  auto fill = [&](auto& p) {
    p.M = Nin; p.N = Nout; p.K = rows; p.k_chunk = rows;
    p.x = x; p.ldx = Nin; p.dz = dz; p.out = dw; p.bias_out = db;
  };
  if (Nin % 4 == 0 && Nout % 4 == 0) {
    DenseWgrad<true> p;
    fill(p);
    g.wg.push_back(p);
  } else {
    DenseWgrad<false> p;
    fill(p);
    g.wgn.push_back(p);
  }
}

// dX = act'(xprev) * (dZ @ W^T): dz [rows][Nout], W [Nin][Nout], xprev/dx [rows][Nin].
void add_dgrad(BwdGroup& g, const float* dz, int rows, int Nout, const float* w, int Nin,
               const float* xprev, int act, float* dx) {
  auto fill = [&](auto& p) {
    p.M = rows; p.N = Nin; p.K = Nout; p.k_chunk = Nout;
    p.dz = dz; p.w = w; p.xprev = xprev; p.ldx = Nin; p.dx = dx; p.act = act;
  };
  if (Nout % 4 == 0 && Nin % 4 == 0) {
    DenseDgrad<true> p;
    fill(p);
    g.dg.push_back(p);
  } else {
    DenseDgrad<false> p;
    fill(p);
    g.dgn.push_back(p);
  }
}

constexpr int kZ = 3;  // sub-problems of one type per backward launch

template <class Q>
bool fill_zset(gemm::ZSet<Q, kZ>& z, int& n, const std::vector<Q>& qs, int& tiles, int& count,
               double& flops, int& kmax) {
  if (qs.size() > (size_t)kZ) return false;
  n = (int)qs.size();
  if (!qs.empty()) static_cast<Q&>(z) = qs[0];
  for (int i = 0; i < n; ++i) {
    z.sub[i] = qs[i];
    tiles = std::max(tiles, (int)(ceil_div(qs[i].M, 32) * ceil_div(qs[i].N, 32)));
    flops += 2.0 * qs[i].M * (double)qs[i].N * qs[i].K;
    kmax = std::max(kmax, qs[i].K);
  }
  count += n;
  return true;
}

template <class Q0, class... R>
bool fill_multi(gemm::ZMulti<gemm::ZSet<Q0, kZ>, gemm::ZSet<R, kZ>...>& m, int& tiles,
                int& count, double& flops, int& kmax, const std::vector<Q0>& q0,
                const std::vector<R>&... r) {
  if (!fill_zset(m.s, m.n, q0, tiles, count, flops, kmax)) return false;
  if constexpr (sizeof...(R) > 0) return fill_multi(m.rest, tiles, count, flops, kmax, r...);
  return true;
}

// One launch over the problems of the given types (gemm_f32_multi_kernel instantiated for
// exactly these types: its LDS and registers are their maximum).
template <class... Q>
int launch_multi(const char* name, hipStream_t st, const std::vector<Q>&... qs) {
  gemm::ZMulti<gemm::ZSet<Q, kZ>...> m;
  int tiles = 0, count = 0, kmax = 0;
  double flops = 0.0;
  if (!fill_multi(m, tiles, count, flops, kmax, qs...))
    return (set_error("too many GEMMs in one backward launch"), ACME_ERR_INVALID);
  if (count == 0) return ACME_OK;
  ACME_PROF_PEAK(name, st, flops, 0.0, 157.3);
  const hipError_t e = gemm::launch_direct_multi(m, tiles, count, kmax, st);
  if (e != hipSuccess) {
    set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(e), __FILE__, __LINE__);
    return ACME_ERR_HIP;
  }
  D4_CHECK();
  return ACME_OK;
}

// The hidden layers' launches carry 4-aligned problems only; the heads' and the first
// layers' the rest.
int launch_bwd(const char* name, BwdGroup& g, hipStream_t st) {
  int rc;
  // (The concat first layer's weight gradient is two DenseWgrad problems, ln_backward.)
  if (g.dgn.empty() && g.wgn.empty())
    rc = launch_multi(name, st, g.dg, g.wg);
  else if (g.dg.empty() && g.wg.empty())
    rc = launch_multi(name, st, g.dgn, g.wgn);
  else
    rc = launch_multi(name, st, g.dg, g.wg, g.dgn, g.wgn);
  g = BwdGroup{};
  return rc;
}

// LayerNorm scale / offset gradients of the step's LayerNorms: the block partials
// [nblk][2][H] of ln_bwd_kernel, summed for both networks in one launch after the last
// one (blockIdx.y = network): 16 float4 columns x 16 partial groups per block, group g
// sums partials g, g+16, ... in order, then the groups are added in order.
struct LnReduce {
  const float* slab;
  int nblk, H;
  float *scale, *offset;
};
struct LnReducePair {
  LnReduce r[2];
};

__global__ void __launch_bounds__(256) ln_param_reduce_kernel(const LnReducePair q) {
  using f32x4 = gemm::f32x4;
  const LnReduce a = q.r[blockIdx.y];
  __shared__ f32x4 red[16][16];
  const int c = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int count4 = a.H / 2;  // 2H floats per partial row
  const int e = blockIdx.x * 16 + c;
  if (blockIdx.x * 16 >= count4) return;  // block-uniform
  const f32x4* s4 = reinterpret_cast<const f32x4*>(a.slab);
  f32x4 acc{0.f, 0.f, 0.f, 0.f};
  if (e < count4) {
#pragma unroll 8
    for (int sp = g; sp < a.nblk; sp += 16) acc += s4[(size_t)sp * count4 + e];
  }
  red[g][c] = acc;
  __syncthreads();
  if (g == 0 && e < count4) {
    f32x4 v = red[0][c];
#pragma unroll
    for (int k = 1; k < 16; ++k) v += red[k][c];
    const int h4 = a.H / 4;
    if (e < h4) reinterpret_cast<f32x4*>(a.scale)[e] = v;
    else reinterpret_cast<f32x4*>(a.offset)[e - h4] = v;
  }
}

// The same reduction as a member of the last backward launch (gemm_direct.h kCustom): a
// 512-thread block sums 16 float4 columns over 32 partial groups (group g: partials g, g+32,
// ...), then the groups in order.  M x N = 32 x (32 blocks) sizes the launch's grid.
struct LnReduceBlock {
  static constexpr bool kCustom = true;
  int M, N, K, k_chunk;
  LnReduce r;
  __device__ void run_block(int blk, float* smem) const {
    using f32x4 = gemm::f32x4;
    static_assert(gemm::kDirectWaves == 8, "512-thread blocks");
    f32x4* red = reinterpret_cast<f32x4*>(smem);  // [32][16]
    const int c = threadIdx.x & 15, g = threadIdx.x >> 4;
    const int count4 = r.H / 2;
    const int e = blk * 16 + c;
    if (blk * 16 >= count4) return;  // block-uniform
    const f32x4* s4 = reinterpret_cast<const f32x4*>(r.slab);
    f32x4 acc{0.f, 0.f, 0.f, 0.f};
    if (e < count4) {
#pragma unroll 4
      for (int sp = g; sp < r.nblk; sp += 32) acc += s4[(size_t)sp * count4 + e];
    }
    red[g * 16 + c] = acc;
    __syncthreads();
    if (g == 0 && e < count4) {
      f32x4 v = red[c];
#pragma unroll
      for (int k = 1; k < 32; ++k) v += red[k * 16 + c];
      const int h4 = r.H / 4;
      if (e < h4) reinterpret_cast<f32x4*>(r.scale)[e] = v;
      else reinterpret_cast<f32x4*>(r.offset)[e - h4] = v;
    }
  }
};

int run_ln_reduces(const std::vector<LnReduce>& ln, hipStream_t st) {
  if (ln.empty()) return ACME_OK;
  if (ln.size() > 2) return (set_error("too many LayerNorm reductions"), ACME_ERR_INVALID);
  LnReducePair q;
  int cols = 0;
  double bytes = 0.0;
  for (size_t i = 0; i < ln.size(); ++i) {
    q.r[i] = ln[i];
    cols = std::max(cols, ln[i].H / 2);
    bytes += 4.0 * (ln[i].nblk + 1) * 2.0 * ln[i].H;
  }
  ACME_PROF("d4pg_ln_param_reduce", st, 0.0, bytes);
  ln_param_reduce_kernel<<<dim3((unsigned)ceil_div(cols, 16), (unsigned)ln.size()), 256, 0, st>>>(q);
  D4_CHECK();
  return ACME_OK;
}

// The step's last backward launch and the LayerNorm parameter reductions: one launch
// (direct engine; the reductions read only ln_bwd's partials), else two.
int launch_bwd_last(const char* name, BwdGroup& g, const std::vector<LnReduce>& ln,
                    hipStream_t st) {
  std::vector<LnReduceBlock> lr;
  for (const LnReduce& x : ln) {
    LnReduceBlock b;
    b.M = 32;
    b.N = 32 * (int)ceil_div(x.H / 2, 16);
    b.K = 0;
    b.k_chunk = 0;
    b.r = x;
    lr.push_back(b);
  }
  int rc;
  if (g.dgn.empty() && g.wgn.empty())
    rc = launch_multi(name, st, g.dg, g.wg, lr);
  else
    rc = launch_multi(name, st, g.dg, g.wg, g.dgn, g.wgn, lr);
  g = BwdGroup{};
  return rc;
}

// Backward through the MLP part of a LayerNormMLP: `g` holds the launch that forms dz[nl-1]
// (the pre-activation gradient of the last hidden layer, `rows` rows) — it is issued here
// with that layer's weight gradient's predecessor problems.  Each layer's launch: its input
// gradient and its weight gradient (over the first `wrows` rows).  Leaves dLoss/d(LayerNorm
// output) in dz[0].
int lnmlp_backward_mlp(acme_d4pg* l, const NetDesc& d, const Acts& a, float* const* dz, int rows,
                       int wrows, BwdGroup& g, const char* tag, hipStream_t st) {
  int rc = launch_bwd(tag, g, st);
  for (int i = d.nl - 1; i >= 1 && rc == ACME_OK; --i) {
    add_wgrad(g, a.h[i - 1], wrows, d.sizes[i - 1], dz[i], d.sizes[i], Pm(l, l->grads, d.w[i]),
              Pm(l, l->grads, d.b[i]));
    add_dgrad(g, dz[i], rows, d.sizes[i], P(l, l->params, d.w[i]), d.sizes[i - 1], a.h[i - 1],
              act_of_layer(i - 1), dz[i - 1]);
    rc = launch_bwd("d4pg_bwd_mlp", g, st);
  }
  return rc;
}

// LayerNorm backward of the first layer; its weight gradient (concat inputs) joins the next
// backward launch, its scale/offset partials the final reductions.
int ln_backward(acme_d4pg* l, const NetDesc& d, const Acts& a, float* dy, int rows, int ce_rows,
                bool dpg, const float* xa, const float* xb, int da, int db, float* slab,
                BwdGroup& g, std::vector<LnReduce>& ln, hipStream_t st) {
  const int H = d.sizes[0];
  const int nblk = (int)ceil_div(rows, kRows);
  {
    ACME_PROF("d4pg_ln_bwd", st, 0.0, 0.0);
    LnBwdArgs b;
    b.dy = dy; b.z = a.z1; b.mean = a.mean; b.rstd = a.rstd;
    b.scale = P(l, l->params, d.scale);
    b.rows = rows; b.ce_rows = ce_rows; b.H = H; b.colslab = slab;
    b.w1 = P(l, l->params, d.w1); b.act_off = l->cfg.obs_dim; b.A = l->cfg.act_dim;
    b.clip = l->cfg.clipping ? 1.f : 0.f; b.invB = 1.f / (float)ce_rows;
    b.t = l->pon.t; b.act_scale = l->act_scale;
    b.du = l->du; b.dqda = l->dqda; b.ploss_part = dpg ? l->ploss_part : nullptr;
    const int c = H <= 256 ? 1 : H <= 512 ? 2 : 4;
    const int am = !dpg || b.A <= 4 ? 4 : b.A <= 8 ? 8 : 16;
    auto k = c == 1 ? (am == 4 ? ln_bwd_kernel<1, 4> : am == 8 ? ln_bwd_kernel<1, 8> : ln_bwd_kernel<1, 16>)
           : c == 2 ? (am == 4 ? ln_bwd_kernel<2, 4> : am == 8 ? ln_bwd_kernel<2, 8> : ln_bwd_kernel<2, 16>)
                    : (am == 4 ? ln_bwd_kernel<4, 4> : am == 8 ? ln_bwd_kernel<4, 8> : ln_bwd_kernel<4, 16>);
    k<<<(unsigned)nblk, 256, 0, st>>>(b);
    D4_CHECK();
  }
  ln.push_back({slab, nblk, H, Pm(l, l->grads, d.scale), Pm(l, l->grads, d.offset)});
  // dW1 = concat(xa, xb)^T dz: the xa rows and the xb rows of dW1 as two weight gradients
  // (strided operands); the bias gradient (column sums of dz) from the first.
  float* dw = Pm(l, l->grads, d.w1);
  add_wgrad(g, xa, ce_rows, da, dy, H, dw, Pm(l, l->grads, d.b1));
  if (db > 0) add_wgrad(g, xb, ce_rows, db, dy, H, dw + (size_t)da * H, nullptr);
  return ACME_OK;
}

int d4pg_step_impl(acme_d4pg* l, const acme_d4pg_batch* bt, const acme_d4pg_outputs* out,
                   bool copy_target, hipStream_t st) {
  const int B = (int)bt->batch;
  const int od = l->cfg.obs_dim, ad = l->cfg.act_dim;
  const NetDesc& pd = l->pol;
  const NetDesc& cd = l->cri;
  int rc;
  if (copy_target) {
    ACME_PROF("d4pg_target_copy", st, 0.0, 2.0 * 4.0 * (double)l->flat);
    ACME_HIP_TRY(hipMemcpyAsync(l->target, l->params, (size_t)l->flat * sizeof(float),
                                hipMemcpyDeviceToDevice, st));
  }
  // Forwards: the online and target evaluations of each network share every launch.
  {
    const NetIn pin[2] = {{l->params, bt->o_t, nullptr, bt->o_t, nullptr, B, B, &l->pon},
                          {l->target, bt->o_t, nullptr, bt->o_t, nullptr, B, B, &l->ptg}};
    // The policy heads run inside the critic's first-layer launch below (a launch of their
    // own measured 2 us slower per step, profiles/r05/ab/d4pg_fused_head.log).
    if ((rc = lnmlp_forward_pair(l, pd, pin, od, 0, "d4pg_policy_ln", st))) return rc;
  }
  {
    NetIn cin[2] = {{l->params, bt->o_tm1, bt->a_tm1, bt->o_t, l->pon.out, B, 2 * B, &l->con},
                    {l->target, bt->o_t, l->ptg.out, bt->o_t, l->ptg.out, B, B, &l->ctg}};
    // Online rows B.. take the online policy's actions (part 1), every target row the
    // target policy's (part 0).
    cin[0].head[1] = {l->pon.h[pd.nl - 1], l->pon.t, l->pon.out};
    cin[0].head_prm = l->params;
    cin[1].head[0] = {l->ptg.h[pd.nl - 1], l->ptg.t, l->ptg.out};
    cin[1].head_prm = l->target;
    if ((rc = critic_forward_pair(l, cin, st))) return rc;
  }
  {
    ACME_PROF("d4pg_loss", st, 0.0, 0.0);
    d4pg_loss_kernel<<<(unsigned)ceil_div(2 * B, 4), 256, 0, st>>>(
        l->con.out, l->ctg.out, bt->r_t, bt->d_t, l->values, B, cd.nout, l->cfg.discount,
        l->dlogits, l->ce);
    D4_CHECK();
  }
  // Critic backward: 2B rows of input gradients (CE rows + dpg rows), weight gradients from
  // the first B.  Launch k carries layer k's input gradient and weight gradient.
  BwdGroup g;
  std::vector<LnReduce> ln;
  const int cL = cd.nl - 1;
  add_wgrad(g, l->con.h[cL], B, cd.sizes[cL], l->dlogits, cd.nout, Pm(l, l->grads, cd.ow),
            Pm(l, l->grads, cd.ob));
  add_dgrad(g, l->dlogits, 2 * B, cd.nout, P(l, l->params, cd.ow), cd.sizes[cL], l->con.h[cL],
            act_of_layer(cL), l->cdz[cL]);
  if ((rc = lnmlp_backward_mlp(l, cd, l->con, l->cdz, 2 * B, B, g, "d4pg_bwd_head", st)) ||
      (rc = ln_backward(l, cd, l->con, l->cdz[0], 2 * B, B, true, bt->o_tm1, bt->a_tm1, od, ad,
                        l->lnslab, g, ln, st)))
    return rc;
  // Policy backward from du = dloss/d(head pre-activation); its head launch also carries the
  // critic's first-layer weight gradient.
  const int pL = pd.nl - 1;
  add_wgrad(g, l->pon.h[pL], B, pd.sizes[pL], l->du, ad, Pm(l, l->grads, pd.ow),
            Pm(l, l->grads, pd.ob));
  add_dgrad(g, l->du, B, ad, P(l, l->params, pd.ow), pd.sizes[pL], l->pon.h[pL],
            act_of_layer(pL), l->pdz[pL]);
  if ((rc = lnmlp_backward_mlp(l, pd, l->pon, l->pdz, B, B, g, "d4pg_bwd_phead", st)) ||
      (rc = ln_backward(l, pd, l->pon, l->pdz[0], B, B, false, bt->o_t, nullptr, od, 0,
                        l->lnslab2, g, ln, st)) ||
      (rc = launch_bwd_last("d4pg_wgrad_first", g, ln, st)))
    return rc;
  // Global-norm clipping + Adam (t = steps taken including this one).
  {
    ACME_PROF("d4pg_adam", st, 0.0, 7.0 * 4.0 * (double)l->flat);
    const int64_t n4 = l->flat / 4, pol4 = l->policy_flat / 4;
    int rc2 = launch_grad_sumsq(l->grads, n4, pol4, l->norm_part, kNormBlocks, l->dev_step, st);
    if (rc2 != ACME_OK) return rc2;
    ClipAdamArgs a;
    a.p = l->params; a.m = l->m; a.v = l->v; a.g = l->grads; a.n4 = n4; a.group0_4 = pol4;
    a.part = l->norm_part; a.nparts = kNormBlocks; a.clipping = l->cfg.clipping;
    a.clip_norm = 40.f;
    a.lr0 = l->cfg.policy_learning_rate; a.lr1 = l->cfg.critic_learning_rate;
    a.b1 = l->cfg.adam_beta1; a.b2 = l->cfg.adam_beta2; a.eps = l->cfg.adam_epsilon;
    a.dev_step = l->dev_step; a.norms = l->norms;
    a.sum_a = l->ploss_part; a.n_a = (int)ceil_div(2 * B, kRows); a.div_a = (float)B;
    a.out_a = out && out->policy_loss ? out->policy_loss : l->loss_tmp + 1;
    a.sum_b = l->ce; a.n_b = B; a.div_b = (float)B;
    a.out_b = out && out->critic_loss ? out->critic_loss : l->loss_tmp;
    rc2 = launch_clip_adam(a, st);
    if (rc2 != ACME_OK) return rc2;
  }
  return ACME_OK;
}

// ------------------------------------------------------------------ step graphs
// The ~40 launches of a step are captured once per (batch pointers, outputs, B, target
// copy) into a hipGraph on a private capture stream and replayed with one
// hipGraphLaunch on the caller's stream: the launch cost leaves the host critical path.
// ACME_NO_GRAPH=1 disables capture; the section profiler also bypasses it (its event
// records belong to individual launches).
bool graphs_enabled() {
  static const bool on = getenv("ACME_NO_GRAPH") == nullptr;
  return on;
}

int run_graph(acme_d4pg* l, const acme_d4pg_batch* bt, const acme_d4pg_outputs* out, bool copy,
              hipStream_t st) {
  const void* key[7] = {bt->o_tm1, bt->a_tm1, bt->r_t, bt->d_t, bt->o_t,
                        out ? out->critic_loss : nullptr, out ? out->policy_loss : nullptr};
  for (auto& g : l->graphs)
    if (g.B == bt->batch && g.copy == copy && memcmp(g.key, key, sizeof(key)) == 0) {
      ACME_HIP_TRY(hipGraphLaunch(g.exec, st));
      return ACME_OK;
    }
  if (l->graphs.size() >= 16) {  // a caller cycling many buffers: start over
    for (auto& g : l->graphs) (void)hipGraphExecDestroy(g.exec);
    l->graphs.clear();
  }
  if (!l->capture) ACME_HIP_TRY(hipStreamCreateWithFlags(&l->capture, hipStreamNonBlocking));
  ACME_HIP_TRY(hipStreamBeginCapture(l->capture, hipStreamCaptureModeRelaxed));
  int rc = d4pg_step_impl(l, bt, out, copy, l->capture);
  hipGraph_t graph = nullptr;
  hipError_t e = hipStreamEndCapture(l->capture, &graph);
  if (rc != ACME_OK) {
    if (graph) (void)hipGraphDestroy(graph);
    return rc;
  }
  if (e != hipSuccess) {
    set_error("step graph capture failed: %s", hipGetErrorString(e));
    return ACME_ERR_HIP;
  }
  hipGraphExec_t exec = nullptr;
  e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  if (e != hipSuccess) {
    set_error("step graph instantiation failed: %s", hipGetErrorString(e));
    return ACME_ERR_HIP;
  }
  acme_d4pg::Graph g;
  memcpy(g.key, key, sizeof(key));
  g.B = bt->batch;
  g.copy = copy;
  g.exec = exec;
  l->graphs.push_back(g);
  ACME_HIP_TRY(hipGraphLaunch(exec, st));
  return ACME_OK;
}

}  // namespace

extern "C" {

int acme_d4pg_destroy(acme_d4pg* l) {
  if (!l) return ACME_OK;
  (void)hipDeviceSynchronize();  // queued work of this learner finishes before its buffers go
  for (auto& g : l->graphs) (void)hipGraphExecDestroy(g.exec);
  if (l->capture) (void)hipStreamDestroy(l->capture);
  for (void* p : l->allocs) (void)hipFree(p);
  delete l;
  return ACME_OK;
}

int acme_d4pg_create(const acme_d4pg_config* cfg, acme_d4pg** out) {
  ACME_CHECK_ARG(cfg && out, "null argument");
  ACME_CHECK_ARG(cfg->obs_dim >= 1 && cfg->act_dim >= 1 && cfg->obs_dim + cfg->act_dim <= kMaxIn,
                 "obs_dim + act_dim must be in [2, %d]", kMaxIn);
  ACME_CHECK_ARG(cfg->act_dim <= ACME_D4PG_MAX_ACT, "act_dim must be <= %d", ACME_D4PG_MAX_ACT);
  ACME_CHECK_ARG(cfg->max_batch >= 1 && cfg->max_batch <= 65536, "max_batch must be in [1, 65536]");
  ACME_CHECK_ARG(cfg->num_atoms >= 2 && cfg->num_atoms <= ACME_D4PG_MAX_ATOMS,
                 "num_atoms must be in [2, %d]", ACME_D4PG_MAX_ATOMS);
  ACME_CHECK_ARG(cfg->vmax > cfg->vmin, "vmax must exceed vmin");
  ACME_CHECK_ARG(cfg->target_update_period >= 1, "target_update_period must be >= 1");
  for (int n : {cfg->num_policy_layers, cfg->num_critic_layers})
    ACME_CHECK_ARG(n >= 1 && n <= ACME_D4PG_MAX_LAYERS, "layer count must be in [1, %d]",
                   ACME_D4PG_MAX_LAYERS);
  for (int i = 0; i < cfg->num_policy_layers; ++i)
    ACME_CHECK_ARG(cfg->policy_sizes[i] >= 4 && cfg->policy_sizes[i] <= kMaxWidth &&
                       cfg->policy_sizes[i] % 4 == 0,
                   "policy layer sizes must be multiples of 4 in [4, %d]", kMaxWidth);
  for (int i = 0; i < cfg->num_critic_layers; ++i)
    ACME_CHECK_ARG(cfg->critic_sizes[i] >= 4 && cfg->critic_sizes[i] <= kMaxWidth &&
                       cfg->critic_sizes[i] % 4 == 0,
                   "critic layer sizes must be multiples of 4 in [4, %d]", kMaxWidth);
  acme_d4pg* l = new acme_d4pg();
  l->cfg = *cfg;
  auto fail = [&](int code) {
    acme_d4pg_destroy(l);
    return code;
  };
  add_net(l, l->pol, "policy", cfg->obs_dim, cfg->num_policy_layers, cfg->policy_sizes,
          cfg->act_dim, "near_zero_initialized_linear");
  l->policy_flat = l->flat;
  add_net(l, l->cri, "critic", cfg->obs_dim + cfg->act_dim, cfg->num_critic_layers,
          cfg->critic_sizes, cfg->num_atoms, "discrete_valued_head/linear");
  const int B = cfg->max_batch;
  int rc;
  int hmax = 0;
  for (int i = 0; i < cfg->num_policy_layers; ++i) hmax = std::max(hmax, cfg->policy_sizes[i]);
  for (int i = 0; i < cfg->num_critic_layers; ++i) hmax = std::max(hmax, cfg->critic_sizes[i]);
  if ((rc = alloc_acts(l, l->pon, l->pol, B, true)) || (rc = alloc_acts(l, l->ptg, l->pol, B, true)) ||
      (rc = alloc_acts(l, l->con, l->cri, 2 * B, false)) ||
      (rc = alloc_acts(l, l->ctg, l->cri, B, false)))
    return fail(rc);
  for (int i = 0; i < l->cri.nl; ++i)
    if ((rc = dev_alloc(l, &l->cdz[i], (int64_t)2 * B * l->cri.sizes[i]))) return fail(rc);
  for (int i = 0; i < l->pol.nl; ++i)
    if ((rc = dev_alloc(l, &l->pdz[i], (int64_t)B * l->pol.sizes[i]))) return fail(rc);
  const int64_t nblk = ceil_div(2 * B, kRows);
  if ((rc = dev_alloc(l, &l->dlogits, (int64_t)2 * B * cfg->num_atoms)) ||
      (rc = dev_alloc(l, &l->du, (int64_t)B * cfg->act_dim)) ||
      (rc = dev_alloc(l, &l->dqda, (int64_t)B * cfg->act_dim)) ||
      (rc = dev_alloc(l, &l->values, cfg->num_atoms)) ||
      (rc = dev_alloc(l, &l->act_lo, cfg->act_dim)) ||
      (rc = dev_alloc(l, &l->act_scale, cfg->act_dim)) ||
      (rc = dev_alloc(l, &l->lnslab, nblk * 2 * hmax)) ||
      (rc = dev_alloc(l, &l->lnslab2, nblk * 2 * hmax)) ||
      (rc = dev_alloc(l, &l->ploss_part, nblk)) ||
      (rc = dev_alloc(l, &l->norm_part, 2 * kNormBlocks)) ||
      (rc = dev_alloc(l, &l->norms, 2)) || (rc = dev_alloc(l, &l->loss_tmp, 2)) ||
      (rc = dev_alloc(l, &l->ce, B)) || (rc = dev_alloc(l, &l->dev_step, 1)))
    return fail(rc);
  // Support: tf.linspace(vmin, vmax, K) (computed in f64, rounded once to f32).
  std::vector<float> vals(cfg->num_atoms), lo(cfg->act_dim), sc(cfg->act_dim);
  const double step = ((double)cfg->vmax - (double)cfg->vmin) / (cfg->num_atoms - 1);
  for (int i = 0; i < cfg->num_atoms; ++i) vals[i] = (float)((double)cfg->vmin + i * step);
  for (int j = 0; j < cfg->act_dim; ++j) {
    lo[j] = cfg->action_min[j];
    sc[j] = cfg->action_max[j] - cfg->action_min[j];
  }
  if (hipMemset(l->dev_step, 0, sizeof(int64_t)) != hipSuccess ||
      hipMemcpy(l->values, vals.data(), vals.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(l->act_lo, lo.data(), lo.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(l->act_scale, sc.data(), sc.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
    return fail((set_error("hipMemcpy of the D4PG constants failed"), ACME_ERR_HIP));
  *out = l;
  return ACME_OK;
}

int64_t acme_d4pg_flat_size(const acme_d4pg* l) { return l ? l->flat : 0; }
int64_t acme_d4pg_policy_size(const acme_d4pg* l) { return l ? l->policy_flat : 0; }
int32_t acme_d4pg_num_tensors(const acme_d4pg* l) { return l ? (int32_t)l->tensors.size() : 0; }

int acme_d4pg_tensor_info(const acme_d4pg* l, int32_t i, int64_t* offset, int64_t* numel,
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

int acme_d4pg_bind(acme_d4pg* l, float* params, float* target, float* grads, float* adam_m,
                   float* adam_v) {
  ACME_CHECK_ARG(l, "null learner");
  ACME_CHECK_ARG(params && target && grads && adam_m && adam_v, "null buffer");
  for (const void* p : {(const void*)params, (const void*)target, (const void*)grads,
                        (const void*)adam_m, (const void*)adam_v})
    ACME_CHECK_ARG(((uintptr_t)p & 15) == 0, "buffers must be 16-byte aligned");
  // Captured graphs bake in the bound buffers: a re-bind invalidates them.
  if (!l->graphs.empty()) {
    ACME_HIP_TRY(hipDeviceSynchronize());
    for (auto& g : l->graphs) (void)hipGraphExecDestroy(g.exec);
    l->graphs.clear();
  }
  l->params = params;
  l->target = target;
  l->grads = grads;
  l->m = adam_m;
  l->v = adam_v;
  return ACME_OK;
}

int acme_d4pg_step(acme_d4pg* l, const acme_d4pg_batch* batch, const acme_d4pg_outputs* out,
                   void* stream) {
  ACME_CHECK_ARG(l && batch, "null argument");
  ACME_CHECK_ARG(l->params, "acme_d4pg_bind must be called first");
  ACME_CHECK_ARG(batch->batch >= 1 && batch->batch <= l->cfg.max_batch,
                 "batch %lld outside [1, max_batch=%d]", (long long)batch->batch,
                 l->cfg.max_batch);
  ACME_CHECK_ARG(batch->o_tm1 && batch->a_tm1 && batch->r_t && batch->d_t && batch->o_t,
                 "null batch field");
  hipStream_t st = as_stream(stream);
  const bool copy = l->num_steps % l->cfg.target_update_period == 0;
  int rc;
  if (graphs_enabled() && !prof::enabled()) {
    rc = run_graph(l, batch, out, copy, st);
  } else {
    rc = d4pg_step_impl(l, batch, out, copy, st);
  }
  if (rc != ACME_OK) return rc;
  l->num_steps += 1;
  return ACME_OK;
}

int acme_d4pg_policy(acme_d4pg* l, const float* obs, int64_t rows, int32_t use_target,
                     float* actions, void* stream) {
  ACME_CHECK_ARG(l && obs && actions, "null argument");
  ACME_CHECK_ARG(l->params, "acme_d4pg_bind must be called first");
  ACME_CHECK_ARG(rows >= 0, "negative row count");
  hipStream_t st = as_stream(stream);
  const int B = l->cfg.max_batch;
  for (int64_t r0 = 0; r0 < rows; r0 += B) {
    const int n = (int)std::min<int64_t>(B, rows - r0);
    const float* o = obs + r0 * l->cfg.obs_dim;
    const NetIn in[2] = {{use_target ? l->target : l->params, o, nullptr, o, nullptr, n, n,
                          &l->ptg},
                         {l->params, o, nullptr, o, nullptr, n, 0, &l->ptg}};
    float* const out[2] = {actions + r0 * l->cfg.act_dim, nullptr};
    int rc = policy_forward_pair(l, in, out, st);
    if (rc != ACME_OK) return rc;
  }
  return ACME_OK;
}

int64_t acme_d4pg_num_steps(const acme_d4pg* l) { return l ? l->num_steps : 0; }
int acme_d4pg_set_num_steps(acme_d4pg* l, int64_t n) {
  ACME_CHECK_ARG(l && n >= 0, "bad argument");
  ACME_HIP_TRY(hipDeviceSynchronize());
  ACME_HIP_TRY(hipMemcpy(l->dev_step, &n, sizeof(n), hipMemcpyHostToDevice));
  l->num_steps = n;
  return ACME_OK;
}

int acme_d4pg_debug_buffer(const acme_d4pg* l, const char* name, const float** out,
                           int64_t* count) {
  ACME_CHECK_ARG(l && name && out && count, "null argument");
  const int B = l->cfg.max_batch, A = l->cfg.act_dim, K = l->cfg.num_atoms;
  struct Item {
    const char* n;
    const float* p;
    int64_t c;
  } items[] = {
      {"p_a", l->pon.out, (int64_t)B * A},      {"t_a", l->ptg.out, (int64_t)B * A},
      {"c_logits", l->con.out, (int64_t)2 * B * K}, {"t_logits", l->ctg.out, (int64_t)B * K},
      {"dlogits", l->dlogits, (int64_t)2 * B * K},  {"dqda", l->dqda, (int64_t)B * A},
      {"du", l->du, (int64_t)B * A},             {"norms", l->norms, 2},
      {"losses", l->loss_tmp, 2},
  };
  for (const Item& it : items)
    if (strcmp(it.n, name) == 0) {
      *out = it.p;
      *count = it.c;
      return ACME_OK;
    }
  set_error("unknown debug buffer '%s'", name);
  return ACME_ERR_INVALID;
}

}  // extern "C"
