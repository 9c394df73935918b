// Fused small kernels of the learner step: duelling head fwd/bwd, DQN loss, bias-grad
// column sums, split-K slab reductions, snt.Adam.
#include "kernels.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "common.h"

namespace acme {
namespace {

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

// One wave per row: lane a < A computes advantage a, lane 63 the value.
__global__ void __launch_bounds__(256) duel_head_kernel(const float* __restrict__ h, int rows,
                                                        int H, int A, const float* __restrict__ wv,
                                                        const float* __restrict__ bv,
                                                        const float* __restrict__ wa,
                                                        const float* __restrict__ ba,
                                                        float* __restrict__ q) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* hv = h + (size_t)row * 2 * H;
  const float* ha = hv + H;
  float acc = 0.f;
  if (lane < A) {
    for (int k = 0; k < H; ++k) acc = fmaf(ha[k], wa[k * A + lane], acc);
    acc += ba[lane];
  } else if (lane == 63) {
    for (int k = 0; k < H; ++k) acc = fmaf(hv[k], wv[k], acc);
    acc += bv[0];
  }
  const float v = __shfl(acc, 63, 64);
  const float adv_sum = wave_sum(lane < A ? acc : 0.f);
  const float mean = adv_sum / (float)A;
  if (lane < A) q[(size_t)row * A + lane] = v + (acc - mean);
}

// dZ of the fused hidden layer: thread per (b, k).
__global__ void duel_head_dz_kernel(const float* __restrict__ h, const float* __restrict__ g,
                                    const int32_t* __restrict__ a, int B, int H, int A,
                                    const float* __restrict__ wv, const float* __restrict__ wa,
                                    float* __restrict__ dzh) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * 2 * H) return;
  const int b = (int)(i / (2 * H));
  const int k = (int)(i - (int64_t)b * 2 * H);
  const float gb = g[b];
  float d;
  if (k < H) {
    d = gb * wv[k];  // dv = sum_a dq_a = g_b
  } else {
    // dadv_j = g_b (1[j == a_b] - 1/A);  dh_k = sum_j dadv_j wa[k][j]
    const float* row = wa + (size_t)(k - H) * A;
    const float inv_a = 1.f / (float)A;
    const int ab = a[b];
    float s = 0.f;
    for (int j = 0; j < A; ++j) s = fmaf(gb * ((j == ab ? 1.f : 0.f) - inv_a), row[j], s);
    d = s;
  }
  dzh[i] = h[i] > 0.f ? d : 0.f;
}

// Head weight/bias gradients: one thread per output column c.
//   c < H               : dwv[c]     = sum_b hv[b][c] g_b
//   H <= c < H + H*A    : dwa[k][j]  = sum_b ha[b][k] g_b (1[j==a_b] - 1/A)
//   c == H + H*A        : dbv        = sum_b g_b
//   next A columns      : dba[j]     = sum_b g_b (1[j==a_b] - 1/A)
__global__ void duel_head_wgrad_kernel(const float* __restrict__ h, const float* __restrict__ g,
                                       const int32_t* __restrict__ a, int B, int H, int A,
                                       float* __restrict__ dwv, float* __restrict__ dbv,
                                       float* __restrict__ dwa, float* __restrict__ dba) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = H + H * A + 1 + A;
  if (c >= total) return;
  const float inv_a = 1.f / (float)A;
  float s = 0.f;
  if (c < H) {
    for (int b = 0; b < B; ++b) s = fmaf(h[(size_t)b * 2 * H + c], g[b], s);
    dwv[c] = s;
  } else if (c < H + H * A) {
    const int k = (c - H) / A, j = (c - H) % A;
    for (int b = 0; b < B; ++b) {
      const float dadv = g[b] * ((j == a[b] ? 1.f : 0.f) - inv_a);
      s = fmaf(h[(size_t)b * 2 * H + H + k], dadv, s);
    }
    dwa[(size_t)k * A + j] = s;
  } else if (c == H + H * A) {
    for (int b = 0; b < B; ++b) s += g[b];
    dbv[0] = s;
  } else {
    const int j = c - (H + H * A + 1);
    for (int b = 0; b < B; ++b) s += g[b] * ((j == a[b] ? 1.f : 0.f) - inv_a);
    dba[j] = s;
  }
}

__global__ void onehot_dq_kernel(const float* __restrict__ g, const int32_t* __restrict__ a,
                                 int B, int A, float* __restrict__ dz) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * A) return;
  const int b = i / A, j = i - b * A;
  dz[i] = j == a[b] ? g[b] : 0.f;
}

constexpr int kLossThreads = 1024;

__global__ void __launch_bounds__(kLossThreads) dqn_loss_kernel(LossArgs p) {
  __shared__ double red[kLossThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nw = blockDim.x >> 6;
  const int B = p.B, A = p.A;
  // 1. Importance-weight normaliser: max_b (1/p_b)^beta = (1/min_b p_b)^beta.
  double pmin = INFINITY;
  for (int b = tid; b < B; b += blockDim.x) pmin = fmin(pmin, p.probs[b]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pmin = fmin(pmin, __shfl_xor(pmin, o, 64));
  if (lane == 0) red[wave] = pmin;
  __syncthreads();
  if (tid == 0) {
    double m = red[0];
    for (int w = 1; w < nw; ++w) m = fmin(m, red[w]);
    red[0] = m;
  }
  __syncthreads();
  pmin = p.global_min_prob ? *p.global_min_prob : red[0];
  __syncthreads();
  const double wmax = pow(1.0 / pmin, (double)p.beta);
  const float inv_b = 1.f / (float)B;
  double lsum = 0.0;
  for (int b = tid; b < B; b += blockDim.x) {
    const float* qt = p.q_on + (size_t)b * A;
    const float* qs = p.q_on + (size_t)(B + b) * A;
    const float* qv = p.q_tg + (size_t)b * A;
    int best = 0;  // tf.argmax: first maximal index
    float bq = qs[0];
    for (int j = 1; j < A; ++j)
      if (qs[j] > bq) {
        bq = qs[j];
        best = j;
      }
    float r = p.r[b];
    r = fminf(fmaxf(r, -p.max_abs_reward), p.max_abs_reward);
    const float dg = __fmul_rn(p.d[b], p.discount);
    const float target = __fadd_rn(r, __fmul_rn(dg, qv[best]));
    const int ab = p.a[b];
    const float td = __fsub_rn(target, qt[ab]);
    const float ax = fabsf(td);
    const float quad = fminf(ax, p.delta);
    const float lin = ax - quad;
    const float hub = __fadd_rn(__fmul_rn(0.5f, __fmul_rn(quad, quad)), __fmul_rn(p.delta, lin));
    const double w = pow(1.0 / p.probs[b], (double)p.beta) / wmax;
    const float wf = (float)w;
    lsum += (double)(hub * wf);
    const float dtd = fminf(fmaxf(td, -p.delta), p.delta);  // d huber / d td
    p.g[b] = -(inv_b * wf * dtd);
    p.td[b] = td;
    p.prio[b] = (double)ax;
    p.a_cache[b] = ab;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lsum += __shfl_xor(lsum, o, 64);
  if (lane == 0) red[wave] = lsum;
  __syncthreads();
  if (tid == 0) {
    double s = 0.0;
    for (int w = 0; w < nw; ++w) s += red[w];
    p.loss[0] = (float)(s / (double)B);
  }
}

__global__ void colsum_partial_kernel(const float* __restrict__ dz, int64_t rows, int n,
                                      int64_t rows_per_chunk, float* __restrict__ partial) {
  extern __shared__ float sm[];
  const int chunk = blockIdx.x;
  const int64_t r0 = (int64_t)chunk * rows_per_chunk;
  const int64_t r1 = min(rows, r0 + rows_per_chunk);
  const int tid = threadIdx.x;
  if (n >= (int)blockDim.x) {
    for (int c = tid; c < n; c += blockDim.x) {
      float s = 0.f;
      for (int64_t r = r0; r < r1; ++r) s += dz[r * n + c];
      partial[(size_t)chunk * n + c] = s;
    }
    return;
  }
  const int lanes = blockDim.x / n;
  const int col = tid % n, rl = tid / n;
  float s = 0.f;
  if (rl < lanes)
    for (int64_t r = r0 + rl; r < r1; r += lanes) s += dz[r * n + col];
  if (rl < lanes) sm[rl * n + col] = s;
  __syncthreads();
  if (tid < n) {
    float t = 0.f;
    for (int k = 0; k < lanes; ++k) t += sm[k * n + tid];
    partial[(size_t)chunk * n + tid] = t;
  }
}

__global__ void slab_reduce_kernel(const float* __restrict__ slab, int splits, int64_t count,
                                   float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += slab[(size_t)k * count + i];
  out[i] = s;
}

using f32x4 = __attribute__((ext_vector_type(4))) float;

// snt.optimizers.Adam (Kingma & Ba Algorithm 1 form):
//   m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g g
//   p -= lr * (m / (1 - b1^t)) / (sqrt(v / (1 - b2^t)) + eps)
__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p,
                                                   const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   int64_t n4, float lr, float b1, float omb1,
                                                   float b2, float omb2, float bc1, float bc2,
                                                   float eps) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 gg = reinterpret_cast<const f32x4*>(g)[i];
    f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
    f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float mj = __fadd_rn(__fmul_rn(b1, mm[j]), __fmul_rn(omb1, gg[j]));
      const float vj = __fadd_rn(__fmul_rn(b2, vv[j]), __fmul_rn(omb2, __fmul_rn(gg[j], gg[j])));
      const float mh = __fdiv_rn(mj, bc1);
      const float vh = __fdiv_rn(vj, bc2);
      const float upd = __fdiv_rn(__fmul_rn(lr, mh), __fadd_rn(__fsqrt_rn(vh), eps));
      mm[j] = mj;
      vv[j] = vj;
      pp[j] = __fsub_rn(pp[j], upd);
    }
    reinterpret_cast<f32x4*>(m)[i] = mm;
    reinterpret_cast<f32x4*>(v)[i] = vv;
    reinterpret_cast<f32x4*>(p)[i] = pp;
  }
}

__global__ void min_f64_kernel(const double* __restrict__ x, int64_t n, double* out) {
  __shared__ double red[16];
  double m = INFINITY;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) m = fmin(m, x[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmin(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) m = fmin(m, red[w]);
    m = fmin(m, red[0]);
    *out = m;
  }
}

}  // namespace

int launch_duel_head(const float* h, int rows, int H, int A, const float* wv, const float* bv,
                     const float* wa, const float* ba, float* q, hipStream_t st) {
  duel_head_kernel<<<(unsigned)ceil_div(rows, 4), 256, 0, st>>>(h, rows, H, A, wv, bv, wa, ba, q);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_duel_head_backward(const float* h, const float* g, const int32_t* a, int B, int H,
                              int A, const float* wv, const float* wa, float* dzh, float* dwv,
                              float* dbv, float* dwa, float* dba, hipStream_t st) {
  const int64_t n = (int64_t)B * 2 * H;
  duel_head_dz_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(h, g, a, B, H, A, wv, wa, dzh);
  ACME_LAUNCH_CHECK();
  const int total = H + H * A + 1 + A;
  duel_head_wgrad_kernel<<<(unsigned)ceil_div(total, 256), 256, 0, st>>>(h, g, a, B, H, A, dwv,
                                                                         dbv, dwa, dba);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_onehot_dq(const float* g, const int32_t* a, int B, int A, float* dz, hipStream_t st) {
  onehot_dq_kernel<<<(unsigned)ceil_div((int64_t)B * A, 256), 256, 0, st>>>(g, a, B, A, dz);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_dqn_loss(const LossArgs& args, hipStream_t st) {
  dqn_loss_kernel<<<1, kLossThreads, 0, st>>>(args);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_colsum(const float* dz, int64_t rows, int n, int chunks, float* partial, float* out,
                  hipStream_t st) {
  ACME_CHECK_ARG(n >= 1 && chunks >= 1, "bad colsum shape");
  const int64_t per = ceil_div(rows, chunks);
  const size_t shm = n < 256 ? 256 * sizeof(float) : 0;
  colsum_partial_kernel<<<chunks, 256, shm, st>>>(dz, rows, n, per, partial);
  ACME_LAUNCH_CHECK();
  return launch_slab_reduce(partial, chunks, n, out, st);
}

int launch_slab_reduce(const float* slab, int splits, int64_t count, float* out, hipStream_t st) {
  slab_reduce_kernel<<<(unsigned)ceil_div(count, 256), 256, 0, st>>>(slab, splits, count, out);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

}  // namespace acme

extern "C" {

int acme_adam_update(float* params, const float* grads, float* m, float* v, int64_t n, float lr,
                     float beta1, float beta2, float eps, int64_t t, void* stream) {
  ACME_CHECK_ARG(params && grads && m && v, "null buffer");
  ACME_CHECK_ARG(n % 4 == 0, "adam buffer length must be a multiple of 4");
  ACME_CHECK_ARG(t >= 1, "adam step must be >= 1");
  const float omb1 = 1.f - beta1, omb2 = 1.f - beta2;
  const float bc1 = 1.f - powf(beta1, (float)t);
  const float bc2 = 1.f - powf(beta2, (float)t);
  const int64_t n4 = n / 4;
  const unsigned grid = (unsigned)std::min<int64_t>(acme::ceil_div(n4, 256), 2048);
  acme::adam_kernel<<<grid, 256, 0, acme::as_stream(stream)>>>(params, grads, m, v, n4, lr, beta1,
                                                                omb1, beta2, omb2, bc1, bc2, eps);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int acme_min_f64(const double* x, int64_t n, double* out_dev, void* stream) {
  ACME_CHECK_ARG(x && out_dev && n >= 1, "bad argument");
  acme::min_f64_kernel<<<1, 1024, 0, acme::as_stream(stream)>>>(x, n, out_dev);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

}  // extern "C"
