// Fused small kernels of the learner step: duelling head fwd/bwd, DQN loss, bias-grad
// column sums, split-K slab reductions, snt.Adam.
#include "kernels.h"
#include "rescale.h"

#include "conv.h"
#include "gemm_p3.h"
#include "gemm_x6.h"

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

// Duelling head epilogue: one wave per row; lane j <= A sums the split-K partials of
// output j (fixed split order) and adds its bias; lane A holds the value.
__global__ void __launch_bounds__(256) duel_head_finish_kernel(const float* __restrict__ slab,
                                                               int splits, int rows, int A,
                                                               const float* __restrict__ bv,
                                                               const float* __restrict__ ba,
                                                               float* __restrict__ q) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int N = A + 1;
  float acc = 0.f;
  if (lane <= A) {
    for (int s = 0; s < splits; ++s) acc += slab[((size_t)s * rows + row) * N + lane];
    acc += lane < A ? ba[lane] : bv[0];
  }
  const float v = __shfl(acc, A, 64);
  const float mean = wave_sum(lane < A ? acc : 0.f) / (float)A;
  if (lane < A) q[(size_t)row * A + lane] = v + (acc - mean);
}

// dZ of the fused hidden layer: thread per (b, k).
__global__ void duel_head_dz_kernel(const float* __restrict__ h, const float* __restrict__ g,
                                    const int32_t* __restrict__ a, int B, int H, int A,
                                    const float* __restrict__ wv, const float* __restrict__ wa,
                                    float* __restrict__ dzh, uint16_t* __restrict__ planes,
                                    int64_t pstride, gemm::PScale* sc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * 2 * H) return;  // (the plane path uses head_dz_planes_kernel)
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
  const float z = h[i] > 0.f ? d : 0.f;
  if (planes) gemm::Planes{planes, pstride, sc}.put(i, z);
  else dzh[i] = z;
}

// Sum of the DuelHeadWgrad slab + scatter of its block-diagonal parts.
// Sum of the fused loss kernel's per-block loss partials over 256 threads, divided by
// mean_over (one fixed order: strided per thread, then the wave tree, then the waves).
__device__ __forceinline__ void loss_sum_block(const double* __restrict__ part, int64_t n,
                                               int mean_over, float* __restrict__ loss) {
  __shared__ double red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double s = 0.0;
  for (int64_t i = tid; i < n; i += 256) s += part[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  if (tid == 0) loss[0] = (float)((((red[0] + red[1]) + red[2]) + red[3]) / (double)mean_over);
}

// The head weight gradients from the split-K slab; with `part`, one extra (last) block forms
// the batch loss from the fused loss kernel's partials (the loss-sum launch folded in).
__global__ void __launch_bounds__(256) duel_head_grad_scatter_kernel(
    const float* __restrict__ slab, int splits, int H, int A, float* __restrict__ dwv,
    float* __restrict__ dbv, float* __restrict__ dwa, float* __restrict__ dba,
    const double* __restrict__ part, int64_t nparts, int mean_over, float* __restrict__ loss) {
  if (part && blockIdx.x == gridDim.x - 1) {
    loss_sum_block(part, nparts, mean_over, loss);
    return;
  }
  const int N = A + 1;
  const int64_t count = (int64_t)(2 * H + 1) * N;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  const int k = (int)(e / N), n = (int)(e - (int64_t)k * N);
  const bool value_w = k < H && n == A, adv_w = k >= H && k < 2 * H && n < A, bias = k == 2 * H;
  if (!(value_w || adv_w || bias)) return;
  float s = 0.f;
  for (int sp = 0; sp < splits; ++sp) s += slab[(size_t)sp * count + e];
  if (value_w) dwv[k] = s;
  else if (adv_w) dwa[(size_t)(k - H) * A + n] = s;
  else if (n == A) dbv[0] = s;
  else dba[n] = s;
}

__global__ void onehot_dq_kernel(const float* __restrict__ g, const int32_t* __restrict__ a,
                                 int B, int A, float* __restrict__ dz) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * A) return;
  const int b = i / A, j = i - b * A;
  dz[i] = j == a[b] ? g[b] : 0.f;
}

constexpr int kLossThreads = 1024;

// One transition of the loss: reward clip, discount, double-Q target, TD, Huber, f64
// importance weight; shared by the loss kernel and the fused loss + head dZ kernel so both
// produce the same bits.
struct LossRow {
  float g, td, hub_w;
};
__device__ __forceinline__ LossRow loss_row(const LossArgs& p, int b, double wmax) {
  const int B = p.B, A = p.A;
  const float* qt = p.q_on + (size_t)b * A;
  const float* qs = p.q_on + (size_t)(B + b) * A;
  const float* qv = p.q_tg + (size_t)b * A;
  // The row's scalars first (and q_tm1[a], which depends only on a), so their latency
  // overlaps the argmax's loads.
  const int ab = p.a[b];
  float r = p.r[b];
  const float dgv = p.d[b];
  const double prob = p.probs[b];
  const float qa = qt[ab];
  // tf.argmax: first maximal index.  The selector row is read 8 entries at a time, all 8
  // loads issued before the compares (clamped addresses): one latency per 8 actions
  // instead of one per action.
  int best = 0;
  float bq = 0.f;
  for (int j0 = 0; j0 < A; j0 += 8) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = qs[min(j0 + k, A - 1)];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int j = j0 + k;
      if (j == 0) {
        bq = v[k];
      } else if (j < A && v[k] > bq) {
        bq = v[k];
        best = j;
      }
    }
  }
  r = fminf(fmaxf(r, -p.max_abs_reward), p.max_abs_reward);
  const float dg = __fmul_rn(dgv, p.discount);
  const float target = __fadd_rn(r, __fmul_rn(dg, qv[best]));
  const float td = __fsub_rn(target, qa);
  const float ax = fabsf(td);
  const float quad = fminf(ax, p.delta);
  const float lin = ax - quad;
  const float hub = __fadd_rn(__fmul_rn(0.5f, __fmul_rn(quad, quad)), __fmul_rn(p.delta, lin));
  float wf;
  if (p.jax) {  // ((1 / probs).astype(f32) ** beta) / max, all in f32 (jax/dqn/learning.py:94-96)
    wf = __fdiv_rn(powf((float)(1.0 / prob), p.beta), (float)wmax);
  } else {      // f64 weights cast at the multiply (tf/dqn/learning.py:138-143)
    wf = (float)(pow(1.0 / prob, (double)p.beta) / wmax);
  }
  const float dtd = fminf(fmaxf(td, -p.delta), p.delta);  // d huber / d td
  const float inv_b = 1.f / (float)p.mean_over;
  return LossRow{-(inv_b * wf * dtd), td, hub * wf};
}

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
  const double wmax = p.jax ? (double)powf((float)(1.0 / pmin), p.beta)
                            : pow(1.0 / pmin, (double)p.beta);
  double lsum = 0.0;
  for (int b = tid; b < B; b += blockDim.x) {
    const LossRow row = loss_row(p, b, wmax);
    lsum += (double)row.hub_w;
    p.g[b] = row.g;
    p.td[b] = row.td;
    p.prio[b] = (double)fabsf(row.td);
    p.a_cache[b] = p.a[b];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lsum += __shfl_xor(lsum, o, 64);
  if (lane == 0) red[wave] = lsum;
  __syncthreads();
  if (tid == 0) {
    double s = 0.0;
    for (int w = 0; w < nw; ++w) s += red[w];
    p.loss[0] = (float)(s / (double)p.mean_over);
  }
}

// Deterministic split-K reduction: 64 outputs x 4 split groups per 256-thread block;
// group g sums splits g, g+4, ... (coalesced 256-B rows per wave), then the four group
// partials are added in order.
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ slab,
                                                          int splits, int64_t count,
                                                          float* __restrict__ out0,
                                                          int64_t split_at,
                                                          float* __restrict__ out1,
                                                          const float* __restrict__ bias,
                                                          int ncols, int relu) {
  __shared__ float red[4][64];
  const int o = threadIdx.x & 63, gr = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + o;
  float s = 0.f;
  if (e < count)
    for (int sp = gr; sp < splits; sp += 4) s += slab[(size_t)sp * count + e];
  red[gr][o] = s;
  __syncthreads();
  if (gr == 0 && e < count) {
    float v = ((red[0][o] + red[1][o]) + red[2][o]) + red[3][o];
    if (bias) {
      v += bias[e % ncols];
      if (relu) v = v > 0.f ? v : 0.f;
    }
    if (e < split_at) out0[e] = v;
    else out1[e - split_at] = v;
  }
}

using f32x4 = __attribute__((ext_vector_type(4))) float;

// Planes of 4 consecutive floats (element 4i .. 4i+3) scaled by w, 8-byte stores per
// plane; returns max |x|.
__device__ __forceinline__ float store_planes4(uint16_t* planes, int64_t pstride, int64_t i,
                                               const f32x4 x, float w) {
  uint16_t h[4], l[4];
  float mx = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    gemm::split2_bits(x[j] * w, h[j], l[j]);
    mx = gemm::amax_max(mx, fabsf(x[j]));
  }
  auto pack = [](const uint16_t* q) {
    return uint2{(uint32_t)q[0] | ((uint32_t)q[1] << 16), (uint32_t)q[2] | ((uint32_t)q[3] << 16)};
  };
  reinterpret_cast<uint2*>(planes)[i] = pack(h);
  reinterpret_cast<uint2*>(planes + pstride)[i] = pack(l);
  return mx;
}

// snt.optimizers.Adam (Kingma & Ba Algorithm 1 form):
//   m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g g
//   p -= lr * (m / (1 - b1^t)) / (sqrt(v / (1 - b2^t)) + eps)
// Vectorised deterministic split-K reduction (count, split_at, ncols multiples of 4):
// 16 float4 columns x 16 split groups per 256-thread block; group g sums splits g, g+16,
// ... in order, then the groups are added in order.
__global__ void __launch_bounds__(256) slab_reduce4_kernel(const float* __restrict__ slab,
                                                           int splits, int64_t count4,
                                                           float* __restrict__ out0,
                                                           int64_t split_at4,
                                                           float* __restrict__ out1,
                                                           const float* __restrict__ bias,
                                                           int ncols, int relu) {
  __shared__ f32x4 red[16][16];
  const int c = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int64_t e = (int64_t)blockIdx.x * 16 + c;
  const f32x4* s4 = reinterpret_cast<const f32x4*>(slab);
  f32x4 acc{0.f, 0.f, 0.f, 0.f};
  if (e < count4) {
    // Loads issued 8 ahead (the adds keep their order, so the sum is unchanged).
#pragma unroll 8
    for (int sp = g; sp < splits; sp += 16) acc += s4[(size_t)sp * count4 + e];
  }
  red[g][c] = acc;
  __syncthreads();
  if (g == 0 && e < count4) {
    f32x4 v = red[0][c];
#pragma unroll
    for (int q = 1; q < 16; ++q) v += red[q][c];
    if (bias) {
      const int col = (int)((e * 4) % ncols);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] += bias[col + j];
        if (relu) v[j] = v[j] > 0.f ? v[j] : 0.f;
      }
    }
    if (e < split_at4) reinterpret_cast<f32x4*>(out0)[e] = v;
    else reinterpret_cast<f32x4*>(out1)[e - split_at4] = v;
  }
}

// Fused hidden-layer finish + duelling head (DQN forward): per row, hid = relu(sum of the
// split-K slab + bias) (written out for the backward), then
// q = v + adv - mean(adv) with v = hid[:H] . wv + bv, adv_j = hid[H:] . wa[:, j] + ba_j
// (acme/tf/networks/duelling.py:51-57).  4 rows per 256-thread block: the advantage
// weights are staged once per block in LDS, each wave finishes one row with lane-parallel
// partial dot products and a fixed shuffle tree (deterministic).
constexpr int kHeadRows = 4;
constexpr int kHeadChunk = 8;  // advantage outputs per accumulation pass
template <int SPL, int HC>
__global__ void __launch_bounds__(256) fc_head_forward_kernel(
    const float* __restrict__ slab, int splits, int rows, int H_, const float* __restrict__ fcb,
    const float* __restrict__ wv, const float* __restrict__ bv, const float* __restrict__ wa,
    const float* __restrict__ ba, int A, float* __restrict__ hid, float* __restrict__ q) {
  const int H = HC > 0 ? HC : H_;  // compile-time hidden width when HC > 0
  // [kHeadRows][2H] hid | [H][A] wa | [H] wv | [kHeadRows][A + 1] dots | 4 x [8][64] partials
  extern __shared__ float sh[];
  float* swa = sh + kHeadRows * 2 * H;
  float* swv = swa + H * A;
  float* dots = swv + H;
  const int r0 = blockIdx.x * kHeadRows;
  const int n4 = 2 * H / 4;
  const int64_t count4 = (int64_t)rows * n4;
  const f32x4* s4 = reinterpret_cast<const f32x4*>(slab);
  if ((H * A) % 4 == 0) {
    const int n = H * A / 4;
#pragma unroll 4
    for (int t = threadIdx.x; t < n; t += 256)
      reinterpret_cast<f32x4*>(swa)[t] = reinterpret_cast<const f32x4*>(wa)[t];
  } else {
    for (int t = threadIdx.x; t < H * A; t += 256) swa[t] = wa[t];
  }
  for (int t = threadIdx.x; t < H; t += 256) swv[t] = wv[t];
#pragma unroll
  for (int t = threadIdx.x; t < kHeadRows * n4; t += 256) {
    const int rr = t / n4, c4 = t - rr * n4;
    const int row = r0 + rr;
    if (row >= rows) continue;
    const int64_t e = (int64_t)row * n4 + c4;
    f32x4 v;
    if constexpr (SPL > 0) {
      f32x4 part[SPL];
#pragma unroll
      for (int sp = 0; sp < SPL; ++sp) part[sp] = s4[(size_t)sp * count4 + e];
      v = part[0];
#pragma unroll
      for (int sp = 1; sp < SPL; ++sp) v += part[sp];
    } else {
      v = s4[e];
      for (int sp = 1; sp < splits; ++sp) v += s4[(size_t)sp * count4 + e];
    }
    const f32x4 b = reinterpret_cast<const f32x4*>(fcb)[c4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const float x = v[jj] + b[jj];
      v[jj] = x > 0.f ? x : 0.f;
    }
    reinterpret_cast<f32x4*>(hid)[e] = v;
    reinterpret_cast<f32x4*>(sh + rr * 2 * H)[c4] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // Outputs o = 0..A (o < A: advantage o, o == A: value), kHeadChunk at a time: each lane
  // accumulates its strided k-slice, the 64 partials go through a per-wave LDS row, and
  // lane jj sums output jj's row in a fixed order (no cross-lane shuffle chains).
  float* red = dots + kHeadRows * (A + 1) + wave * kHeadChunk * 64;
  float* zero = dots + kHeadRows * (A + 1) + 4 * kHeadChunk * 64;  // one zero word
  if (threadIdx.x == 0) zero[0] = 0.f;
  __syncthreads();
  for (int rr = wave; rr < kHeadRows; rr += 4) {
    const float* h = sh + rr * 2 * H;
    for (int o0 = 0; o0 <= A; o0 += kHeadChunk) {
      // Per-output weight column (uniform): advantage o -> wa[:, o] (stride A) over
      // hid[H:]; value -> wv (stride 1) over hid[:H]; past the end -> a zero word.
      const float* wp[kHeadChunk];
      int ws[kHeadChunk], hoff[kHeadChunk];
#pragma unroll
      for (int jj = 0; jj < kHeadChunk; ++jj) {
        const int o = o0 + jj;
        wp[jj] = o < A ? swa + o : (o == A ? swv : zero);
        ws[jj] = o < A ? A : (o == A ? 1 : 0);
        hoff[jj] = o < A ? H : 0;
      }
      float acc[kHeadChunk];
#pragma unroll
      for (int jj = 0; jj < kHeadChunk; ++jj) acc[jj] = 0.f;
#pragma unroll 8
      for (int k = lane; k < H; k += 64) {
#pragma unroll
        for (int jj = 0; jj < kHeadChunk; ++jj)
          acc[jj] = fmaf(h[hoff[jj] + k], wp[jj][k * ws[jj]], acc[jj]);
      }
#pragma unroll
      for (int jj = 0; jj < kHeadChunk; ++jj) red[jj * 64 + lane] = acc[jj];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lane < kHeadChunk && o0 + lane <= A) {
        const f32x4* r4 = reinterpret_cast<const f32x4*>(red + lane * 64);
        f32x4 t = r4[0];
#pragma unroll
        for (int q = 1; q < 16; ++q) t += r4[q];
        const int o = o0 + lane;
        dots[rr * (A + 1) + o] = ((t[0] + t[1]) + (t[2] + t[3])) + (o == A ? bv[0] : ba[o]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  __syncthreads();
  if (threadIdx.x < kHeadRows) {
    const int rr = threadIdx.x, row = r0 + rr;
    if (row < rows) {
      const float* d = dots + rr * (A + 1);
      float mean = 0.f;
      for (int jj = 0; jj < A; ++jj) mean += d[jj];
      mean /= (float)A;
      for (int jj = 0; jj < A; ++jj) q[(size_t)row * A + jj] = d[A] + (d[jj] - mean);
    }
  }
}

// The same for the Nature head (2H = 1024 hidden units, compile-time A): thread t owns hidden
// columns [4t, 4t + 4) of the block's R rows, so the split-K sum, bias and ReLU land in its
// registers and the row's dot products start from them (t < 128: the value half against
// wv; t >= 128: the advantage half against its 4 rows of wa, A float4 loads issued with the
// slab loads).  Per-thread partials go through LDS and each output is summed by one wave in
// a fixed order (lane pairs, then a shuffle tree), so the result is deterministic.  One
// wait for every global load of the block.  Launched with R = 1 row per block.
template <int SPL, int A, int R>
__global__ void __launch_bounds__(256) fc_head1024_kernel(
    const float* __restrict__ slab, int rows, const float* __restrict__ fcb,
    const float* __restrict__ wv, const float* __restrict__ bv, const float* __restrict__ wa,
    const float* __restrict__ ba, float* __restrict__ hid, float* __restrict__ q) {
  constexpr int N4 = 256, HALF = 128;
  __shared__ float part[R][A + 1][HALF];
  __shared__ float dots[R][A + 1];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int r0 = blockIdx.x * R;
  const int64_t count4 = (int64_t)rows * N4;
  const f32x4* s4 = reinterpret_cast<const f32x4*>(slab);
  f32x4 sp[R][SPL];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int row = r0 + r < rows ? r0 + r : rows - 1;  // a clamped duplicate, never stored
    const int64_t e = (int64_t)row * N4 + t;
#pragma unroll
    for (int k = 0; k < SPL; ++k) sp[r][k] = s4[(size_t)k * count4 + e];
  }
  const bool adv = t >= HALF;
  const int c = adv ? t - HALF : t;  // this thread's 4 hidden units within its half
  f32x4 w[A];
  if (adv) {
    const f32x4* wa4 = reinterpret_cast<const f32x4*>(wa) + (size_t)c * A;  // wa rows 4c .. 4c+3
#pragma unroll
    for (int i = 0; i < A; ++i) w[i] = wa4[i];
  } else {
    w[0] = reinterpret_cast<const f32x4*>(wv)[c];
  }
  const f32x4 b = reinterpret_cast<const f32x4*>(fcb)[t];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    f32x4 v = sp[r][0];
#pragma unroll
    for (int k = 1; k < SPL; ++k) v += sp[r][k];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const float x = v[jj] + b[jj];
      v[jj] = x > 0.f ? x : 0.f;
    }
    if (r0 + r < rows) reinterpret_cast<f32x4*>(hid)[(int64_t)(r0 + r) * N4 + t] = v;
    if (adv) {
      const float* wf = reinterpret_cast<const float*>(w);  // [4][A], compile-time indices
#pragma unroll
      for (int o = 0; o < A; ++o) {
        float acc = v[0] * wf[o];
        acc = fmaf(v[1], wf[A + o], acc);
        acc = fmaf(v[2], wf[2 * A + o], acc);
        acc = fmaf(v[3], wf[3 * A + o], acc);
        part[r][o][c] = acc;
      }
    } else {
      float acc = v[0] * w[0][0];
      acc = fmaf(v[1], w[0][1], acc);
      acc = fmaf(v[2], w[0][2], acc);
      acc = fmaf(v[3], w[0][3], acc);
      part[r][A][c] = acc;
    }
  }
  __syncthreads();
  for (int j = wave; j < R * (A + 1); j += 4) {
    const int r = j / (A + 1), o = j - r * (A + 1);
    float x = part[r][o][2 * lane] + part[r][o][2 * lane + 1];
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
    if (lane == 0) dots[r][o] = x + (o == A ? bv[0] : ba[o]);
  }
  __syncthreads();
  if (t < R * A) {
    const int r = t / A, jj = t - r * A, row = r0 + r;
    if (row < rows) {
      float mean = 0.f;
      for (int k = 0; k < A; ++k) mean += dots[r][k];
      mean /= (float)A;
      q[(size_t)row * A + jj] = dots[r][A] + (dots[r][jj] - mean);
    }
  }
}

// dZ of 8 consecutive hidden units k0 .. k0 + 7 of one row (all in the value half or all in
// the advantage half: H % 8 == 0): k < H: g_b wv[k]; k >= H: dadv_i = g_b (1[i == a_b] -
// 1/A), dh_k = sum_i dadv_i wa[k][i] in order i = 0 .. A-1; masked by hid > 0.  The eight
// sums advance together, so each step over i issues eight independent loads (one branch per
// thread, outside the loads).
__device__ __forceinline__ void head_dz8(int k0, int H, int A, float gb, int ab, float inv_a,
                                         const float* __restrict__ wv,
                                         const float* __restrict__ wa, const float (&hv)[8],
                                         float (&d)[8]) {
  float v[8];
  if (k0 < H) {
    const f32x4 w0 = reinterpret_cast<const f32x4*>(wv + k0)[0];
    const f32x4 w1 = reinterpret_cast<const f32x4*>(wv + k0)[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = gb * w0[j];
      v[4 + j] = gb * w1[j];
    }
  } else {
    const float* rows = wa + (size_t)(k0 - H) * A;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
#pragma unroll 6
    for (int i = 0; i < A; ++i) {
      const float c = gb * ((i == ab ? 1.f : 0.f) - inv_a);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaf(c, rows[(size_t)j * A + i], v[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = hv[j] > 0.f ? v[j] : 0.f;
}

// Planes of 8 consecutive values at element e scaled by w (16-B stores); returns max |d|.
__device__ __forceinline__ float store_planes8(uint16_t* planes, int64_t pstride, int64_t e,
                                              const float (&d)[8], float w) {
  uint32_t ph[4], pl[4];
  float mx = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint16_t x0, y0, x1, y1;
    gemm::split2_bits(d[2 * j] * w, x0, y0);
    gemm::split2_bits(d[2 * j + 1] * w, x1, y1);
    ph[j] = x0 | ((uint32_t)x1 << 16);
    pl[j] = y0 | ((uint32_t)y1 << 16);
    mx = gemm::amax_max(mx, gemm::amax_max(fabsf(d[2 * j]), fabsf(d[2 * j + 1])));
  }
  *reinterpret_cast<uint4*>(planes + e) = uint4{ph[0], ph[1], ph[2], ph[3]};
  *reinterpret_cast<uint4*>(planes + pstride + e) = uint4{pl[0], pl[1], pl[2], pl[3]};
  return mx;
}

// Loss + head dZ in one launch (plane path).  Blocks [0, nb) each write the dZ planes of
// 256 / (2H / 8) rows (8 units per thread, as head_dz_planes_kernel), recomputing g_b of
// their rows with loss_row (the loss kernel's bits); the last block is the loss kernel
// (loss, TD errors, priorities, g and the action cache of every row).  Saves the loss
// launch and its dependency on the critical path.
__global__ void __launch_bounds__(256) dqn_loss_head_dz_kernel(
    LossArgs p, const float* __restrict__ h, int H, const float* __restrict__ wv,
    const float* __restrict__ wa, uint16_t* __restrict__ planes, int64_t pstride,
    gemm::PScale* __restrict__ sc) {
  __shared__ double red[4];
  __shared__ float gs[8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int B = p.B, A = p.A;
  // This thread's dZ operands (hidden units and action) are loaded first, at a clamped
  // index (the loss block's threads load a duplicate they never use), so their latency
  // overlaps the normaliser and loss below instead of following them.
  const int per = 2 * H / 8;  // threads per row (divides 256: launch_dqn_loss_head_dz)
  const int64_t t = (int64_t)blockIdx.x * 256 + tid;
  const int64_t tc = t < (int64_t)B * per ? t : (int64_t)B * per - 1;
  const int b = (int)(tc / per), k0 = 8 * (int)(tc - (int64_t)b * per);
  const float* hr = h + (size_t)b * 2 * H + k0;
  const f32x4 h0 = reinterpret_cast<const f32x4*>(hr)[0], h1 = reinterpret_cast<const f32x4*>(hr)[1];
  const int ab = p.a[b];
  // Importance-weight normaliser: max_b (1/p_b)^beta = (1/min_b p_b)^beta.
  double pmin = INFINITY;
  for (int b = tid; b < B; b += 256) pmin = fmin(pmin, p.probs[b]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pmin = fmin(pmin, __shfl_xor(pmin, o, 64));
  if (lane == 0) red[wave] = pmin;
  __syncthreads();
  pmin = fmin(fmin(red[0], red[1]), fmin(red[2], red[3]));
  if (p.global_min_prob) pmin = *p.global_min_prob;
  const double wmax = p.jax ? (double)powf((float)(1.0 / pmin), p.beta)
                            : pow(1.0 / pmin, (double)p.beta);
  if (!p.loss_part && blockIdx.x == gridDim.x - 1) {
    __syncthreads();  // red is reused below
    double lsum = 0.0;
    for (int b = tid; b < B; b += 256) {
      const LossRow row = loss_row(p, b, wmax);
      lsum += (double)row.hub_w;
      p.g[b] = row.g;
      p.td[b] = row.td;
      p.prio[b] = (double)fabsf(row.td);
      p.a_cache[b] = p.a[b];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) lsum += __shfl_xor(lsum, o, 64);
    if (lane == 0) red[wave] = lsum;
    __syncthreads();
    if (tid == 0) p.loss[0] = (float)((((red[0] + red[1]) + red[2]) + red[3]) / (double)p.mean_over);
    return;
  }
  const int b0 = (int)((int64_t)blockIdx.x * 256 / per);
  if (p.loss_part) {
    // This block's rows own their loss outputs (as the loss block does for every row) and
    // the block's f64 loss partial, summed in row order.
    __shared__ double hs[8];
    if (tid < 256 / per) {
      const int b = b0 + tid;
      double hw = 0.0;
      if (b < B) {
        const LossRow row = loss_row(p, b, wmax);
        gs[tid] = row.g;
        hw = (double)row.hub_w;
        p.g[b] = row.g;
        p.td[b] = row.td;
        p.prio[b] = (double)fabsf(row.td);
        p.a_cache[b] = p.a[b];
      }
      hs[tid] = hw;
    }
    __syncthreads();
    if (tid == 0) {
      double sum = 0.0;
      for (int i = 0; i < 256 / per; ++i) sum += hs[i];
      p.loss_part[blockIdx.x] = sum;
    }
  } else if (tid < 256 / per && b0 + tid < B) {
    gs[tid] = loss_row(p, b0 + tid, wmax).g;
  }
  __syncthreads();
  const bool live = t < (int64_t)B * per;
  const float gb = gs[live ? b - b0 : 0];
  const float inv_a = 1.f / (float)A;
  const float hv[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
  float d[8];
  head_dz8(k0, H, A, gb, ab, inv_a, wv, wa, hv, d);
  float mx = 0.f;
  if (live) mx = store_planes8(planes, pstride, (int64_t)b * 2 * H + k0, d, sc->w);
  gemm::amax_commit(sc, mx);
}

// The online duelling head fused with the loss and the head dZ (plane path, Nature head
// 2H = 1024, compile-time A).  Block b owns batch row b: the split-K sum, bias and ReLU of
// hidden rows b (o_tm1) and B + b (o_t, the double-Q selector) as fc_head1024_kernel, their
// q rows, the row's loss outputs (loss_row: reward clip, double-Q target, TD, Huber, IS
// weight; the normaliser from all B probabilities, read by every block), then dZ of hidden
// row b as planes from the registers that hold its units and their weights (head_dz8's
// terms in its order), masked by its ReLU.  One launch for the online head, the loss and
// the head dZ: the head's launch and its boundary leave the step's critical path.
template <int SPL, int A>
__global__ void __launch_bounds__(256) dqn_head_loss_dz_kernel(
    LossArgs p, const float* __restrict__ slab, const float* __restrict__ fcb,
    const float* __restrict__ wv, const float* __restrict__ bv, const float* __restrict__ wa,
    const float* __restrict__ ba, float* __restrict__ hid, uint16_t* __restrict__ planes,
    int64_t pstride, gemm::PScale* __restrict__ sc) {
  constexpr int N4 = 256, HALF = 128, R = 2, H = 512;
  __shared__ float part[R][A + 1][HALF];
  __shared__ float dots[R][A + 1];
  __shared__ double red[4];
  __shared__ float s_g;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int B = p.B, b = blockIdx.x;
  const int64_t count4 = (int64_t)2 * B * N4;  // the online slab holds 2B rows
  const f32x4* s4 = reinterpret_cast<const f32x4*>(slab);
  f32x4 sp[R][SPL];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t e = (int64_t)(r == 0 ? b : B + b) * N4 + t;
#pragma unroll
    for (int k = 0; k < SPL; ++k) sp[r][k] = s4[(size_t)k * count4 + e];
  }
  const bool adv = t >= HALF;
  const int c = adv ? t - HALF : t;  // this thread's 4 hidden units within its half
  f32x4 w[A];
  if (adv) {
    const f32x4* wa4 = reinterpret_cast<const f32x4*>(wa) + (size_t)c * A;  // wa rows 4c .. 4c+3
#pragma unroll
    for (int i = 0; i < A; ++i) w[i] = wa4[i];
  } else {
    w[0] = reinterpret_cast<const f32x4*>(wv)[c];
  }
  const f32x4 bias = reinterpret_cast<const f32x4*>(fcb)[t];
  const int ab = p.a[b];
  // Importance-weight normaliser: max_b (1/p_b)^beta = (1/min_b p_b)^beta.
  double pmin = INFINITY;
  for (int i = t; i < B; i += 256) pmin = fmin(pmin, p.probs[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pmin = fmin(pmin, __shfl_xor(pmin, o, 64));
  if (lane == 0) red[wave] = pmin;
  f32x4 h_own;  // hidden row b, this thread's units (the dZ mask)
#pragma unroll
  for (int r = 0; r < R; ++r) {
    f32x4 v = sp[r][0];
#pragma unroll
    for (int k = 1; k < SPL; ++k) v += sp[r][k];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const float x = v[jj] + bias[jj];
      v[jj] = x > 0.f ? x : 0.f;
    }
    reinterpret_cast<f32x4*>(hid)[(int64_t)(r == 0 ? b : B + b) * N4 + t] = v;
    if (r == 0) h_own = v;
    if (adv) {
      const float* wf = reinterpret_cast<const float*>(w);  // [4][A], compile-time indices
#pragma unroll
      for (int o = 0; o < A; ++o) {
        float acc = v[0] * wf[o];
        acc = fmaf(v[1], wf[A + o], acc);
        acc = fmaf(v[2], wf[2 * A + o], acc);
        acc = fmaf(v[3], wf[3 * A + o], acc);
        part[r][o][c] = acc;
      }
    } else {
      float acc = v[0] * w[0][0];
      acc = fmaf(v[1], w[0][1], acc);
      acc = fmaf(v[2], w[0][2], acc);
      acc = fmaf(v[3], w[0][3], acc);
      part[r][A][c] = acc;
    }
  }
  __syncthreads();
  for (int j = wave; j < R * (A + 1); j += 4) {
    const int r = j / (A + 1), o = j - r * (A + 1);
    float x = part[r][o][2 * lane] + part[r][o][2 * lane + 1];
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
    if (lane == 0) dots[r][o] = x + (o == A ? bv[0] : ba[o]);
  }
  __syncthreads();
  if (t < R * A) {
    const int r = t / A, jj = t - r * A;
    float mean = 0.f;
    for (int k = 0; k < A; ++k) mean += dots[r][k];
    mean /= (float)A;
    const_cast<float*>(p.q_on)[(size_t)(r == 0 ? b : B + b) * A + jj] =
        dots[r][A] + (dots[r][jj] - mean);
  }
  __syncthreads();  // the block's q rows are in global memory for loss_row
  if (t == 0) {
    pmin = fmin(fmin(red[0], red[1]), fmin(red[2], red[3]));
    if (p.global_min_prob) pmin = *p.global_min_prob;
    const double wmax = p.jax ? (double)powf((float)(1.0 / pmin), p.beta)
                              : pow(1.0 / pmin, (double)p.beta);
    const LossRow row = loss_row(p, b, wmax);
    s_g = row.g;
    p.g[b] = row.g;
    p.td[b] = row.td;
    p.prio[b] = (double)fabsf(row.td);
    p.a_cache[b] = ab;
    p.loss_part[b] = (double)row.hub_w;
  }
  __syncthreads();
  // dZ of hidden units 4c .. 4c+3 of this thread's half (head_dz8's terms, in its order).
  const float gb = s_g;
  float v4[4];
  if (!adv) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v4[j] = gb * w[0][j];
  } else {
    const float inv_a = 1.f / (float)A;
    const float* wf = reinterpret_cast<const float*>(w);
#pragma unroll
    for (int j = 0; j < 4; ++j) v4[j] = 0.f;
#pragma unroll
    for (int i = 0; i < A; ++i) {
      const float cc = gb * ((i == ab ? 1.f : 0.f) - inv_a);
#pragma unroll
      for (int j = 0; j < 4; ++j) v4[j] = fmaf(cc, wf[j * A + i], v4[j]);
    }
  }
  f32x4 d;
#pragma unroll
  for (int j = 0; j < 4; ++j) d[j] = h_own[j] > 0.f ? v4[j] : 0.f;
  const int64_t i4 = ((int64_t)b * 2 * H + (adv ? H : 0) + 4 * c) / 4;
  const float mx = store_planes4(planes, pstride, i4, d, sc->w);
  gemm::amax_commit(sc, mx);
}

// dZ of the fused hidden layer as planes, 8 consecutive units per thread:
// k < H: g_b wv[k];  k >= H: g_b (wa[k-H][a_b] - mean_j wa[k-H][j]); masked by hid > 0.
__global__ void __launch_bounds__(256) head_dz_planes_kernel(
    const float* __restrict__ h, const float* __restrict__ g, const int32_t* __restrict__ a,
    int B, int H, int A, const float* __restrict__ wv, const float* __restrict__ wa,
    uint16_t* __restrict__ planes, int64_t pstride, gemm::PScale* __restrict__ sc) {
  const int per = 2 * H / 8;
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool live = t0 < (int64_t)B * per;
  const int64_t t = live ? t0 : (int64_t)B * per - 1;  // clamped: every lane reaches the amax
  const int b = (int)(t / per), k0 = 8 * (int)(t - (int64_t)b * per);
  const float gb = g[b];
  const int ab = a[b];
  const float inv_a = 1.f / (float)A;
  const float* hr = h + (size_t)b * 2 * H + k0;
  const f32x4 h0 = reinterpret_cast<const f32x4*>(hr)[0], h1 = reinterpret_cast<const f32x4*>(hr)[1];
  const float hv[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
  float d[8];
  head_dz8(k0, H, A, gb, ab, inv_a, wv, wa, hv, d);
  float mx = 0.f;
  if (live) mx = store_planes8(planes, pstride, (int64_t)b * 2 * H + k0, d, sc->w);
  gemm::amax_commit(sc, mx);
}

// snt.Adam / optix.adam on float4 i of the flat buffers, the gradient given.
struct AdamConsts {
  float lr, b1, omb1, b2, omb2, bc1, bc2, eps;
  int optix;
  int toff = 1;  // device count: t = *dev_steps + toff (0 when the step was counted before Adam)
};

// Returns max |p| written to the planes (0 without planes).  skip (a guarded step that
// overflowed): p, m and v stay; the planes of p are rewritten at pw.
__device__ __forceinline__ float adam_update4(int64_t i, f32x4 gg, float* __restrict__ p,
                                              float* __restrict__ m, float* __restrict__ v,
                                              const AdamConsts& c, uint16_t* __restrict__ planes,
                                              int64_t pstride, float pw, bool skip = false) {
  if (skip) {
    if (!planes) return 0.f;
    return store_planes4(planes, pstride, i, reinterpret_cast<const f32x4*>(p)[i], pw);
  }
  // The moments are streamed (read once, written once per step) with non-temporal
  // accesses, so they bypass the caches the next step's forwards read the parameter planes
  // through.
  f32x4 mm = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(m) + i);
  f32x4 vv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(v) + i);
  f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float mj = __fadd_rn(__fmul_rn(c.b1, mm[j]), __fmul_rn(c.omb1, gg[j]));
    const float vj =
        __fadd_rn(__fmul_rn(c.b2, vv[j]), __fmul_rn(c.omb2, __fmul_rn(gg[j], gg[j])));
    const float mh = __fdiv_rn(mj, c.bc1);
    const float vh = __fdiv_rn(vj, c.bc2);
    const float den = __fadd_rn(__fsqrt_rn(vh), c.eps);
    const float upd = c.optix ? __fmul_rn(c.lr, __fdiv_rn(mh, den))
                              : __fdiv_rn(__fmul_rn(c.lr, mh), den);
    mm[j] = mj;
    vv[j] = vj;
    pp[j] = __fsub_rn(pp[j], upd);
  }
  __builtin_nontemporal_store(mm, reinterpret_cast<f32x4*>(m) + i);
  __builtin_nontemporal_store(vv, reinterpret_cast<f32x4*>(v) + i);
  reinterpret_cast<f32x4*>(p)[i] = pp;
  // (No amax here: a block handles about one float4 per thread, so a per-block
  // reduction and atomic cost as much as the update; 45 -> 58 us measured.  The
  // parameters' maximum is taken by launch_param_amax every few steps; adam_planes_check
  // commits it only when a write overflowed.)
  return planes ? store_planes4(planes, pstride, i, pp, pw) : 0.f;
}

// A parameter-plane write that overflowed (rare): the wave's max |p| goes to the record,
// whose flag it raises, so the end-of-step rescale moves the scale (the next step's forward
// then overflows and is skipped, and its Adam pass rewrites the planes at the new scale).
__device__ __forceinline__ void adam_planes_check(gemm::PScale* psc, float mx, float pw) {
  if (psc && __builtin_amdgcn_ballot_w64(!(mx * pw < 65520.f)) != 0ull)
    gemm::amax_commit(psc, mx);
}

__device__ __forceinline__ void adam_tail(const AdamTail& t, const Gate& gate) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  if (t.clear) {
    t.clear->on = 0u;
    t.clear->prm = 0u;
  }
  for (int i = 0; i < t.ncommit; ++i)
    if (!(i >= t.skip_lo && i < t.skip_hi)) t.commit[i].r = t.commit[i].wi;
  if (t.params) {
    const float wi = t.params->wi;
    t.params->r = t.params->rl = wi;
    // The target's planes take the parameters' at the step's copy, which a skipped step
    // does not make (launch_copy_gated).
    if (t.target && !gate_skip(gate)) t.target->r = t.target->rl = wi;
  }
}

__device__ __forceinline__ void adam_bias_corrections(AdamConsts& c, const int64_t* dev_steps) {
  if (dev_steps) {  // device-side step count: same expressions as the host's
    const float tf = (float)(*dev_steps + c.toff);
    c.bc1 = 1.f - powf(c.b1, tf);
    c.bc2 = 1.f - powf(c.b2, tf);
  }
}

__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p,
                                                   const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   int64_t n4, AdamConsts c,
                                                   uint16_t* __restrict__ planes,
                                                   int64_t pstride, gemm::PScale* __restrict__ psc,
                                                   const int64_t* __restrict__ dev_steps,
                                                   const Gate gate, const AdamTail tail) {
  adam_tail(tail, gate);
  adam_bias_corrections(c, dev_steps);
  const bool skip = gate_skip(gate);
  const float pw = planes ? psc->w : 0.f;
  float mx = 0.f;
#pragma unroll 2
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x)
    mx = gemm::amax_max(mx, adam_update4(i, skip ? f32x4{} : __builtin_nontemporal_load(
                                                        reinterpret_cast<const f32x4*>(g) + i),
                                p, m, v, c, planes, pstride, pw, skip));
  if (planes) adam_planes_check(psc, mx, pw);
}

// Adam whose gradients for some ranges are still split-K slabs (the conv weight gradients
// of the fused DQN step): the first blocks each reduce 16 float4 of a slab range exactly
// as slab_reduce4_kernel does (16 split groups, the same addition order, so the same bits),
// store the reduced gradient into g and update those parameters; the other blocks update
// [dense_off4, dense_off4 + dense_n4) from g as adam_kernel does.
__global__ void __launch_bounds__(256) adam_slabs_kernel(float* __restrict__ p,
                                                         float* __restrict__ g,
                                                         float* __restrict__ m,
                                                         float* __restrict__ v, AdamSlabs s,
                                                         AdamConsts c,
                                                         uint16_t* __restrict__ planes,
                                                         int64_t pstride,
                                                         gemm::PScale* __restrict__ psc,
                                                         const int64_t* __restrict__ dev_steps,
                                                         const Gate gate, const AdamTail tail) {
  adam_tail(tail, gate);
  adam_bias_corrections(c, dev_steps);
  const bool skip = gate_skip(gate);
  const float pw = planes ? psc->w : 0.f;
  float mx = 0.f;
  const int nsb = s.block_end[s.nseg - 1];
  if ((int)blockIdx.x < nsb) {
    __shared__ f32x4 red[16][16];
    int k = 0;
    while ((int)blockIdx.x >= s.block_end[k]) ++k;
    const AdamSlabs::Seg& q = s.seg[k];
    const int cc = threadIdx.x & 15, gq = threadIdx.x >> 4;
    const int64_t f = (int64_t)(blockIdx.x - (k ? s.block_end[k - 1] : 0)) * 16 + cc;
    const f32x4* s4 = reinterpret_cast<const f32x4*>(q.slab) + q.e4;
    f32x4 acc{0.f, 0.f, 0.f, 0.f};
    if (f < q.n4) {
#pragma unroll 8
      for (int sp = gq; sp < q.splits; sp += 16) acc += s4[(size_t)sp * q.count4 + f];
    }
    red[gq][cc] = acc;
    __syncthreads();
    if (gq == 0 && f < q.n4) {
      f32x4 gg = red[0][cc];
#pragma unroll
      for (int r = 1; r < 16; ++r) gg += red[r][cc];
      reinterpret_cast<f32x4*>(g)[q.off4 + f] = gg;  // the step's gradient stays readable
      mx = adam_update4(q.off4 + f, gg, p, m, v, c, planes, pstride, pw, skip);
    }
    if (planes) adam_planes_check(psc, mx, pw);
    return;
  }
  for (int64_t i = (int64_t)(blockIdx.x - nsb) * blockDim.x + threadIdx.x; i < s.dense_n4;
       i += (int64_t)(gridDim.x - nsb) * blockDim.x) {
    const int64_t j = s.dense_off4 + i;
    mx = gemm::amax_max(mx, adam_update4(j, skip ? f32x4{} : __builtin_nontemporal_load(
                                                        reinterpret_cast<const f32x4*>(g) + j),
                                p, m, v, c, planes, pstride, pw, skip));
  }
  if (planes) adam_planes_check(psc, mx, pw);
}

__global__ void count_step_kernel(int64_t* c) { *c += 1; }

// Two device copies (16-byte units) unless the gate's step was skipped.
__global__ void __launch_bounds__(256) copy_gated_kernel(uint4* __restrict__ d0,
                                                         const uint4* __restrict__ s0, int64_t n0,
                                                         uint4* __restrict__ d1,
                                                         const uint4* __restrict__ s1, int64_t n1,
                                                         const Gate gate) {
  if (gate_skip(gate)) return;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n0 + n1; i += stride) {
    if (i < n0) d0[i] = s0[i];
    else d1[i - n0] = s1[i - n0];
  }
}


// Planes of x at the scale record's read scale (1 / r, set or kept by
// plane_scale_set_kernel; exact for a power of two); no amax.
__global__ void __launch_bounds__(256) split_planes_kernel(const float* __restrict__ x, int64_t n4,
                                                           uint16_t* __restrict__ planes,
                                                           int64_t pstride,
                                                           const gemm::PScale* __restrict__ sc) {
  const float w = 1.f / sc->r;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x)
    store_planes4(planes, pstride, i, reinterpret_cast<const f32x4*>(x)[i], w);
}

// Planes of x at the record's current write scale w, with the maximum of |x| committed to
// the record's amax slots: the end-of-step rescale turns it into the next step's w (lagged
// amax, as for the activations).  One pass instead of amax + scale set + split.
__global__ void __launch_bounds__(256) split_planes_lagged_kernel(const float* __restrict__ x,
                                                                  int64_t n4,
                                                                  uint16_t* __restrict__ planes,
                                                                  int64_t pstride,
                                                                  gemm::PScale* __restrict__ sc) {
  const float w = sc->w;
  float mx = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x)
    mx = gemm::amax_max(mx, store_planes4(planes, pstride, i, reinterpret_cast<const f32x4*>(x)[i], w));
  gemm::amax_commit(sc, mx);
}

// max |x| into sc->amax (which is 0 between rescales).
__global__ void __launch_bounds__(256) amax_kernel(const float* __restrict__ x, int64_t n4,
                                                   gemm::PScale* __restrict__ sc) {
  float mx = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    mx = gemm::amax_max(mx, gemm::amax_max(gemm::amax_max(fabsf(v[0]), fabsf(v[1])),
                                           gemm::amax_max(fabsf(v[2]), fabsf(v[3]))));
  }
  gemm::amax_commit(sc, mx);
}

// The power of two w that puts a (> 0, finite) at 2^7 <= a w < 2^8 (gemm_p3.h); exponent
// clamped so w and 1 / w stay normal f32.
__device__ __forceinline__ int scale_exp(float a) {
  int k;
  (void)frexpf(a, &k);  // a = m 2^k, m in [0.5, 1)
  const int e = 8 - k;
  return e < -100 ? -100 : (e > 100 ? 100 : e);
}

// The record's amax (max over its slots, read by every lane of one wave) and its slots
// cleared.  Non-negative floats order as their bits; NaN above infinity.
__device__ __forceinline__ float take_amax(gemm::PScale* sc, int lane) {
  uint32_t a = sc->slot[lane].v;
  sc->slot[lane].v = 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) a = max(a, (uint32_t)__shfl_xor((int)a, o, 64));
  return __builtin_bit_cast(float, a);
}

// Sets a record for planes about to be written at 1 / r from the amax just collected (one
// wave), slots cleared.  keep != 0: a record whose read scale r already suits the data
// (2^4 <= amax / r < 2^12, e.g. restored from a checkpoint together with the parameters it
// was written for) is left as it is, so the rewritten planes are the bits its writer
// produced and the next write uses the restored w; otherwise w from the amax (1 if it is
// 0) and r = wi = 1 / w.
__global__ void __launch_bounds__(64) plane_scale_set_kernel(gemm::PScale* __restrict__ sc,
                                                             int* __restrict__ overflow,
                                                             int keep) {
  const float a = take_amax(sc, threadIdx.x);
  if (threadIdx.x != 0) return;
  if (!(a <= 3.0e38f) && overflow) atomicOr(overflow, 1);  // NaN / infinite input
  const float y = a / sc->r;
  if (keep && a > 0.f && y >= 16.f && y < 4096.f) return;
  const int e = a > 0.f && a <= 3.0e38f ? scale_exp(a) : 0;
  sc->w = ldexpf(1.f, e);
  sc->r = sc->wi = sc->rl = ldexpf(1.f, -e);
}

// A rescale job (rescale.h) as its own launch: one workgroup of 256 threads.
__global__ void __launch_bounds__(256) plane_rescale_kernel(const RescaleJob job) {
  rescale_block(job);
}

// This rank's skip decision into dst: its gate, the sticky hold, and the end-of-step
// rescale's own test on the transient records [0, n) outside [skip_lo, skip_hi) (a tensor
// that overflowed or underflowed its planes: rescale.h), so the ranks' all-reduced decision
// is the one every rank's rescale would take.  One wave.
__global__ void __launch_bounds__(64) gate_publish_kernel(const Gate gate, float* dst,
                                                          const gemm::PScale* __restrict__ s,
                                                          int n, int skip_lo, int skip_hi) {
  const int lane = threadIdx.x;
  bool bad = false;
  for (int i = 0; i < n; ++i) {
    if (i >= skip_lo && i < skip_hi) continue;
    uint32_t a = s[i].slot[lane].v;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a = max(a, (uint32_t)__shfl_xor((int)a, o, 64));
    const float am = __builtin_bit_cast(float, a), aw = am * s[i].w;
    bad = bad || (am != 0.f && (!(aw < 65520.f) || aw < 1.f));
  }
  if (lane == 0) *dst = (gate_skip(gate) || gate.g->hold != 0u || bad) ? 1.f : 0.f;
}

__global__ void __launch_bounds__(256) frames_f16_kernel(const uint8_t* __restrict__ a,
                                                         const uint8_t* __restrict__ b,
                                                         int64_t split8, int64_t n8,
                                                         uint16_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint2 w = i < split8 ? reinterpret_cast<const uint2*>(a)[i]
                               : reinterpret_cast<const uint2*>(b)[i - split8];
    // f16(byte) is exact (8 significant bits).
    reinterpret_cast<uint4*>(out)[i] =
        uint4{gemm::f16x2_of_bytes(w.x, 0), gemm::f16x2_of_bytes(w.x, 16),
              gemm::f16x2_of_bytes(w.y, 0), gemm::f16x2_of_bytes(w.y, 16)};
  }
}

__global__ void __launch_bounds__(256) join_planes_kernel(const uint16_t* __restrict__ planes,
                                                          int64_t pstride, int64_t n,
                                                          float* __restrict__ x,
                                                          const gemm::PScale* __restrict__ sc) {
  const gemm::CPlanes c{planes, pstride, sc};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    x[i] = c.value(i);
}


// Each thread's float4 indices i = tid_global + k * stride, k = 0, 1, ...: the loads of
// kBatch consecutive k are issued together (clamped indices, no branch around a load), then
// summed in k order, so the sum is the plain sequential one.  (One load per iteration left
// ~19 dependent round trips per thread at IMPALA's 4.9 M parameters on 256 blocks.)
constexpr int kSumsqBatch = 8;
__global__ void __launch_bounds__(256) grad_sumsq_kernel(const float* __restrict__ g, int64_t n4,
                                                         int64_t pol4, double* __restrict__ part,
                                                         int64_t* __restrict__ dev_step,
                                                         StepGuard* __restrict__ guard,
                                                         uint32_t* __restrict__ tmo,
                                                         int64_t* __restrict__ host_skipped) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    bool skip = false;
    if (guard) {  // the step's flags: planes overflowed, or the LSTM unroll timed out
      const uint32_t t = tmo ? tmo[0] : 0u;
      skip = (guard->on | t) != 0u;
      guard->last = skip ? 1u : 0u;
      guard->on = 0u;
      if (t) {
        tmo[0] = 0u;
        tmo[1] += 1u;  // timeouts so far (sticky count)
      }
      if (skip) {
        const int64_t k = guard->skipped + 1;
        guard->skipped = k;
        if (host_skipped) *host_skipped = k;
      } else {
        guard->applied += 1;
      }
    }
    if (dev_step && !skip) *dev_step += 1;
  }
  __shared__ double red[2][4];
  double s0 = 0.0, s1 = 0.0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const f32x4* g4 = reinterpret_cast<const f32x4*>(g);
  for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < n4; i0 += kSumsqBatch * stride) {
    f32x4 x[kSumsqBatch];
#pragma unroll
    for (int k = 0; k < kSumsqBatch; ++k) x[k] = g4[min(i0 + k * stride, n4 - 1)];
#pragma unroll
    for (int k = 0; k < kSumsqBatch; ++k) {
      const int64_t i = i0 + k * stride;
      if (i >= n4) break;
      const double q = (double)x[k][0] * x[k][0] + (double)x[k][1] * x[k][1] +
                       (double)x[k][2] * x[k][2] + (double)x[k][3] * x[k][3];
      if (i < pol4) s0 += q;
      else s1 += q;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s0 += __shfl_xor(s0, o, 64);
    s1 += __shfl_xor(s1, o, 64);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wave] = s0;
    red[1][wave] = s1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[blockIdx.x] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    part[gridDim.x + blockIdx.x] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
  }
}

__global__ void __launch_bounds__(256) clip_adam_kernel(const ClipAdamArgs a) {
  __shared__ double red[2][4];
  __shared__ float scl[4];
  const float tf = (float)*a.dev_step;
  const float bc1 = 1.f - powf(a.b1, tf), bc2 = 1.f - powf(a.b2, tf);
  const float omb1 = 1.f - a.b1, omb2 = 1.f - a.b2;
  double s0 = 0.0, s1 = 0.0;
  for (int i = threadIdx.x; i < a.nparts; i += 256) {
    s0 += a.part[i];
    s1 += a.part[a.nparts + i];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s0 += __shfl_xor(s0, o, 64);
    s1 += __shfl_xor(s1, o, 64);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wave] = s0;
    red[1][wave] = s1;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const int k = threadIdx.x;
    const double ss = ((red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
    const float G = (float)sqrt(ss);
    float s = 1.f;
    if (a.optix) {  // optix.clip_by_global_norm: (t / G) * c when G >= c
      if (a.clipping && !(G < a.clip_norm)) s = -1.f;  // marks "divide by G, times c"
    } else if (a.clipping && G > 0.f) {  // tf.clip_by_global_norm
      s = a.clip_norm * fminf(1.f / G, 1.f / a.clip_norm);
    }
    scl[k] = s;
    scl[2 + k] = G;
    if (blockIdx.x == 0 && a.norms) a.norms[k] = G;
  }
  // The logged losses: wave 1 sums sum_a, wave 2 sum_b (lane-strided partials, then a
  // fixed shuffle tree: deterministic).
  if (blockIdx.x == 0 && (wave == 1 || wave == 2)) {
    const float* src = wave == 1 ? a.sum_a : a.sum_b;
    float* dst = wave == 1 ? a.out_a : a.out_b;
    const int n = wave == 1 ? a.n_a : a.n_b;
    if (dst) {
      float t = 0.f;
      for (int i = lane; i < n; i += 64) t += src[i];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
      if (lane == 0) *dst = t / (wave == 1 ? a.div_a : a.div_b);
    }
  }
  __syncthreads();
  if (gate_skip(a.gate)) return;  // a skipped step: parameters and moments stay
  // kAdamBatch grid-stride positions per pass, every load issued before the first update
  // (clamped indices; the stores are guarded).
  constexpr int kAdamBatch = 4;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const f32x4* __restrict__ g4 = reinterpret_cast<const f32x4*>(a.g);
  f32x4* __restrict__ m4 = reinterpret_cast<f32x4*>(a.m);
  f32x4* __restrict__ v4 = reinterpret_cast<f32x4*>(a.v);
  f32x4* __restrict__ p4 = reinterpret_cast<f32x4*>(a.p);
  for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < a.n4; i0 += kAdamBatch * stride) {
    f32x4 gb[kAdamBatch], mb[kAdamBatch], vb[kAdamBatch], pb[kAdamBatch];
#pragma unroll
    for (int k = 0; k < kAdamBatch; ++k) {
      const int64_t i = min(i0 + k * stride, a.n4 - 1);
      gb[k] = g4[i];
      mb[k] = m4[i];
      vb[k] = v4[i];
      pb[k] = p4[i];
    }
#pragma unroll
    for (int k = 0; k < kAdamBatch; ++k) {
      const int64_t i = i0 + k * stride;
      if (i >= a.n4) break;
      const bool g0 = i < a.group0_4;
      const float s = g0 ? scl[0] : scl[1];
      const float G = g0 ? scl[2] : scl[3];
      const float lr = g0 ? a.lr0 : a.lr1;
      const f32x4 gg = gb[k];
      f32x4 mm = mb[k], vv = vb[k], pp = pb[k];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float gj = s < 0.f ? __fmul_rn(__fdiv_rn(gg[j], G), a.clip_norm) : __fmul_rn(gg[j], s);
        const float mj = __fadd_rn(__fmul_rn(a.b1, mm[j]), __fmul_rn(omb1, gj));
        const float vj = __fadd_rn(__fmul_rn(a.b2, vv[j]), __fmul_rn(omb2, __fmul_rn(gj, gj)));
        const float mh = __fdiv_rn(mj, bc1);
        const float vh = __fdiv_rn(vj, bc2);
        const float den = __fadd_rn(__fsqrt_rn(vh), a.eps);
        const float upd = a.optix ? __fmul_rn(lr, __fdiv_rn(mh, den)) : __fdiv_rn(__fmul_rn(lr, mh), den);
        mm[j] = mj;
        vv[j] = vj;
        pp[j] = __fsub_rn(pp[j], upd);
      }
      m4[i] = mm;
      v4[i] = vv;
      p4[i] = pp;
    }
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

int launch_duel_head_finish(const float* slab, int splits, int rows, int A, const float* bv,
                            const float* ba, float* q, hipStream_t st) {
  duel_head_finish_kernel<<<(unsigned)ceil_div(rows, 4), 256, 0, st>>>(slab, splits, rows, A, bv,
                                                                       ba, q);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_duel_head_dz(const float* h, const float* g, const int32_t* a, int B, int H, int A,
                        const float* wv, const float* wa, float* dzh, hipStream_t st,
                        uint16_t* planes, int64_t pstride, gemm::PScale* sc) {
  ACME_CHECK_ARG(!planes || sc, "planes need a scale record");
  const int64_t n = (int64_t)B * 2 * H;
  duel_head_dz_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(h, g, a, B, H, A, wv, wa, dzh,
                                                                   planes, pstride, sc);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_duel_head_grad_scatter(const float* slab, int splits, int H, int A, float* dwv,
                                  float* dbv, float* dwa, float* dba, hipStream_t st,
                                  const double* part, int64_t nparts, int mean_over,
                                  float* loss) {
  ACME_CHECK_ARG(!part || (loss && nparts >= 1 && mean_over >= 1), "bad loss sum args");
  const int64_t count = (int64_t)(2 * H + 1) * (A + 1);
  duel_head_grad_scatter_kernel<<<(unsigned)(ceil_div(count, 256) + (part ? 1 : 0)), 256, 0,
                                  st>>>(slab, splits, H, A, dwv, dbv, dwa, dba, part, nparts,
                                        mean_over, loss);
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

int launch_fc_head_forward(const float* slab, int splits, int rows, int H, const float* fcb,
                           const float* wv, const float* bv, const float* wa, const float* ba,
                           int A, float* hid, float* q, hipStream_t st) {
  ACME_CHECK_ARG(H % 2 == 0 && A >= 1 && splits >= 1 && rows >= 1, "bad head shape");
  const size_t shmem =
      sizeof(float) * (kHeadRows * 2 * H + (size_t)H * A + H + kHeadRows * (A + 1) +
                       4 * kHeadChunk * 64 + 4);
  ACME_CHECK_ARG(shmem <= 65536, "head too large for the fused head kernel");
  const bool wa16 = reinterpret_cast<uintptr_t>(wa) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(wv) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(fcb) % 16 == 0;
  if (H == 512 && A == 18 && wa16 && (splits == 4 || splits == 8 || splits == 16)) {
    // One row per block (2 rows: 12.7 us, 4 rows: 16.3 us, 1 row: 11.4 us per launch).
    if (splits == 16)
      fc_head1024_kernel<16, 18, 1><<<rows, 256, 0, st>>>(slab, rows, fcb, wv, bv, wa, ba, hid, q);
    else if (splits == 8)
      fc_head1024_kernel<8, 18, 1><<<rows, 256, 0, st>>>(slab, rows, fcb, wv, bv, wa, ba, hid, q);
    else
      fc_head1024_kernel<4, 18, 1><<<rows, 256, 0, st>>>(slab, rows, fcb, wv, bv, wa, ba, hid, q);
    ACME_LAUNCH_CHECK();
    return ACME_OK;
  }
  const unsigned grid = (unsigned)ceil_div(rows, kHeadRows);
  if (H == 512 && wa16 && splits == 8)
    fc_head_forward_kernel<8, 512><<<grid, 256, shmem, st>>>(slab, splits, rows, H, fcb, wv, bv, wa,
                                                              ba, A, hid, q);
  else if (H == 512 && wa16 && splits == 4)
    fc_head_forward_kernel<4, 512><<<grid, 256, shmem, st>>>(slab, splits, rows, H, fcb, wv, bv, wa,
                                                              ba, A, hid, q);
  else
    fc_head_forward_kernel<0, 0><<<grid, 256, shmem, st>>>(slab, splits, rows, H, fcb, wv, bv, wa,
                                                            ba, A, hid, q);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int64_t dqn_loss_head_dz_blocks(int B, int H) { return ceil_div((int64_t)B * (2 * H / 8), 256); }

bool dqn_head_loss_dz_fusable(int H, int A, int splits, const float* wv, const float* wa,
                              const float* fcb) {
  return H == 512 && A == 18 && (splits == 4 || splits == 8) &&
         reinterpret_cast<uintptr_t>(wa) % 16 == 0 && reinterpret_cast<uintptr_t>(wv) % 16 == 0 &&
         reinterpret_cast<uintptr_t>(fcb) % 16 == 0;
}

int launch_dqn_head_loss_dz(const LossArgs& args, const float* slab, int splits, int H,
                            const float* fcb, const float* wv, const float* bv, const float* wa,
                            const float* ba, float* hid, uint16_t* planes, int64_t pstride,
                            gemm::PScale* sc, hipStream_t st) {
  ACME_CHECK_ARG(dqn_head_loss_dz_fusable(H, args.A, splits, wv, wa, fcb) && args.loss_part &&
                     planes && sc && args.B >= 1,
                 "bad fused head / loss / head dZ arguments");
  if (splits == 8)
    dqn_head_loss_dz_kernel<8, 18><<<(unsigned)args.B, 256, 0, st>>>(args, slab, fcb, wv, bv, wa, ba,
                                                                   hid, planes, pstride, sc);
  else
    dqn_head_loss_dz_kernel<4, 18><<<(unsigned)args.B, 256, 0, st>>>(args, slab, fcb, wv, bv, wa, ba,
                                                                   hid, planes, pstride, sc);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

__global__ void __launch_bounds__(256) dqn_loss_sum_kernel(const double* __restrict__ part,
                                                           int64_t n, int mean_over,
                                                           float* __restrict__ loss) {
  loss_sum_block(part, n, mean_over, loss);
}

int launch_dqn_loss_sum(const double* part, int64_t n, int mean_over, float* loss, hipStream_t st) {
  ACME_CHECK_ARG(part && loss && n >= 1 && mean_over >= 1, "bad loss sum args");
  dqn_loss_sum_kernel<<<1, 256, 0, st>>>(part, n, mean_over, loss);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_dqn_loss_head_dz(const LossArgs& args, const float* h, int H, const float* wv,
                            const float* wa, uint16_t* planes, int64_t pstride, gemm::PScale* sc,
                            hipStream_t st) {
  ACME_CHECK_ARG(args.B >= 1 && args.A >= 1 && h && wv && wa && planes && sc,
                 "bad loss / head dZ args");
  const int per = 2 * H / 8;
  ACME_CHECK_ARG(H % 8 == 0 && per >= 32 && 256 % per == 0, "hidden size %d: 2H/8 must divide 256", H);
  ACME_CHECK_ARG(reinterpret_cast<uintptr_t>(wv) % 16 == 0, "wv must be 16-byte aligned");
  const int64_t nb = ceil_div((int64_t)args.B * per, 256);
  dqn_loss_head_dz_kernel<<<(unsigned)(args.loss_part ? nb : nb + 1), 256, 0, st>>>(
      args, h, H, wv, wa, planes, pstride, sc);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_head_dz_planes(const float* h, const float* g, const int32_t* a, int B, int H, int A,
                          const float* wv, const float* wa, uint16_t* planes, int64_t pstride,
                          gemm::PScale* sc, hipStream_t st) {
  ACME_CHECK_ARG(H % 8 == 0 && pstride % 8 == 0 && reinterpret_cast<uintptr_t>(wv) % 16 == 0 && sc,
                 "bad head_dz shape");
  const int64_t n = (int64_t)B * (2 * H / 8);
  head_dz_planes_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(h, g, a, B, H, A, wv, wa,
                                                                    planes, pstride, sc);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_slab_reduce(const float* slab, int splits, int64_t count, float* out0,
                       int64_t split_at, float* out1, const float* bias, int ncols, int relu,
                       hipStream_t st) {
  ACME_CHECK_ARG(splits >= 1 && count >= 1, "bad slab shape");
  const bool vec = count % 4 == 0 && split_at % 4 == 0 && (!bias || ncols % 4 == 0) &&
                   reinterpret_cast<uintptr_t>(slab) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(out0) % 16 == 0 &&
                   (split_at >= count || reinterpret_cast<uintptr_t>(out1) % 16 == 0);
  if (vec) {
    const int64_t count4 = count / 4;
    slab_reduce4_kernel<<<(unsigned)ceil_div(count4, 16), 256, 0, st>>>(
        slab, splits, count4, out0, split_at / 4, out1, bias, ncols, relu);
    ACME_LAUNCH_CHECK();
    return ACME_OK;
  }
  slab_reduce_kernel<<<(unsigned)ceil_div(count, 64), 256, 0, st>>>(slab, splits, count, out0,
                                                                    split_at, out1, bias, ncols,
                                                                    relu);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_grad_sumsq(const float* g, int64_t n4, int64_t group0_4, double* part, int nparts,
                      int64_t* dev_step, hipStream_t st, StepGuard* guard, uint32_t* lstm_tmo,
                      int64_t* host_skipped) {
  ACME_CHECK_ARG(g && part && nparts >= 1, "bad argument");
  grad_sumsq_kernel<<<(unsigned)nparts, 256, 0, st>>>(g, n4, group0_4, part, dev_step, guard,
                                                      lstm_tmo, host_skipped);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1,
                float b2, float eps, int64_t t, uint16_t* planes, int64_t pstride, hipStream_t st,
                int optix, int64_t* dev_steps, gemm::PScale* psc, const Gate& gate, bool count,
                const AdamTail& tail) {
  ACME_CHECK_ARG(p && g && m && v, "null buffer");
  ACME_CHECK_ARG(!planes || psc, "parameter planes need a scale record");
  ACME_CHECK_ARG(n % 4 == 0, "adam buffer length must be a multiple of 4");
  ACME_CHECK_ARG(pstride % 4 == 0, "plane stride must be a multiple of 4");
  ACME_CHECK_ARG(t >= 1 || dev_steps, "adam step must be >= 1");
  // With a device count not advanced here (count == false), the caller's rescale has
  // already counted this step: t = *dev_steps.
  const AdamConsts c{lr, b1, 1.f - b1, b2, 1.f - b2,
                     dev_steps ? 0.f : 1.f - powf(b1, (float)t),
                     dev_steps ? 0.f : 1.f - powf(b2, (float)t), eps, optix, count ? 1 : 0};
  const int64_t n4 = n / 4;
  // Grid cap 8192: 47.7 -> 45.2 us against 2048.  Non-temporal gradient / moment traffic:
  // 45.8 -> 45.1 us, and the next step's forwards (which read the parameter planes) ~1 us
  // faster each.
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n4, 256), 8192);
  adam_kernel<<<std::max(grid, 1u), 256, 0, st>>>(p, g, m, v, n4, c, planes, pstride, psc,
                                                  dev_steps, gate, tail);
  ACME_LAUNCH_CHECK();
  if (dev_steps && count) {
    count_step_kernel<<<1, 1, 0, st>>>(dev_steps);
    ACME_LAUNCH_CHECK();
  }
  return ACME_OK;
}

int launch_adam_slabs(float* p, float* g, float* m, float* v, const AdamSlabs& slabs,
                      float lr, float b1, float b2, float eps, const int64_t* dev_steps,
                      uint16_t* planes, int64_t pstride, gemm::PScale* psc, int optix,
                      const Gate& gate, const AdamTail& tail, hipStream_t st) {
  ACME_CHECK_ARG(p && g && m && v && (!planes || psc) && dev_steps, "null buffer");
  ACME_CHECK_ARG(slabs.nseg >= 1 && slabs.nseg <= AdamSlabs::kMaxSegs, "bad slab Adam arguments");
  AdamSlabs s = slabs;
  int blocks = 0;
  for (int k = 0; k < s.nseg; ++k) {
    const AdamSlabs::Seg& q = s.seg[k];
    ACME_CHECK_ARG(q.slab && q.splits >= 1 && q.n4 >= 1 && q.e4 + q.n4 <= q.count4,
                   "bad slab segment %d", k);
    blocks += (int)ceil_div(q.n4, 16);
    s.block_end[k] = blocks;
  }
  const AdamConsts c{lr, b1, 1.f - b1, b2, 1.f - b2, 0.f, 0.f, eps, optix, 0};
  const int dense = (int)std::min<int64_t>(ceil_div(s.dense_n4, 256), 8192);
  adam_slabs_kernel<<<(unsigned)(blocks + std::max(dense, 1)), 256, 0, st>>>(
      p, g, m, v, s, c, planes, pstride, psc, dev_steps, gate, tail);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_split_planes(const float* x, int64_t n, uint16_t* planes, int64_t pstride,
                        gemm::PScale* sc, hipStream_t st, int* overflow, int keep_scale) {
  ACME_CHECK_ARG(n % 4 == 0 && pstride % 4 == 0 && sc, "plane split needs multiples of 4");
  const int64_t n4 = n / 4;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n4, 256), 2048);
  amax_kernel<<<std::max(grid, 1u), 256, 0, st>>>(x, n4, sc);
  ACME_LAUNCH_CHECK();
  plane_scale_set_kernel<<<1, 64, 0, st>>>(sc, overflow, keep_scale);
  ACME_LAUNCH_CHECK();
  split_planes_kernel<<<std::max(grid, 1u), 256, 0, st>>>(x, n4, planes, pstride, sc);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_split_planes_lagged(const float* x, int64_t n, uint16_t* planes, int64_t pstride,
                               gemm::PScale* sc, hipStream_t st) {
  ACME_CHECK_ARG(n % 4 == 0 && pstride % 4 == 0 && sc, "plane split needs multiples of 4");
  const int64_t n4 = n / 4;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n4, 256), 2048);
  split_planes_lagged_kernel<<<std::max(grid, 1u), 256, 0, st>>>(x, n4, planes, pstride, sc);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_param_amax(const float* x, int64_t n, gemm::PScale* sc, hipStream_t st) {
  ACME_CHECK_ARG(x && sc && n % 4 == 0, "bad amax arguments");
  const int64_t n4 = n / 4;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n4, 256 * 8), 1024);
  amax_kernel<<<std::max(grid, 1u), 256, 0, st>>>(x, n4, sc);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_rescale_job(const RescaleJob& job, hipStream_t st) {
  plane_rescale_kernel<<<1, 256, 0, st>>>(job);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_plane_rescale(gemm::PScale* recs, int n_transient, int n, int copy_from, int copy_to,
                         int* overflow, hipStream_t st, int skip_lo, int skip_hi,
                         const RescaleGuard& rg, int defer_r) {
  ACME_CHECK_ARG(recs && overflow && n >= 1 && n <= 15 && n_transient >= 0 && n_transient <= n,
                 "bad rescale arguments");
  ACME_CHECK_ARG(copy_to < 0 || (copy_to >= n && copy_from >= 0 && copy_from < n),
                 "bad rescale copy");
  RescaleJob job;
  job.s = recs;
  job.nt = n_transient;
  job.n = n;
  job.copy_from = copy_from;
  job.copy_to = copy_to;
  job.overflow = overflow;
  job.skip_lo = skip_lo;
  job.skip_hi = skip_hi;
  job.defer_r = defer_r;
  job.rg = rg;
  return launch_rescale_job(job, st);
}

int launch_copy_gated(void* dst0, const void* src0, size_t bytes0, void* dst1, const void* src1,
                      size_t bytes1, const Gate& gate, hipStream_t st) {
  if ((bytes0 | bytes1) % 16 != 0 ||
      ((reinterpret_cast<uintptr_t>(dst0) | reinterpret_cast<uintptr_t>(src0) |
        reinterpret_cast<uintptr_t>(dst1) | reinterpret_cast<uintptr_t>(src1)) & 15) != 0)
    return (set_error("launch_copy_gated: 16-byte sizes and alignment"), ACME_ERR_INVALID);
  const int64_t n0 = (int64_t)(bytes0 / 16), n1 = (int64_t)(bytes1 / 16);
  if (n0 + n1 == 0) return ACME_OK;
  const int64_t blocks = std::min<int64_t>(ceil_div(n0 + n1, 256), 2048);
  copy_gated_kernel<<<(unsigned)blocks, 256, 0, st>>>(
      static_cast<uint4*>(dst0), static_cast<const uint4*>(src0), n0, static_cast<uint4*>(dst1),
      static_cast<const uint4*>(src1), n1, gate);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_gate_publish(const Gate& gate, float* dst, hipStream_t st, const gemm::PScale* s,
                        int n, int skip_lo, int skip_hi) {
  ACME_CHECK_ARG(gate.g && dst && (n == 0 || s), "null argument");
  gate_publish_kernel<<<1, 64, 0, st>>>(gate, dst, s, n, skip_lo, skip_hi);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_frames_f16(const uint8_t* a, const uint8_t* b, int split, int rows, int frame_bytes,
                      uint16_t* out, hipStream_t st) {
  ACME_CHECK_ARG(frame_bytes % 8 == 0, "frame bytes must be a multiple of 8");
  ACME_CHECK_ARG(reinterpret_cast<uintptr_t>(a) % 8 == 0 && reinterpret_cast<uintptr_t>(b) % 8 == 0,
                 "uint8 frame buffers must be 8-byte aligned");
  const int64_t per = frame_bytes / 8;
  const int64_t n8 = per * rows;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n8, 256), 8192);
  frames_f16_kernel<<<std::max(grid, 1u), 256, 0, st>>>(a, b, per * split, n8, out);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_join_planes(const uint16_t* planes, int64_t pstride, int64_t n, float* x,
                       const gemm::PScale* sc, hipStream_t st) {
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n, 256), 4096);
  join_planes_kernel<<<std::max(grid, 1u), 256, 0, st>>>(planes, pstride, n, x, sc);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int launch_clip_adam(const ClipAdamArgs& a, hipStream_t st) {
  ACME_CHECK_ARG(a.p && a.m && a.v && a.g && a.part && a.dev_step, "bad argument");
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(a.n4, 256), 1024);
  clip_adam_kernel<<<std::max(grid, 1u), 256, 0, st>>>(a);
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
  return acme::launch_adam(params, grads, m, v, n, lr, beta1, beta2, eps, t, nullptr, 0,
                           acme::as_stream(stream));
}

int acme_dense_forward(const float* x, int64_t rows, int64_t in, const float* w, const float* b,
                       int64_t out, int32_t act, float* y, void* stream) {
  ACME_CHECK_ARG(x && w && b && y, "null buffer");
  ACME_CHECK_ARG(rows >= 1 && rows < (1 << 30) && in >= 4 && in % 4 == 0 && out >= 4 &&
                     out % 4 == 0 && in < (1 << 30) && out < (1 << 30),
                 "bad dense shape [%lld x %lld] -> %lld", (long long)rows, (long long)in,
                 (long long)out);
  ACME_CHECK_ARG(act >= 0 && act <= 3, "unknown activation %d", act);
  acme::conv::DenseFwd<true> p;
  p.M = (int)rows; p.N = (int)out; p.K = (int)in; p.k_chunk = (int)in;
  p.x = x; p.x2 = x; p.split_b = (int)rows; p.ldx = (int)in;
  p.w = w; p.bias = b; p.y = y; p.act = act; p.slab = nullptr;
  hipError_t e = acme::gemm::launch_matmul<128, 128, 2, 2>(p, 1, acme::as_stream(stream));
  if (e != hipSuccess) {
    acme::set_error("dense launch failed: %s", hipGetErrorString(e));
    return ACME_ERR_HIP;
  }
  return ACME_OK;
}

extern "C++" {
namespace {
template <int BK, int WK>
hipError_t dense_staged(const acme::conv::DenseFwd<true>& p, int multi, hipStream_t st) {
  if (!multi) return acme::gemm::launch_gemm<32, 32, 1, 1, BK, WK>(p, 1, st);
  using Q = acme::conv::DenseFwd<true>;
  acme::gemm::ZMulti<acme::gemm::ZSet<Q, 1>> m;
  const Q one[1] = {p};
  m.s = acme::gemm::make_zset(one);
  m.n = 1;
  const int tiles = ((p.N + 31) / 32) * ((p.M + 31) / 32);
  return acme::gemm::launch_gemm_multi<32, 32, 1, 1, BK, WK>(m, tiles, 1, st);
}
}  // namespace
}  // extern "C++"

int acme_dense_forward_staged(const float* x, int64_t rows, int64_t in, const float* w,
                              const float* b, int64_t out, int32_t act, float* y, int32_t bk,
                              int32_t wk, int32_t multi, void* stream) {
  ACME_CHECK_ARG(x && w && b && y, "null buffer");
  ACME_CHECK_ARG(rows >= 1 && rows < (1 << 30) && in >= 4 && in % 4 == 0 && out >= 4 &&
                     out % 4 == 0 && in < (1 << 30) && out < (1 << 30),
                 "bad dense shape [%lld x %lld] -> %lld", (long long)rows, (long long)in,
                 (long long)out);
  ACME_CHECK_ARG(act >= 0 && act <= 3, "unknown activation %d", act);
  acme::conv::DenseFwd<true> p;
  p.M = (int)rows; p.N = (int)out; p.K = (int)in; p.k_chunk = (int)in;
  p.x = x; p.x2 = x; p.split_b = (int)rows; p.ldx = (int)in;
  p.w = w; p.bias = b; p.y = y; p.act = act; p.slab = nullptr;
  const hipStream_t st = acme::as_stream(stream);
  hipError_t e;
  if (bk == 16 && wk == 8) e = dense_staged<16, 8>(p, multi, st);
  else if (bk == 32 && wk == 4) e = dense_staged<32, 4>(p, multi, st);
  else if (bk == 32 && wk == 8) e = dense_staged<32, 8>(p, multi, st);
  else if (bk == 16 && wk == 16) e = dense_staged<16, 16>(p, multi, st);
  else return (acme::set_error("unsupported (BK %d, WK %d)", bk, wk), ACME_ERR_INVALID);
  if (e != hipSuccess) {
    acme::set_error("dense launch failed: %s", hipGetErrorString(e));
    return ACME_ERR_HIP;
  }
  return ACME_OK;
}

int acme_min_f64(const double* x, int64_t n, double* out_dev, void* stream) {
  ACME_CHECK_ARG(x && out_dev && n >= 1, "bad argument");
  acme::min_f64_kernel<<<1, 1024, 0, acme::as_stream(stream)>>>(x, n, out_dev);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

}  // extern "C"
