// The snt.LSTM unroll's building blocks shared by the recurrent learners (IMPALA, R2D2):
// the OAR embedding loaders of the input projection (acme/tf/networks/embedding.py:26-45)
// and the per-step cell kernels, forward and BPTT (snt.LSTM: gates = x W_i + h W_h + b
// split as i, f, g, o; c' = sigmoid(f) c + sigmoid(i) tanh(g); h' = sigmoid(o) tanh(c')).
// Included into each learner's translation unit (internal linkage).
#pragma once

#include <hip/hip_runtime.h>

#include "common.h"
#include "conv.h"
#include "gemm.h"

namespace {

using namespace acme;
using namespace acme::conv;

constexpr int kUnits = 8;  // LSTM units per block of the backward cell kernel

__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + expf(-x)); }

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

// ------------------------------------------------------------------ OAR embedding loaders
// Embedding row m = [feat[m][0:F] | one_hot(prev_a[m], A) | tanh(prev_r[m])], D = F + A + 1.
struct Oar {
  const float* feat;  // [rows][F]
  int F, A;
  const int32_t* prev_a;
  const float* prev_r;
  __device__ float at(int m, int k) const {
    if (k < F) return feat[(size_t)m * F + k];
    k -= F;
    if (k < A) return prev_a[m] == k ? 1.f : 0.f;
    return k == A ? tanhf(prev_r[m]) : 0.f;
  }
  __device__ f32x4 four(int m, int k) const {
    if ((F & 3) == 0 && k + 3 < F) return *reinterpret_cast<const f32x4*>(feat + (size_t)m * F + k);
    f32x4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = at(m, k + j);
    return r;
  }
};

// gx = emb @ W_i (+ b when not split): M = rows, N = 4H, K = D.
struct OarFwd {
  static constexpr int A_MODE = gemm::KCONTIG, B_MODE = gemm::RCONTIG;
  int M, N, K, k_chunk;
  Oar x;
  const float* w;     // [D][4H]
  const float* bias;  // [4H]
  float* y;           // [rows][4H]
  float* slab;        // split-K partials [splits][M][N] (bias added by the reduction)
  struct ARow {
    int m;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int m) const { return ARow{m}; }
  __device__ f32x4 a_load(const ARow& a, int k) const {
    if (a.m >= M || k >= K) return gemm::zero4();
    f32x4 r = x.four(a.m, k);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (k + j >= K) r[j] = 0.f;
    return r;
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ f32x4 b_load(const BRow& b, int k) const {
    if (b.n >= N || k >= K) return gemm::zero4();
    return load_row4<true>(w + (size_t)k * N, b.n, N);
  }
  __device__ void store(int m, int n, float v, int split) const {
    if (slab) slab[((size_t)split * M + m) * N + n] = v;
    else y[(size_t)m * N + n] = v + bias[n];
  }
};

// dW_i = emb^T dgates (M = D, N = 4H, K = rows), db = column sums of dgates.
struct OarWgrad {
  static constexpr int A_MODE = gemm::RCONTIG, B_MODE = gemm::RCONTIG;
  static constexpr bool kColSum = true;
  int M, N, K, k_chunk;
  Oar x;
  const float* dz;  // [rows][4H]
  float* out;
  float* bias_out;
  struct ARow {
    int i;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int i) const { return ARow{i}; }
  __device__ f32x4 a_load(const ARow& a, int m) const {
    if (m >= K || a.i >= M) return gemm::zero4();
    f32x4 r = x.four(m, a.i);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (a.i + j >= M) r[j] = 0.f;
    return r;
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ f32x4 b_load(const BRow& b, int m) const {
    if (b.n >= N || m >= K) return gemm::zero4();
    return load_row4<true>(dz + (size_t)m * N, b.n, N);
  }
  __device__ void store(int i, int n, float v, int) const { out[(size_t)i * N + n] = v; }
  __device__ void store_colsum(int n, float v, int) const { bias_out[n] = v; }
};

// ------------------------------------------------------------------ LSTM cell kernels
// kUnits units per block (4 * kUnits = 32 gate columns q * H + u).  The recurrent
// mat-vecs are spread over 256 threads as 32 columns (or units) x 8 (or 32) k-slices with
// 16 batch rows per pass in registers, so every W_h element read feeds 16 FMAs and the
// k-slices are summed once through LDS.
constexpr int kRowChunk = 16;

// Forward step t for all B sequences: z = gx + h_prev @ W_h, then the snt.LSTM cell
// update.  h_prev row b lives at hp + b * hp_stride (the core state for t = 0, the
// previous step's h otherwise).  Row (b, t) of gx / gates / h / c is b * rs_b + t * rs_t
// (batch-major: rs_b = T, rs_t = 1; time-major: rs_b = 1, rs_t = B); grid.y blocks own bc
// batch rows each (lstm_fwd_smem(bc, H) bytes of LDS).  kFwdUnits units per block (16 gate columns); the
// block's W_h columns are staged through LDS in k-chunks with float4 loads.
constexpr int kFwdUnits = 4;
constexpr int kFwdPre = 4;  // float4 loads per thread of h_prev / W_h issued up front

__global__ void __launch_bounds__(256) lstm_fwd_step_kernel(
    const float* __restrict__ gx, const float* __restrict__ wh, const float* __restrict__ hp,
    int64_t hp_stride, const float* __restrict__ cp, int64_t cp_stride, int B, int64_t rs_b,
    int64_t rs_t, int t, int H, float* __restrict__ gates, float* __restrict__ h_out,
    float* __restrict__ c_out, int bc) {
  constexpr int NC = 4 * kFwdUnits;    // gate columns per block (4 segments of kFwdUnits)
  constexpr int KS = 256 / NC;         // k-slices
  static_assert(kRowChunk * NC == 256, "one reduction output per thread");
  const int u0 = blockIdx.x * kFwdUnits;
  {  // this block's batch rows [rb0, rb0 + bc): the pointers start at row rb0
    const int rb0 = blockIdx.y * bc;
    B = min(bc, B - rb0);
    gx += (size_t)rb0 * rs_b * 4 * H;
    hp += (size_t)rb0 * hp_stride;
    cp += (size_t)rb0 * cp_stride;
    gates += (size_t)rb0 * rs_b * 4 * H;
    h_out += (size_t)rb0 * rs_b * H;
    c_out += (size_t)rb0 * rs_b * H;
  }
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* hs = smem;                            // [B][H] (this block's rows)
  float* ws = hs + (size_t)B * H;              // [H][NC]
  float* red = ws + (size_t)H * NC;            // [KS][kRowChunk][NC]
  float* zs = red + KS * kRowChunk * NC;       // [B][NC]
  // Every global load of the step is issued up front (the cell state this thread updates,
  // h_prev, the block's W_h columns as float4 segments), so the step pays one latency.
  const bool cell_thread = (int)threadIdx.x < B * kFwdUnits;  // B <= 64 for one pass
  const float cprev_pre = cell_thread ? cp[(size_t)(threadIdx.x / kFwdUnits) * cp_stride + u0 +
                                           threadIdx.x % kFwdUnits]
                                      : 0.f;
  const int oi = threadIdx.x / NC, occ = threadIdx.x % NC;
  auto gx_at = [&](int ob) {
    return ob < B ? gx[((size_t)ob * rs_b + (size_t)t * rs_t) * 4 * H + (occ / kFwdUnits) * H + u0 +
                       (occ % kFwdUnits)]
                  : 0.f;
  };
  const float gx0 = gx_at(oi);  // the first pass's gx term, in flight with the staging
  const int nh4 = B * H / 4, nw4 = H * 4;
  if (nh4 <= 256 * kFwdPre && nw4 <= 256 * kFwdPre) {
    // Up to kFwdPre float4 of h_prev and of W_h per thread: every load issued (clamped
    // addresses, no branches around them) before the first LDS store, one latency.
    f32x4 hv[kFwdPre], wv[kFwdPre];
#pragma unroll
    for (int q = 0; q < kFwdPre; ++q) {
      const int e = min((int)threadIdx.x + 256 * q, nh4 - 1);
      const int b = e / (H / 4), k = 4 * (e % (H / 4));
      hv[q] = *reinterpret_cast<const f32x4*>(hp + (size_t)b * hp_stride + k);
    }
#pragma unroll
    for (int q = 0; q < kFwdPre; ++q) {
      const int e = min((int)threadIdx.x + 256 * q, nw4 - 1);
      const int k = e / 4, g = e % 4;
      wv[q] = *reinterpret_cast<const f32x4*>(wh + (size_t)k * 4 * H + g * H + u0);
    }
#pragma unroll
    for (int q = 0; q < kFwdPre; ++q) {
      const int e = (int)threadIdx.x + 256 * q;
      if (e < nh4) {
        const int b = e / (H / 4), k = 4 * (e % (H / 4));
        *reinterpret_cast<f32x4*>(hs + (size_t)b * H + k) = hv[q];
      }
    }
#pragma unroll
    for (int q = 0; q < kFwdPre; ++q) {
      const int e = (int)threadIdx.x + 256 * q;
      if (e < nw4) {
        const int k = e / 4, g = e % 4;
        *reinterpret_cast<f32x4*>(ws + (size_t)k * NC + g * kFwdUnits) = wv[q];
      }
    }
  } else {
    // Larger staging (R2D2's H = 512 over tens of rows): rounds of kStageBatch float4 per
    // thread, every load of a round issued before its stores (a load-store pair per
    // iteration paid one memory latency per float4: 25 us per step at B 32, H 512).
    constexpr int kStageBatch = 16;
    for (int e0 = threadIdx.x; e0 < nh4; e0 += 256 * kStageBatch) {
      f32x4 v[kStageBatch];
#pragma unroll
      for (int q = 0; q < kStageBatch; ++q) {
        const int e = min(e0 + 256 * q, nh4 - 1);
        const int b = e / (H / 4), k = 4 * (e % (H / 4));
        v[q] = *reinterpret_cast<const f32x4*>(hp + (size_t)b * hp_stride + k);
      }
      // Stores at the clamped index too (a duplicate store of the same value): a store under
      // a branch let the compiler sink its load into the branch, one exposed latency each.
#pragma unroll
      for (int q = 0; q < kStageBatch; ++q) {
        const int e = min(e0 + 256 * q, nh4 - 1);
        const int b = e / (H / 4), k = 4 * (e % (H / 4));
        *reinterpret_cast<f32x4*>(hs + (size_t)b * H + k) = v[q];
      }
    }
    for (int e0 = threadIdx.x; e0 < nw4; e0 += 256 * kStageBatch) {
      f32x4 v[kStageBatch];
#pragma unroll
      for (int q = 0; q < kStageBatch; ++q) {
        const int e = min(e0 + 256 * q, nw4 - 1);
        const int k = e / 4, g = e % 4;
        v[q] = *reinterpret_cast<const f32x4*>(wh + (size_t)k * 4 * H + g * H + u0);
      }
#pragma unroll
      for (int q = 0; q < kStageBatch; ++q) {
        const int e = min(e0 + 256 * q, nw4 - 1);
        const int k = e / 4, g = e % 4;
        *reinterpret_cast<f32x4*>(ws + (size_t)k * NC + g * kFwdUnits) = v[q];
      }
    }
  }
  __syncthreads();
  const int c = threadIdx.x % NC, sl = threadIdx.x / NC;
  for (int b0 = 0; b0 < B; b0 += kRowChunk) {
    // The gx term of this thread's reduction output.
    const int ob = b0 + oi;
    const float gxv = b0 == 0 ? gx0 : gx_at(ob);
    float acc[kRowChunk];
#pragma unroll
    for (int i = 0; i < kRowChunk; ++i) acc[i] = 0.f;
    // Rows past B read row B - 1 (clamped, no branch around the LDS reads: a branch per
    // row serialised every read behind its own wait); their sums are never stored.
    int roff[kRowChunk];
#pragma unroll
    for (int i = 0; i < kRowChunk; ++i) roff[i] = min(b0 + i, B - 1) * H;
    for (int k = sl; k < H; k += KS) {
      const float w = ws[k * NC + c];
#pragma unroll
      for (int i = 0; i < kRowChunk; ++i) acc[i] = fmaf(hs[roff[i] + k], w, acc[i]);
    }
#pragma unroll
    for (int i = 0; i < kRowChunk; ++i) red[(sl * kRowChunk + i) * NC + c] = acc[i];
    __syncthreads();
    if (ob < B) {  // 256 threads = kRowChunk rows x NC columns
      float z = 0.f;
      for (int s2 = 0; s2 < KS; ++s2) z += red[(s2 * kRowChunk + oi) * NC + occ];
      zs[ob * NC + occ] = gxv + z;
    }
    __syncthreads();
  }
  for (int o = threadIdx.x; o < B * kFwdUnits; o += blockDim.x) {
    const int b = o / kFwdUnits, u = o - b * kFwdUnits, j = u0 + u;
    const float* z = zs + (size_t)b * NC;
    const float ig = sigmoidf(z[u]), fg = sigmoidf(z[kFwdUnits + u]);
    const float gg = tanhf(z[2 * kFwdUnits + u]), og = sigmoidf(z[3 * kFwdUnits + u]);
    const float cprev = o == (int)threadIdx.x && cell_thread ? cprev_pre
                                                             : cp[(size_t)b * cp_stride + j];
    const float cn = __fadd_rn(__fmul_rn(fg, cprev), __fmul_rn(ig, gg));  // no contraction:
    const float hn = __fmul_rn(og, tanhf(cn));  // the persistent kernel computes the same bits
    const size_t row = (size_t)b * rs_b + (size_t)t * rs_t;
    gates[row * 4 * H + j] = ig;
    gates[row * 4 * H + H + j] = fg;
    gates[row * 4 * H + 2 * H + j] = gg;
    gates[row * 4 * H + 3 * H + j] = og;
    c_out[row * H + j] = cn;
    h_out[row * H + j] = hn;
  }
}

size_t lstm_fwd_smem(int B, int H) {
  constexpr int NC = 4 * kFwdUnits;
  return ((size_t)B * H + (size_t)H * NC + (size_t)(256 / NC) * kRowChunk * NC +
          (size_t)B * NC) * sizeof(float);
}

// Backward step t: dh = dh_head[t] + dgates[t+1] @ W_h^T (t < T-1), dc = dc_carry +
// dh o (1 - tanh^2 c), gate gradients (pre-activation), dc_carry <- dc f.  Rows as the
// forward's (b * rs_b + t * rs_t).
__global__ void __launch_bounds__(256) lstm_bwd_step_kernel(
    const float* __restrict__ dh_head, const float* __restrict__ wh, const float* __restrict__ gates,
    const float* __restrict__ c_all, const float* __restrict__ c0, int64_t c0_stride,
    float* __restrict__ dc_carry, float* __restrict__ dgates, int B, int T, int t, int H,
    int64_t rs_b, int64_t rs_t) {
  constexpr int KS = 256 / kUnits;  // 32 k-slices: consecutive threads read consecutive k
  constexpr int KC = 256;           // k-chunk staged in LDS per pass
  __shared__ float red[kUnits][kRowChunk][KS + 1];
  __shared__ __attribute__((aligned(16))) float ds[kRowChunk][KC];
  const int u0 = blockIdx.x * kUnits;
  const int sl = threadIdx.x % KS, u = threadIdx.x / KS;
  const float* w = wh + (size_t)(u0 + u) * 4 * H;
  // The cell-gradient operands of this thread's (unit, row) in the first row pass, loaded
  // before the mat-vec so that their latency overlaps it (clamped addresses, used only by
  // the threads and rows that own them).
  struct CellIn {
    float ig, fg, gg, og, cn, cprev, dh, dc;
  };
  auto cell_in = [&](int b0) {
    const int uu = threadIdx.x / kRowChunk, i = threadIdx.x % kRowChunk;
    const int b = min(b0 + i, B - 1), j = u0 + min(uu, kUnits - 1);
    const size_t row = (size_t)b * rs_b + (size_t)t * rs_t;
    const float* g = gates + row * 4 * H;
    CellIn x;
    x.ig = g[j]; x.fg = g[H + j]; x.gg = g[2 * H + j]; x.og = g[3 * H + j];
    x.cn = c_all[row * H + j];
    x.cprev = t > 0 ? c_all[(row - rs_t) * H + j] : c0[(size_t)b * c0_stride + j];
    x.dh = dh_head[row * H + j];
    x.dc = dc_carry[(size_t)b * H + j];
    return x;
  };
  // grid.y > 1: workgroup y takes the row chunks y, y + gridDim.y, ... (more workgroups in
  // flight for a long batch; the IMPALA learner launches one).
  const int bfirst = blockIdx.y * kRowChunk;
  const CellIn first = cell_in(bfirst);
  for (int b0 = bfirst; b0 < B; b0 += gridDim.y * kRowChunk) {
    float acc[kRowChunk];
#pragma unroll
    for (int i = 0; i < kRowChunk; ++i) acc[i] = 0.f;
    if (t + 1 < T) {
      // Stage dgates[t+1][b0 .. b0+15][kc .. kc+255] with float4 loads (4 per thread) and
      // this thread's 8 W_h values; chunk kc + KC is loaded into registers before chunk kc
      // is computed from LDS, so one load latency is exposed per step instead of one per
      // chunk.  Loads past B or 4H read clamped addresses and are replaced by zeros
      // (selects, not branches around the loads).
      constexpr int NQ = kRowChunk * KC / 4 / 256;
      float wv[KC / KS], wn[KC / KS];
      f32x4 v4[NQ], vn[NQ];
      auto load = [&](int kc, float (&wr)[KC / KS], f32x4 (&vr)[NQ]) {
#pragma unroll
        for (int j = 0; j < KC / KS; ++j) {
          const int k = kc + sl + KS * j;
          const float x = w[min(k, 4 * H - 1)];
          wr[j] = k < 4 * H ? x : 0.f;
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const int e = (int)threadIdx.x + 256 * q;  // float4 index in the chunk
          const int i = e / (KC / 4), k = kc + 4 * (e % (KC / 4));
          const bool ok = b0 + i < B && k < 4 * H;
          const f32x4 x = *reinterpret_cast<const f32x4*>(
              dgates + ((size_t)min(b0 + i, B - 1) * rs_b + (size_t)(t + 1) * rs_t) * 4 * H +
              min(k, 4 * H - 4));
          vr[q] = ok ? x : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      };
      load(0, wv, v4);
      for (int kc = 0; kc < 4 * H; kc += KC) {
        __syncthreads();  // previous chunk fully consumed
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const int e = (int)threadIdx.x + 256 * q;
          *reinterpret_cast<f32x4*>(&ds[e / (KC / 4)][4 * (e % (KC / 4))]) = v4[q];
        }
        __syncthreads();
        // The next chunk (the last one again at the end: no branch around the loads, whose
        // join would wait for them before the compute below).
        load(kc + KC < 4 * H ? kc + KC : kc, wn, vn);
#pragma unroll
        for (int j = 0; j < KC / KS; ++j) {
          const int k = sl + KS * j;
#pragma unroll
          for (int i = 0; i < kRowChunk; ++i) acc[i] = fmaf(ds[i][k], wv[j], acc[i]);
        }
#pragma unroll
        for (int j = 0; j < KC / KS; ++j) wv[j] = wn[j];
#pragma unroll
        for (int q = 0; q < NQ; ++q) v4[q] = vn[q];
      }
    }
#pragma unroll
    for (int i = 0; i < kRowChunk; ++i) red[u][i][sl] = acc[i];
    __syncthreads();
    if ((int)threadIdx.x < kUnits * kRowChunk) {
      const int uu = threadIdx.x / kRowChunk, i = threadIdx.x % kRowChunk, b = b0 + i;
      if (b < B) {
        float dhn = 0.f;
        for (int s2 = 0; s2 < KS; ++s2) dhn += red[uu][i][s2];
        const int j = u0 + uu;
        const size_t row = (size_t)b * rs_b + (size_t)t * rs_t;
        const CellIn x = b0 == bfirst ? first : cell_in(b0);
        const float ig = x.ig, fg = x.fg, gg = x.gg, og = x.og;
        const float cn = x.cn, cprev = x.cprev;
        const float tc = tanhf(cn);
        const float dh = x.dh + dhn;
        const float dc = x.dc + dh * og * (1.f - tc * tc);
        float* dg = dgates + row * 4 * H;
        dg[j] = dc * gg * ig * (1.f - ig);
        dg[H + j] = dc * cprev * fg * (1.f - fg);
        dg[2 * H + j] = dc * ig * (1.f - gg * gg);
        dg[3 * H + j] = dh * tc * og * (1.f - og);
        dc_carry[(size_t)b * H + j] = dc * fg;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- persistent unroll
// The whole LSTM forward (and, below, BPTT) in ONE launch: workgroup (rg, cg) owns kRgRows
// batch rows (a row group) x kRgUnits units (cg), i.e. 4 * kRgUnits gate columns, and keeps
// its W_h slice (all H k of those columns) in registers for the whole unroll.  A step needs
// h_{t-1} of its own rows only (the sequences are independent), so each workgroup exchanges
// kRgRows x H values per step with the H / kRgUnits workgroups of its row group, as 8-byte
// {tag, value} granules (agent-scope relaxed atomic stores and loads: the data is its own
// flag, cdna_hip_programming.md G16 / MI355X_MICROARCH.md "handoff-1to1").  Two granule
// buffers alternate by step parity; a workgroup cannot publish step t + 1 before every
// workgroup of its row group has published step t, i.e. finished reading step t - 1, so a
// buffer is only rewritten after its readers are done.  Spins are bounded: a timeout writes
// `tmo` and every workgroup leaves the kernel (the learner's logged loss then reads NaN).
// The workgroups must be co-resident: at most 256 of them (ceil(B / 4) x H / 16), H
// threads each, which an idle MI355X dispatches at once (hipLaunchCooperativeKernel would
// guarantee it but measured a 13.5 us gap before and after each launch).  Granule tags carry
// a per-launch epoch, so the buffers are not cleared between launches.  A row group's
// workgroups share blockIdx % RG, i.e. one XCD (one L2) when RG = 8.
// Rows (b, t) of gx / gates / h / c / dh / dgates are b * rs_b + t * rs_t (IMPALA batch-major,
// R2D2 time-major).  H = 256 (IMPALA): 2.5 us per step (hand-off 0.9, mat-vec 0.6, cell 0.7).
using gu64 = __attribute__((address_space(1))) unsigned long long;
using gu32 = __attribute__((address_space(1))) unsigned;
constexpr unsigned kSpinLimit = 1u << 22;
constexpr int kRgRows = 4;    // batch rows per row group (2: twice the workgroups, small B)
constexpr int kRgUnits = 16;  // units per workgroup: 64 gate columns
constexpr int kRgCols = 4 * kRgUnits;

// A workgroup has NT = H threads (H / 64 waves), so every thread holds the same W_h share
// (64 floats) and takes the same 4 granules per step at any H.
template <int H, int R = kRgRows>
struct RgShape {
  static_assert(H == 256 || H == 512, "persistent unroll: H of 256 or 512");
  static_assert(R == 1 || R == 2 || R == 4, "persistent unroll: 1, 2 or 4 rows per row group");
  static constexpr int NT = H;                     // threads per workgroup
  static constexpr int G = H / kRgUnits;           // workgroups per row group
  static constexpr int NS = NT / 16;               // forward: k-slices
  static constexpr int KW = H / NS;                // forward: k per slice (16)
  static constexpr int HV = R * H / NT;            // forward: h values brought in per thread
  static constexpr int UT = H / 4;                 // backward: threads per gate-column slice
  static constexpr int GS = NT / UT;               // backward: gate-column slices (4)
  static constexpr int GW = kRgCols / GS;          // backward: gate columns per slice (16)
  static constexpr int PV = G * R * kRgUnits / NT; // backward: granules per thread (R)
};

__device__ __forceinline__ void put_granule(unsigned long long* g, unsigned tag, float v) {
  __hip_atomic_store((gu64*)(g), ((unsigned long long)tag << 32) | __float_as_uint(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Waits until the N granules at g[k] (per-thread list, `live` masks absent rows) carry `tag`,
// then returns their values; false on timeout (after writing `tmo`).
template <int N>
__device__ bool take_granules(const unsigned long long* const (&g)[N], const bool (&live)[N],
                              unsigned tag, float (&out)[N], unsigned* tmo) {
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const unsigned long long v =
          live[k] ? __hip_atomic_load((const gu64*)(g[k]), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT)
                  : ((unsigned long long)tag << 32);
      out[k] = __uint_as_float((unsigned)v);
      ok &= (unsigned)(v >> 32) == tag;
    }
    if (__all(ok)) return true;
    if (spins >= kSpinLimit) {
      if ((threadIdx.x & 63) == 0)
        __hip_atomic_store((gu32*)(tmo), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

using f32x2 = __attribute__((ext_vector_type(2))) float;

// Rows (r, r + 1) of a mat-vec in one packed FMA (v_pk_fma_f32): each row's sum keeps its
// own order, so the result is the scalar loop's.
__device__ __forceinline__ f32x2 fma2(float a0, float a1, float w, f32x2 acc) {
  return __builtin_elementwise_fma(f32x2{a0, a1}, f32x2{w, w}, acc);
}

// Global gate column of this workgroup's gate column `col` (gate q = col / kRgUnits).
template <int H>
__device__ __forceinline__ int rg_gate_col(int cg, int col) {
  return (col / kRgUnits) * H + cg * kRgUnits + col % kRgUnits;
}

// Per-step timestamps of workgroup 0 (wall_clock64, 100 MHz) into trace[4 t + i] when a
// trace buffer is given (debug_buffer "lstm_trace", ACME_V_RGTRACE=1 at creation).
#define RG_STAMP(i)                                                  \
  do {                                                               \
    if (trace && blockIdx.x == 0 && threadIdx.x == 0)                \
      trace[(size_t)t * 4 + (i)] = (unsigned long long)wall_clock64(); \
  } while (0)

// Forward: thread (ks = tid / 16, cq = tid % 16) accumulates 4 rows x 4 gate columns over
// the 16-k slice ks (W in registers, h_{t-1} broadcast from LDS: each h value read feeds 4
// columns x 2 rows, LDS return bandwidth rather than the FMAs bounds the step); the H / 16
// slices are summed in order with gx; threads < 64 run the cells (c in registers).
template <int H, int R = kRgRows>
__global__ void __launch_bounds__(H) lstm_fwd_rg_kernel(
    const float* __restrict__ gx, const float* __restrict__ wh, const float* __restrict__ h0,
    int64_t h0_stride, const float* __restrict__ c0, int64_t c0_stride, int B, int T,
    int64_t rs_b, int64_t rs_t, float* __restrict__ gates, float* __restrict__ h_out,
    float* __restrict__ c_out, unsigned long long* xg, unsigned tag0, unsigned* tmo,
    unsigned long long* trace = nullptr) {
  using S = RgShape<H, R>;
  constexpr int U = kRgUnits, NC = kRgCols, KW = S::KW, HV = S::HV, NS = S::NS;
  // H = 512: the next step's gx is prefetched and the 32 slices are summed in two halves by
  // all threads (a 32-long dependent chain of LDS reads in the 64 cell threads took 1.8 us
  // per step); H = 256 keeps IMPALA's order and schedule.
  constexpr bool kWide = H > 256;
  static_assert(!kWide || R == 4, "H = 512: 4 rows per row group");
  __shared__ __attribute__((aligned(16))) float hs[R][H];
  __shared__ float red[NS][R][NC];
  __shared__ float red2[2][R * NC];
  __shared__ int s_fail;
  const int RG = (B + R - 1) / R;
  const int rg = blockIdx.x % RG, cg = blockIdx.x / RG;
  const int b0 = rg * R;
  const int tid = threadIdx.x, cq = tid & 15, ks = tid >> 4;
  if (tid == 0) s_fail = 0;
  float w[4][KW];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int gc = rg_gate_col<H>(cg, 4 * cq + c);
#pragma unroll
    for (int kk = 0; kk < KW; ++kk) w[c][kk] = wh[(size_t)(ks * KW + kk) * 4 * H + gc];
  }
  // Cell threads: (row, unit) = (tid / U, tid % U) for tid < R * U.
  const bool cell = tid < R * U;
  const int crow = tid / U, cu = tid % U, cb = min(b0 + crow, B - 1), cj = cg * U + cu;
  const bool cell_live = cell && b0 + crow < B;
  float creg = cell ? c0[(size_t)cb * c0_stride + cj] : 0.f;
  // The HV h_{t-1} values this thread brings into LDS: e = HV tid + i -> (row e / H, unit).
  const unsigned long long* gp[HV];
  bool glive[HV];
  // The cell's gx terms (its four gate columns) of step t: loaded at the step's start, or
  // (kWide) once step t - 1's h_{t-2} had arrived, so their latency overlaps a whole step.
  float gxv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    gxv[q] = kWide && cell ? gx[(size_t)cb * rs_b * 4 * H + q * H + cj] : 0.f;
  for (int t = 0; t < T; ++t) {
    RG_STAMP(0);
    if (!kWide) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        gxv[q] = cell ? gx[((size_t)cb * rs_b + (size_t)t * rs_t) * 4 * H + q * H + cj] : 0.f;
    }
    float hv[HV];
    if (t == 0) {
#pragma unroll
      for (int i = 0; i < HV; ++i) {
        const int e = HV * tid + i, r = e / H, u = e % H;
        hv[i] = h0[(size_t)min(b0 + r, B - 1) * h0_stride + u];
      }
    } else {
      const unsigned long long* base = xg + (size_t)((t - 1) & 1) * B * H;
#pragma unroll
      for (int i = 0; i < HV; ++i) {
        const int e = HV * tid + i, r = e / H, u = e % H;
        glive[i] = b0 + r < B;
        gp[i] = base + (size_t)min(b0 + r, B - 1) * H + u;
      }
      if (!take_granules<HV>(gp, glive, tag0 + (unsigned)t, hv, tmo)) s_fail = 1;
    }
    RG_STAMP(1);
    float gxn[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      gxn[q] = kWide && cell && t + 1 < T
                   ? gx[((size_t)cb * rs_b + (size_t)(t + 1) * rs_t) * 4 * H + q * H + cj]
                   : 0.f;
    if constexpr (HV % 4 == 0) {
#pragma unroll
      for (int i = 0; i < HV; i += 4)
        *reinterpret_cast<f32x4*>(&hs[0][0] + HV * tid + i) =
            f32x4{hv[i], hv[i + 1], hv[i + 2], hv[i + 3]};
    } else if constexpr (HV == 1) {
      (&hs[0][0])[tid] = hv[0];
    } else {
#pragma unroll
      for (int i = 0; i < HV; i += 2)
        *reinterpret_cast<f32x2*>(&hs[0][0] + HV * tid + i) = f32x2{hv[i], hv[i + 1]};
    }
    __syncthreads();
    if (s_fail) return;  // every workgroup leaves on a timeout (its own wait fails too)
    if constexpr (R == 1) {  // one row: scalar FMAs, the same per-row order
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k4 = 0; k4 < KW / 4; ++k4) {
        const f32x4 h = *reinterpret_cast<const f32x4*>(&hs[0][ks * KW + 4 * k4]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[c] = fmaf(h[j], w[c][4 * k4 + j], acc[c]);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) red[ks][0][4 * cq + c] = acc[c];
    } else {
    f32x2 acc[R / 2][4];  // per row pair (2p, 2p + 1) and column
#pragma unroll
    for (int pr = 0; pr < R / 2; ++pr)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[pr][c] = f32x2{0.f, 0.f};
#pragma unroll
    for (int k4 = 0; k4 < KW / 4; ++k4) {
      const int k0 = ks * KW + 4 * k4;
      f32x4 hr[R];
#pragma unroll
      for (int r = 0; r < R; ++r) hr[r] = *reinterpret_cast<const f32x4*>(&hs[r][k0]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int pr = 0; pr < R / 2; ++pr)
            acc[pr][c] = fma2(hr[2 * pr][j], hr[2 * pr + 1][j], w[c][4 * k4 + j], acc[pr][c]);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int pr = 0; pr < R / 2; ++pr) {
        red[ks][2 * pr][4 * cq + c] = acc[pr][c][0];
        red[ks][2 * pr + 1][4 * cq + c] = acc[pr][c][1];
      }
    }
    __syncthreads();
    if (kWide) {  // thread (half, output): the half's NS / 2 slices of one of R x NC outputs
      const int o = tid % (R * NC), half = tid / (R * NC);
      const float* rp = &red[half * (NS / 2)][0][0] + o;
      float sum = rp[0];
#pragma unroll
      for (int k = 1; k < NS / 2; ++k) sum += rp[k * R * NC];
      red2[half][o] = sum;
      __syncthreads();
    }
    RG_STAMP(2);
    if (cell) {
      // z = gx + the NS k-slices' partial sums, in order (kWide: two halves in order).
      float z[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cc = q * U + cu;
        float sum;
        if (kWide) {
          sum = red2[0][crow * NC + cc] + red2[1][crow * NC + cc];
        } else {
          sum = red[0][crow][cc];
#pragma unroll
          for (int k = 1; k < NS; ++k) sum += red[k][crow][cc];
        }
        z[q] = gxv[q] + sum;
      }
      const float ig = sigmoidf(z[0]), fg = sigmoidf(z[1]);
      const float gg = tanhf(z[2]), og = sigmoidf(z[3]);
      const float cn = __fadd_rn(__fmul_rn(fg, creg), __fmul_rn(ig, gg));
      const float hn = __fmul_rn(og, tanhf(cn));
      creg = cn;
      if (cell_live) {
        const size_t row = (size_t)cb * rs_b + (size_t)t * rs_t;
        gates[row * 4 * H + cj] = ig;
        gates[row * 4 * H + H + cj] = fg;
        gates[row * 4 * H + 2 * H + cj] = gg;
        gates[row * 4 * H + 3 * H + cj] = og;
        c_out[row * H + cj] = cn;
        h_out[row * H + cj] = hn;
        if (t + 1 < T) put_granule(xg + (size_t)(t & 1) * B * H + (size_t)cb * H + cj,
                                   tag0 + (unsigned)(t + 1), hn);
      }
    }
    RG_STAMP(3);
    if (kWide) {
#pragma unroll
      for (int q = 0; q < 4; ++q) gxv[q] = gxn[q];
    }
  }
}

// Backward: per step t (T-1 .. t_stop) the cells of (row group, unit group) take dh =
// dh_head + the partial products published at step t + 1 (summed over the G producers in
// order), form their gate gradients (dgates, stored) and carry dc in registers; then thread
// (gs = tid / UT, uq = tid % UT) forms its 4 units' share of this workgroup's partial
// product for dh_{t-1} over the gate-column slice gs (W_h row slice in registers), and the
// slices are summed in order and published (4 rows x H values), each consumer reading its 16
// units of every producer.  BPTT stops at t_stop (R2D2's burn-in: no gradient into it).
template <int H, int R = kRgRows>
__global__ void __launch_bounds__(H) lstm_bwd_rg_kernel(
    const float* __restrict__ dh_head, const float* __restrict__ wh,
    const float* __restrict__ gates, const float* __restrict__ c_all,
    const float* __restrict__ c0, int64_t c0_stride, int B, int T, int t_stop, int64_t rs_b,
    int64_t rs_t, float* __restrict__ dgates, unsigned long long* xb, unsigned tag0,
    unsigned* tmo, unsigned long long* trace = nullptr) {
  using S = RgShape<H, R>;
  constexpr int U = kRgUnits, NC = kRgCols, G = S::G;
  constexpr int UT = S::UT, GS = S::GS, GW = S::GW, PV = S::PV, NT = S::NT;
  // H = 512: the 32 producers' partials are summed by all threads in 8 groups of 4, then by
  // the cells over the 8 groups in order (IMPALA's H = 256 keeps one chain of 16).
  constexpr bool kWide = H > 256;
  static_assert(!kWide || R == 4, "H = 512: 4 rows per row group");
  constexpr int PG = NT / (R * U);  // producer groups (kWide)
  __shared__ float pp[G][R][U];
  __shared__ float pp2[PG][R * U];
  __shared__ __attribute__((aligned(16))) float dgs[R][NC];
  __shared__ float red[GS][R][H];
  __shared__ int s_fail;
  const int RG = (B + R - 1) / R;
  const int rg = blockIdx.x % RG, cg = blockIdx.x / RG;
  const int b0 = rg * R;
  const int tid = threadIdx.x;
  const int uq = tid % UT, gs = tid / UT;
  if (tid == 0) s_fail = 0;
  float w[4][GW];  // W_h[4 uq + uu][this workgroup's gate column GW gs + gg]
#pragma unroll
  for (int uu = 0; uu < 4; ++uu)
#pragma unroll
    for (int gg = 0; gg < GW; ++gg)
      w[uu][gg] = wh[(size_t)(4 * uq + uu) * 4 * H + rg_gate_col<H>(cg, GW * gs + gg)];
  const bool cell = tid < R * U;
  const int crow = tid / U, cu = tid % U, cb = min(b0 + crow, B - 1), cj = cg * U + cu;
  const bool cell_live = cell && b0 + crow < B;
  float dcarry = 0.f;
  // Granules this thread takes: e = PV tid + i -> (producer e / (R U), row, unit).
  const unsigned long long* gp[PV];
  bool glive[PV];
  // Cell operands of step t; step t - 1's are loaded once step t's partial products have
  // arrived, so their latency overlaps a whole step.
  struct CellOps {
    float ig, fg, gg, og, cn, cprev, dhh;
  };
  auto cell_ops = [&](int t) {
    CellOps x{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (cell) {
      const size_t row = (size_t)cb * rs_b + (size_t)t * rs_t;
      const float* gr = gates + row * 4 * H;
      x.ig = gr[cj]; x.fg = gr[H + cj]; x.gg = gr[2 * H + cj]; x.og = gr[3 * H + cj];
      x.cn = c_all[row * H + cj];
      x.cprev = t > 0 ? c_all[(row - rs_t) * H + cj] : c0[(size_t)cb * c0_stride + cj];
      x.dhh = dh_head[row * H + cj];
    }
    return x;
  };
  CellOps ops = cell_ops(T - 1);
  for (int t = T - 1; t >= t_stop; --t) {
    RG_STAMP(0);
    const size_t row = (size_t)cb * rs_b + (size_t)t * rs_t;
    const float ig = ops.ig, fg = ops.fg, gg = ops.gg, og = ops.og, cn = ops.cn;
    const float cprev = ops.cprev, dhh = ops.dhh;
    if (t + 1 < T) {
      const unsigned long long* base = xb + (size_t)((t + 1) & 1) * G * B * H;
      float v[PV];
#pragma unroll
      for (int i = 0; i < PV; ++i) {
        const int e = PV * tid + i, pg = e / (R * U), r = (e / U) % R, u = e % U;
        glive[i] = b0 + r < B;
        gp[i] = base + ((size_t)pg * B + min(b0 + r, B - 1)) * H + cg * U + u;
      }
      if (!take_granules<PV>(gp, glive, tag0 + (unsigned)(t + 1), v, tmo)) s_fail = 1;
#pragma unroll
      for (int i = 0; i < PV; ++i) (&pp[0][0][0])[PV * tid + i] = v[i];
    }
    RG_STAMP(1);
    if (t > t_stop) ops = cell_ops(t - 1);
    __syncthreads();
    if (s_fail) return;
    if (kWide && t + 1 < T) {
      const int o = tid % (R * U), part = tid / (R * U);
      const float* src = &pp[part * (G / PG)][0][0] + o;
      float sum = src[0];
#pragma unroll
      for (int k = 1; k < G / PG; ++k) sum += src[k * R * U];
      pp2[part][o] = sum;
      __syncthreads();
    }
    if (cell) {
      float dhn = 0.f;
      if (t + 1 < T) {
        if (kWide) {
#pragma unroll
          for (int part = 0; part < PG; ++part) dhn += pp2[part][tid];
        } else {
          for (int pg = 0; pg < G; ++pg) dhn += pp[pg][crow][cu];
        }
      }
      const float tc = tanhf(cn);
      const float dh = dhh + dhn;
      const float dc = dcarry + dh * og * (1.f - tc * tc);
      const float di = dc * gg * ig * (1.f - ig), df = dc * cprev * fg * (1.f - fg);
      const float dg = dc * ig * (1.f - gg * gg), dO = dh * tc * og * (1.f - og);
      dcarry = dc * fg;
      dgs[crow][cu] = di;
      dgs[crow][U + cu] = df;
      dgs[crow][2 * U + cu] = dg;
      dgs[crow][3 * U + cu] = dO;
      if (cell_live) {
        float* d = dgates + row * 4 * H;
        d[cj] = di;
        d[H + cj] = df;
        d[2 * H + cj] = dg;
        d[3 * H + cj] = dO;
      }
    }
    __syncthreads();
    RG_STAMP(2);
    if (t > t_stop) {
      if constexpr (R == 1) {  // one row: scalar FMAs, the same per-row order
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int g4 = 0; g4 < GW / 4; ++g4) {
          const f32x4 d = *reinterpret_cast<const f32x4*>(&dgs[0][GW * gs + 4 * g4]);
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int uu = 0; uu < 4; ++uu) acc[uu] = fmaf(d[j], w[uu][4 * g4 + j], acc[uu]);
        }
#pragma unroll
        for (int uu = 0; uu < 4; ++uu) red[gs][0][4 * uq + uu] = acc[uu];
      } else {
      f32x2 acc[R / 2][4];  // per row pair (2p, 2p + 1) and unit
#pragma unroll
      for (int pr = 0; pr < R / 2; ++pr)
#pragma unroll
        for (int uu = 0; uu < 4; ++uu) acc[pr][uu] = f32x2{0.f, 0.f};
#pragma unroll
      for (int g4 = 0; g4 < GW / 4; ++g4) {
        f32x4 dr[R];
#pragma unroll
        for (int r = 0; r < R; ++r) dr[r] = *reinterpret_cast<const f32x4*>(&dgs[r][GW * gs + 4 * g4]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int uu = 0; uu < 4; ++uu)
#pragma unroll
            for (int pr = 0; pr < R / 2; ++pr)
              acc[pr][uu] = fma2(dr[2 * pr][j], dr[2 * pr + 1][j], w[uu][4 * g4 + j], acc[pr][uu]);
      }
#pragma unroll
      for (int uu = 0; uu < 4; ++uu)
#pragma unroll
        for (int pr = 0; pr < R / 2; ++pr) {
          red[gs][2 * pr][4 * uq + uu] = acc[pr][uu][0];
          red[gs][2 * pr + 1][4 * uq + uu] = acc[pr][uu][1];
        }
      }
      __syncthreads();
      // Thread u = tid publishes this workgroup's partial for its unit, R rows (the
      // gate-column slices summed in order).
      unsigned long long* out = xb + (size_t)(t & 1) * G * B * H + (size_t)cg * B * H;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (b0 + r >= B) continue;
        float v = red[0][r][tid];
#pragma unroll
        for (int k = 1; k < GS; ++k) v += red[k][r][tid];
        put_granule(out + (size_t)(b0 + r) * H + tid, tag0 + (unsigned)t, v);
      }
    }
    RG_STAMP(3);
  }
}
#undef RG_STAMP

// gx = OAR(emb) @ W_i + b from the plane GEMM's split-K partials of feat @ W_i[0:F]: the
// one-hot(prev a) row of W_i, tanh(prev r) times its last row and the bias are added here
// (the embedding's last A + 1 columns), one thread per (row, 4 gate columns).
__global__ void __launch_bounds__(256) oar_finish_kernel(const float* __restrict__ slab,
                                                         int splits, int rows, int N,
                                                         const float* __restrict__ wi_tail,
                                                         const float* __restrict__ bias,
                                                         const int32_t* __restrict__ prev_a,
                                                         const float* __restrict__ prev_r, int A,
                                                         float* __restrict__ gx) {
  const int n4 = N / 4;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * n4) return;
  const int m = (int)(i / n4), c = (int)(i - (int64_t)m * n4);
  const int64_t cnt = (int64_t)rows * N;
  f32x4 v = reinterpret_cast<const f32x4*>(slab)[i];
  for (int s = 1; s < splits; ++s) v += reinterpret_cast<const f32x4*>(slab + s * cnt)[i];
  const int a = prev_a[m];
  const float tr = tanhf(prev_r[m]);
  const f32x4 wa = reinterpret_cast<const f32x4*>(wi_tail + (size_t)a * N)[c];
  const f32x4 wr = reinterpret_cast<const f32x4*>(wi_tail + (size_t)A * N)[c];
  const f32x4 b = reinterpret_cast<const f32x4*>(bias)[c];
  f32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = ((v[j] + wa[j]) + tr * wr[j]) + b[j];
  reinterpret_cast<f32x4*>(gx)[i] = o;
}

// The last A + 1 rows of dW_i (the one-hot and tanh(prev r) embedding columns):
// dW[F + j][n] = sum over rows with prev_a == j of dgates[m][n], dW[F + A][n] = sum of
// tanh(prev_r[m]) dgates[m][n].  One pass over dgates: block = 64 columns x W waves (W =
// blockDim.x / 64), wave w takes rows m = w, w + W, ... (kTailBatch loads in flight per
// lane).  A row's action is wave-uniform, so the wave adds the row into its own LDS
// accumulator row [w][a][lane]; the W wave partials of each output are then added in wave
// order.  Deterministic.  (One block per output row, each re-reading all of dgates with 80
// dependent loads per wave, took 21.6 us.)
constexpr int kTailBatch = 10;
inline int tail_waves(int A) { return A + 1 <= 32 ? 8 : 4; }  // LDS W (A + 1) 256 B <= 64 KB
__global__ void __launch_bounds__(512) oar_wgrad_tail_kernel(
    const float* __restrict__ dg, int rows, int N, const int32_t* __restrict__ prev_a,
    const float* __restrict__ prev_r, int A, float* __restrict__ dw_tail) {
  extern __shared__ float tacc[];  // [W][A + 1][64]
  const int W = blockDim.x >> 6;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + lane, nc = min(n, N - 1);
  const int J = A + 1;
  float* my = tacc + (size_t)wave * J * 64;
  for (int j = 0; j < J; ++j) my[j * 64 + lane] = 0.f;
  float racc = 0.f;
  for (int m0 = wave; m0 < rows; m0 += W * kTailBatch) {
    float g[kTailBatch], tr[kTailBatch];
    int act[kTailBatch];
#pragma unroll
    for (int b = 0; b < kTailBatch; ++b) {
      const int mc = min(m0 + b * W, rows - 1);
      g[b] = dg[(size_t)mc * N + nc];
      act[b] = prev_a[mc];
      tr[b] = prev_r[mc];
    }
#pragma unroll
    for (int b = 0; b < kTailBatch; ++b) {
      if (m0 + b * W >= rows) break;
      const int a = __builtin_amdgcn_readfirstlane(act[b]);
      if ((unsigned)a < (unsigned)A) my[a * 64 + lane] += g[b];
      racc = fmaf(tanhf(tr[b]), g[b], racc);
    }
  }
  my[A * 64 + lane] = racc;
  __syncthreads();
  for (int e = threadIdx.x; e < J * 64; e += blockDim.x) {
    const int j = e >> 6, nn = blockIdx.x * 64 + (e & 63);
    if (nn >= N) continue;
    float t = tacc[e];
    for (int w = 1; w < W; ++w) t += tacc[(size_t)w * J * 64 + e];
    dw_tail[(size_t)j * N + nn] = t;
  }
}

}  // namespace
