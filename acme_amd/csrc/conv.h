// Implicit-GEMM problems for the Q-network layers (NHWC activations, HWIO weights).
//
// Reference layers: snt.Conv2D with Sonnet's default SAME padding and NHWC layout
// (acme/tf/networks/atari.py:41-48), snt.Linear / snt.nets.MLP (duelling.py:37-38).
// TF SAME padding: out = ceil(in / stride), total pad = max((out-1)*s + k - in, 0),
// pad_top = total / 2 (so conv2 of the Nature torso pads 1 top / 2 bottom).
//
// Conventions: W is [KH][KW][CI][CO] (= a [K][CO] matrix, K = KH*KW*CI), bias [CO].
// Forward   : Y[m][co]   = relu(sum_k im2col(X)[m][k] W[k][co] + b[co]),  m = (b,oh,ow)
// Wgrad     : dW[k][co]  = sum_m im2col(X)[m][k] dZ[m][co]  (split over m, f32 slabs)
// Dgrad     : dX[p][ci]  = sum_{kh,kw,co} dZ[b, oh, ow][co] W[kh][kw][ci][co], masked by the
//             previous layer's ReLU (dX is then that layer's dZ).
// dZ always denotes the gradient w.r.t. a layer's pre-activation.
#pragma once

#include "gemm.h"

namespace acme {
namespace conv {

using gemm::f32x4;
using gemm::KCONTIG;
using gemm::RCONTIG;
using gemm::zero4;

template <int IH_, int IW_, int CI_, int OH_, int OW_, int CO_, int KH_, int KW_, int S_,
          int PT_, int PL_>
struct Geom {
  static constexpr int IH = IH_, IW = IW_, CI = CI_, OH = OH_, OW = OW_, CO = CO_;
  static constexpr int KH = KH_, KW = KW_, S = S_, PT = PT_, PL = PL_;
  static constexpr int K = KH * KW * CI;
  static constexpr int IPIX = IH * IW, OPIX = OH * OW;
  static_assert(CI % 4 == 0 && CO % 4 == 0, "channel counts must be multiples of 4");
};

// Input element types: uint8 observations scaled by 1/255 (AtariWrapper to_float,
// acme/wrappers/atari_wrapper.py:284-306) or f32 activations.
struct InU8 {
  using T = uint8_t;
  // float32(x / 255.0) for a byte x: reciprocal multiply + one fma residual correction,
  // which equals the correctly rounded quotient for all 256 byte values (checked
  // exhaustively, tests/test_oracle_cpu.py::test_u8_scaling_exact).
  __device__ static __forceinline__ float scale(uint32_t x) {
    const float xf = (float)x;
    const float c = 1.0f / 255.0f;
    const float q = xf * c;
    return __builtin_fmaf(__builtin_fmaf(-q, 255.0f, xf), c, q);
  }
  __device__ static __forceinline__ f32x4 load4(const uint8_t* p) {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(p);
    return f32x4{scale(w & 0xff), scale((w >> 8) & 0xff), scale((w >> 16) & 0xff),
                 scale(w >> 24)};
  }
};
struct InF32 {
  using T = float;
  __device__ static __forceinline__ f32x4 load4(const float* p) {
    return *reinterpret_cast<const f32x4*>(p);
  }
};

// ------------------------------------------------------------------ forward
template <class G, class In>
struct ConvFwd {
  // B is read k-contiguous: 4 scalar loads w[k..k+3][n] per vector (lanes with
  // consecutive n make each load one coalesced run), so both operands store as rows of
  // 4 consecutive k (conflict-free swizzled LDS, no register transposes).
  static constexpr int A_MODE = KCONTIG, B_MODE = KCONTIG;
  int M, N, K, k_chunk;
  const typename In::T* x;   // rows [0, split_b) of the batch
  const typename In::T* x2;  // rows [split_b, batch) (may alias x)
  int split_b;
  const float* w;
  const float* bias;
  float* y;
  struct ARow {
    const typename In::T* base;
    int ih0, iw0;
    bool ok;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int m) const {
    ARow a;
    a.ok = m < M;
    const int mm = a.ok ? m : 0;
    const int b = mm / G::OPIX, rem = mm - b * G::OPIX;
    const int oh = rem / G::OW, ow = rem - oh * G::OW;
    a.base = b < split_b ? x + (size_t)b * G::IPIX * G::CI
                         : x2 + (size_t)(b - split_b) * G::IPIX * G::CI;
    a.ih0 = oh * G::S - G::PT;
    a.iw0 = ow * G::S - G::PL;
    return a;
  }
  __device__ f32x4 a_load(const ARow& a, int k) const {
    const int kh = k / (G::KW * G::CI), r = k - kh * (G::KW * G::CI);
    const int kw = r / G::CI, ci = r - kw * G::CI;
    const int ih = a.ih0 + kh, iw = a.iw0 + kw;
    if (!a.ok || (unsigned)ih >= (unsigned)G::IH || (unsigned)iw >= (unsigned)G::IW) return zero4();
    return In::load4(a.base + (ih * G::IW + iw) * G::CI + ci);
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ f32x4 b_load(const BRow& b, int k) const {
    if (b.n >= N) return zero4();
    const float* p = w + (size_t)k * G::CO + b.n;
    return f32x4{p[0], p[G::CO], p[2 * G::CO], p[3 * G::CO]};
  }
  __device__ void store(int m, int n, float v, int) const {
    v += bias[n];
    y[(size_t)m * G::CO + n] = v > 0.f ? v : 0.f;
  }
};

// ------------------------------------------------------------------ weight grad
template <class G, class In>
struct ConvWgrad {
  // Row-contiguous operands (4 filter taps / 4 channels at one pixel): measured faster on
  // the f32 engine than k-contiguous 4-pixel gathers on either engine (profiles/r01).
  static constexpr int A_MODE = RCONTIG, B_MODE = RCONTIG;
  static constexpr bool kColSum = true;  // bias gradient = column sums of dZ
  int M, N, K, k_chunk;  // M = G::K rows (kh,kw,ci), N = CO, K = batch * OPIX
  const typename In::T* x;
  const float* dz;  // [batch * OPIX][CO]
  float* slab;      // [splits][M + 1][N]; row M holds the split's bias-gradient partial
  struct ARow {
    int dh, dw, ci;
    bool ok;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int i) const {
    ARow a;
    a.ok = i < M;
    const int ii = a.ok ? i : 0;
    const int kh = ii / (G::KW * G::CI), r = ii - kh * (G::KW * G::CI);
    const int kw = r / G::CI;
    a.ci = r - kw * G::CI;
    a.dh = kh - G::PT;
    a.dw = kw - G::PL;
    return a;
  }
  __device__ f32x4 a_load(const ARow& a, int m) const {
    if (!a.ok) return zero4();
    const int b = m / G::OPIX, rem = m - b * G::OPIX;
    const int oh = rem / G::OW, ow = rem - oh * G::OW;
    const int ih = oh * G::S + a.dh, iw = ow * G::S + a.dw;
    if ((unsigned)ih >= (unsigned)G::IH || (unsigned)iw >= (unsigned)G::IW) return zero4();
    return In::load4(x + ((size_t)b * G::IPIX + ih * G::IW + iw) * G::CI + a.ci);
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ f32x4 b_load(const BRow& b, int m) const {
    if (b.n >= N) return zero4();
    return *reinterpret_cast<const f32x4*>(dz + (size_t)m * G::CO + b.n);
  }
  __device__ void store(int i, int n, float v, int split) const {
    slab[((size_t)split * (M + 1) + i) * N + n] = v;
  }
  __device__ void store_colsum(int n, float v, int split) const {
    slab[((size_t)split * (M + 1) + M) * N + n] = v;
  }
};

// ------------------------------------------------------------------ input grad
// Stride-S input gradient by sub-pixel decomposition: input pixels are grouped by
// parity class (PH, PW) = ((ih + PT) mod S, (iw + PL) mod S); within a class only the
// taps kh = PH + S*jh, kw = PW + S*jw contribute, so each class is a dense implicit GEMM
// with reduction (KH/S)*(KW/S)*CO instead of KH*KW*CO with (S^2-1)/S^2 zeros.
template <class G, int PH, int PW>
struct ConvDgradSub {
  static_assert(G::KH % G::S == 0 && G::KW % G::S == 0, "kernel must be a multiple of stride");
  static constexpr int A_MODE = KCONTIG, B_MODE = KCONTIG;
  static constexpr int S = G::S;
  static constexpr int RH = ((PH - G::PT) % S + S) % S;  // first ih of the class
  static constexpr int RW = ((PW - G::PL) % S + S) % S;
  static constexpr int NH = (G::IH - RH + S - 1) / S;    // class rows
  static constexpr int NW = (G::IW - RW + S - 1) / S;
  static constexpr int JH = G::KH / S, JW = G::KW / S;
  static constexpr int KR = JH * JW * G::CO;             // reduction length
  int M, N, K, k_chunk;  // M = batch * NH * NW, N = CI, K = KR
  const float* dz;
  const float* w;
  const float* xprev;
  float* dx;
  struct ARow {
    const float* base;
    int oh0, ow0;  // (ih + PT - PH) / S, (iw + PL - PW) / S
    bool ok;
  };
  struct BRow {
    int ci;
  };
  __device__ static void decode(int m, int& b, int& ih, int& iw) {
    b = m / (NH * NW);
    const int rem = m - b * (NH * NW);
    const int i = rem / NW, j = rem - i * NW;
    ih = RH + S * i;
    iw = RW + S * j;
  }
  __device__ ARow a_row(int m) const {
    ARow a;
    a.ok = m < M;
    int b, ih, iw;
    decode(a.ok ? m : 0, b, ih, iw);
    a.base = dz + (size_t)b * G::OPIX * G::CO;
    a.oh0 = (ih + G::PT - PH) / S;
    a.ow0 = (iw + G::PL - PW) / S;
    return a;
  }
  __device__ f32x4 a_load(const ARow& a, int k) const {
    const int jh = k / (JW * G::CO), r = k - jh * (JW * G::CO);
    const int jw = r / G::CO, co = r - jw * G::CO;
    const int oh = a.oh0 - jh, ow = a.ow0 - jw;
    if (!a.ok || (unsigned)oh >= (unsigned)G::OH || (unsigned)ow >= (unsigned)G::OW) return zero4();
    return *reinterpret_cast<const f32x4*>(a.base + (oh * G::OW + ow) * G::CO + co);
  }
  __device__ BRow b_row(int ci) const { return BRow{ci}; }
  __device__ f32x4 b_load(const BRow& b, int k) const {
    if (b.ci >= N) return zero4();
    const int jh = k / (JW * G::CO), r = k - jh * (JW * G::CO);
    const int jw = r / G::CO, co = r - jw * G::CO;
    const int kh = PH + S * jh, kw = PW + S * jw;
    return *reinterpret_cast<const f32x4*>(w + ((size_t)(kh * G::KW + kw) * G::CI + b.ci) * G::CO + co);
  }
  __device__ void store(int m, int ci, float v, int) const {
    int b, ih, iw;
    decode(m, b, ih, iw);
    const size_t idx = ((size_t)b * G::IPIX + ih * G::IW + iw) * G::CI + ci;
    dx[idx] = xprev[idx] > 0.f ? v : 0.f;
  }
};
// All S*S parity classes of the sub-pixel input gradient in ONE launch: blockIdx.z is
// the class (the GEMM engines call for_z(z) per block, and z is not a K split), so the
// four class GEMMs share one grid and the CUs hold several blocks at a time.
template <class G>
struct ConvDgradSubZ {
  static_assert(G::KH % G::S == 0 && G::KW % G::S == 0, "kernel must be a multiple of stride");
  static constexpr int A_MODE = KCONTIG, B_MODE = KCONTIG;
  static constexpr bool kZClass = true;
  static constexpr int S = G::S;
  static constexpr int JH = G::KH / S, JW = G::KW / S;
  static constexpr int KR = JH * JW * G::CO;
  int M, N, K, k_chunk;  // M = rows of the largest class (grid), N = CI, K = KR
  int batch;
  const float* dz;
  const float* w;
  const float* xprev;
  float* dx;
  int ph = 0, pw = 0, rh = 0, rw = 0, nh = 1, nw = 1, mc = 0;  // set by for_z
  __device__ ConvDgradSubZ for_z(int z) const {
    ConvDgradSubZ q = *this;
    q.ph = z / S;
    q.pw = z % S;
    q.rh = ((q.ph - G::PT) % S + S) % S;
    q.rw = ((q.pw - G::PL) % S + S) % S;
    q.nh = (G::IH - q.rh + S - 1) / S;
    q.nw = (G::IW - q.rw + S - 1) / S;
    q.mc = batch * q.nh * q.nw;
    return q;
  }
  static int max_rows(int batch) {
    int best = 0;
    for (int ph = 0; ph < S; ++ph)
      for (int pw = 0; pw < S; ++pw) {
        const int rh = ((ph - G::PT) % S + S) % S, rw = ((pw - G::PL) % S + S) % S;
        const int n = batch * ((G::IH - rh + S - 1) / S) * ((G::IW - rw + S - 1) / S);
        best = n > best ? n : best;
      }
    return best;
  }
  struct ARow {
    const float* base;
    int oh0, ow0;
    bool ok;
  };
  struct BRow {
    int ci;
  };
  __device__ void decode(int m, int& b, int& ih, int& iw) const {
    b = m / (nh * nw);
    const int rem = m - b * (nh * nw);
    const int i = rem / nw, j = rem - i * nw;
    ih = rh + S * i;
    iw = rw + S * j;
  }
  __device__ ARow a_row(int m) const {
    ARow a;
    a.ok = m < mc;
    int b, ih, iw;
    decode(a.ok ? m : 0, b, ih, iw);
    a.base = dz + (size_t)b * G::OPIX * G::CO;
    a.oh0 = (ih + G::PT - ph) / S;
    a.ow0 = (iw + G::PL - pw) / S;
    return a;
  }
  __device__ f32x4 a_load(const ARow& a, int k) const {
    const int jh = k / (JW * G::CO), r = k - jh * (JW * G::CO);
    const int jw = r / G::CO, co = r - jw * G::CO;
    const int oh = a.oh0 - jh, ow = a.ow0 - jw;
    if (!a.ok || (unsigned)oh >= (unsigned)G::OH || (unsigned)ow >= (unsigned)G::OW) return zero4();
    return *reinterpret_cast<const f32x4*>(a.base + (oh * G::OW + ow) * G::CO + co);
  }
  __device__ BRow b_row(int ci) const { return BRow{ci}; }
  __device__ f32x4 b_load(const BRow& b, int k) const {
    if (b.ci >= N) return zero4();
    const int jh = k / (JW * G::CO), r = k - jh * (JW * G::CO);
    const int jw = r / G::CO, co = r - jw * G::CO;
    const int kh = ph + S * jh, kw = pw + S * jw;
    return *reinterpret_cast<const f32x4*>(w + ((size_t)(kh * G::KW + kw) * G::CI + b.ci) * G::CO + co);
  }
  __device__ void store(int m, int ci, float v, int) const {
    if (m >= mc) return;
    int b, ih, iw;
    decode(m, b, ih, iw);
    const size_t idx = ((size_t)b * G::IPIX + ih * G::IW + iw) * G::CI + ci;
    dx[idx] = xprev[idx] > 0.f ? v : 0.f;
  }
};

template <class G>
struct ConvDgrad {
  static constexpr int A_MODE = KCONTIG, B_MODE = KCONTIG;
  int M, N, K, k_chunk;  // M = batch * IPIX, N = CI, K = KH*KW*CO
  const float* dz;       // [batch][OH][OW][CO]
  const float* w;        // [KH][KW][CI][CO]
  const float* xprev;    // [batch][IH][IW][CI] post-ReLU activations of the previous layer
  float* dx;             // [batch][IH][IW][CI] = dZ of the previous layer
  struct ARow {
    const float* base;
    int th0, tw0;
    bool ok;
  };
  struct BRow {
    int ci;
  };
  __device__ ARow a_row(int m) const {
    ARow a;
    a.ok = m < M;
    const int mm = a.ok ? m : 0;
    const int b = mm / G::IPIX, rem = mm - b * G::IPIX;
    const int ih = rem / G::IW, iw = rem - ih * G::IW;
    a.base = dz + (size_t)b * G::OPIX * G::CO;
    a.th0 = ih + G::PT;
    a.tw0 = iw + G::PL;
    return a;
  }
  __device__ f32x4 a_load(const ARow& a, int k) const {
    const int kh = k / (G::KW * G::CO), r = k - kh * (G::KW * G::CO);
    const int kw = r / G::CO, co = r - kw * G::CO;
    const int th = a.th0 - kh, tw = a.tw0 - kw;
    if (!a.ok || th < 0 || tw < 0) return zero4();
    if (G::S > 1 && ((th % G::S) != 0 || (tw % G::S) != 0)) return zero4();
    const int oh = th / G::S, ow = tw / G::S;
    if (oh >= G::OH || ow >= G::OW) return zero4();
    return *reinterpret_cast<const f32x4*>(a.base + (oh * G::OW + ow) * G::CO + co);
  }
  __device__ BRow b_row(int ci) const { return BRow{ci}; }
  __device__ f32x4 b_load(const BRow& b, int k) const {
    if (b.ci >= N) return zero4();
    const int kh = k / (G::KW * G::CO), r = k - kh * (G::KW * G::CO);
    const int kw = r / G::CO, co = r - kw * G::CO;
    return *reinterpret_cast<const f32x4*>(w + ((size_t)(kh * G::KW + kw) * G::CI + b.ci) * G::CO + co);
  }
  __device__ void store(int m, int ci, float v, int) const {
    const size_t idx = (size_t)m * G::CI + ci;
    dx[idx] = xprev[idx] > 0.f ? v : 0.f;
  }
};

// ------------------------------------------------------------------ dense layers
// X [rows][ldx] (row stride ldx >= Kin), W [Kin][Nout], Y [rows][Nout].
// VEC: Kin, Nout, ldx multiples of 4 (16-B aligned rows) -> float4 loads.
template <bool VEC>
__device__ __forceinline__ f32x4 load_row4(const float* p, int k, int lim) {
  if (VEC) return *reinterpret_cast<const f32x4*>(p + k);
  f32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = (k + j < lim) ? p[k + j] : 0.f;
  return r;
}

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_ELU = 2, ACT_TANH = 3 };

// Forward activation (tf.nn.relu / tf.nn.elu = expm1 for x < 0 / tf.tanh).
__device__ __forceinline__ float act_fwd(int act, float v) {
  if (act == ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == ACT_ELU) return v < 0.f ? expm1f(v) : v;
  if (act == ACT_TANH) return tanhf(v);
  return v;
}
// Gradient through an activation, from its OUTPUT y (TF's ReluGrad / EluGrad / TanhGrad).
__device__ __forceinline__ float act_bwd(int act, float y, float g) {
  if (act == ACT_RELU) return y > 0.f ? g : 0.f;
  if (act == ACT_ELU) return y < 0.f ? g * (y + 1.f) : g;
  if (act == ACT_TANH) return g * (1.f - y * y);
  return g;
}

template <bool VEC, class In = InF32>
struct DenseFwd {
  static constexpr int A_MODE = KCONTIG, B_MODE = KCONTIG;  // B: 4 scalar loads w[k..k+3][n]
  int M, N, K, k_chunk;
  const typename In::T* x;
  const typename In::T* x2;
  int split_b;
  int ldx;
  const float* w;
  const float* bias;
  float* y;
  int act;
  float* slab = nullptr;  // split-K: raw partial sums [splits][M][N]; finalised later
  struct ARow {
    const typename In::T* p;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int m) const {
    if (m >= M) return ARow{nullptr};
    return ARow{m < split_b ? x + (size_t)m * ldx : x2 + (size_t)(m - split_b) * ldx};
  }
  __device__ f32x4 a_load(const ARow& a, int k) const {
    if (!a.p) return zero4();
    if constexpr (sizeof(typename In::T) == 1) {
      if (VEC) return In::load4(a.p + k);
      f32x4 r;
      for (int j = 0; j < 4; ++j) r[j] = (k + j < K) ? In::scale(a.p[k + j]) : 0.f;
      return r;
    } else {
      return load_row4<VEC>(reinterpret_cast<const float*>(a.p), k, K);
    }
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ f32x4 b_load(const BRow& b, int k) const {
    if (b.n >= N || k >= K) return zero4();
    const float* p = w + (size_t)k * N + b.n;
    return f32x4{p[0], k + 1 < K ? p[N] : 0.f, k + 2 < K ? p[2 * N] : 0.f,
                 k + 3 < K ? p[3 * N] : 0.f};
  }
  __device__ void store(int m, int n, float v, int split) const {
    if (slab) {
      slab[((size_t)split * M + m) * N + n] = v;
      return;
    }
    v += bias[n];
    y[(size_t)m * N + n] = act_fwd(act, v);
  }
  // Prefetched epilogue (gemm.h HasPreStore): the bias of every output loaded up front
  // (bias is required, also with a slab, where it is loaded and not used).
  static constexpr bool kPreStore = true;
  __device__ float pre(int, int n) const { return bias[n]; }
  __device__ float finish(float v, float b) const { return slab ? v : act_fwd(act, v + b); }
  __device__ void put(int m, int n, float v, int split) const {
    if (slab) slab[((size_t)split * M + m) * N + n] = v;
    else y[(size_t)m * N + n] = v;
  }
  // Direct engine (gemm_direct.h): x [M][ldx] rows, W [K][N] columns.  Requires
  // split_b >= M (one input: the descriptor has one base).
  static constexpr bool kStrided = sizeof(typename In::T) == 4;
  static constexpr bool kAVec = VEC, kBVec = false;
  __device__ gemm::StridedOp a_op() const {
    return {reinterpret_cast<const float*>(x), (uint32_t)(4u * M * ldx), 4u * ldx, 4u};
  }
  __device__ gemm::StridedOp b_op() const { return {w, (uint32_t)(4u * K * N), 4u, 4u * N}; }
};

// Weight gradient of a dense layer, single split: dW = X^T dZ written straight into the
// gradient buffer, bias gradient = column sums of dZ (LDS colsum hook).
template <bool VEC, class In = InF32>
struct DenseWgrad {
  // Both operands k-contiguous over 4 consecutive batch rows (4 scalar loads per vector).
  static constexpr int A_MODE = KCONTIG, B_MODE = KCONTIG;
  static constexpr bool kColSum = true;
  int M, N, K, k_chunk;  // M = Kin, N = Nout, K = rows (batch)
  const typename In::T* x;
  int ldx;
  const float* dz;  // [batch][N]
  float* out;       // [M][N] weight gradient
  float* bias_out;  // [N] bias gradient
  struct ARow {
    int i;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int i) const { return ARow{i}; }
  __device__ f32x4 a_load(const ARow& a, int m) const {
    if (a.i >= M || m >= K) return zero4();
    f32x4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (m + j >= K) {
        r[j] = 0.f;
      } else if constexpr (sizeof(typename In::T) == 1) {
        r[j] = In::scale(reinterpret_cast<const uint8_t*>(x)[(size_t)(m + j) * ldx + a.i]);
      } else {
        r[j] = reinterpret_cast<const float*>(x)[(size_t)(m + j) * ldx + a.i];
      }
    }
    return r;
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ f32x4 b_load(const BRow& b, int m) const {
    if (b.n >= N || m >= K) return zero4();
    const float* p = dz + (size_t)m * N + b.n;
    return f32x4{p[0], m + 1 < K ? p[N] : 0.f, m + 2 < K ? p[2 * N] : 0.f,
                 m + 3 < K ? p[3 * N] : 0.f};
  }
  __device__ void store(int i, int n, float v, int) const { out[(size_t)i * N + n] = v; }
  __device__ void store_colsum(int n, float v, int) const {
    if (bias_out) bias_out[n] = v;  // null: a bias gradient another problem writes
  }
  // Direct engine (gemm_direct.h): x [K][ldx] and dz [K][N] read down their columns.
  static constexpr bool kStrided = sizeof(typename In::T) == 4;
  static constexpr bool kAVec = false, kBVec = false;
  __device__ gemm::StridedOp a_op() const {
    return {reinterpret_cast<const float*>(x), (uint32_t)(4u * K * ldx), 4u, 4u * ldx};
  }
  __device__ gemm::StridedOp b_op() const { return {dz, (uint32_t)(4u * K * N), 4u, 4u * N}; }
};

template <bool VEC>
struct DenseDgrad {
  static constexpr int A_MODE = KCONTIG, B_MODE = KCONTIG;
  int M, N, K, k_chunk;  // M = rows, N = Kin, K = Nout
  const float* dz;       // [rows][K]
  const float* w;        // [N][K]
  const float* xprev;    // [rows][ldx] post-ReLU input (mask), may be null (no mask)
  int ldx;
  float* dx;             // [rows][ldx]
  int act = ACT_RELU;    // activation that produced xprev
  struct ARow {
    const float* p;
  };
  struct BRow {
    const float* p;
  };
  __device__ ARow a_row(int m) const { return ARow{m < M ? dz + (size_t)m * K : nullptr}; }
  __device__ f32x4 a_load(const ARow& a, int k) const {
    if (!a.p) return zero4();
    return load_row4<VEC>(a.p, k, K);
  }
  __device__ BRow b_row(int n) const { return BRow{n < N ? w + (size_t)n * K : nullptr}; }
  __device__ f32x4 b_load(const BRow& b, int k) const {
    if (!b.p) return zero4();
    return load_row4<VEC>(b.p, k, K);
  }
  __device__ void store(int m, int n, float v, int) const {
    const size_t idx = (size_t)m * ldx + n;
    if (xprev) v = act_bwd(act, xprev[idx], v);
    dx[idx] = v;
  }
  // Prefetched epilogue (gemm.h HasPreStore): the masks loaded up front (from dx when
  // there is no mask: a valid address whose value is not used).
  static constexpr bool kPreStore = true;
  __device__ float pre(int m, int n) const {
    return (xprev ? xprev : static_cast<const float*>(dx))[(size_t)m * ldx + n];
  }
  __device__ float finish(float v, float xp) const { return xprev ? act_bwd(act, xp, v) : v; }
  __device__ void put(int m, int n, float v, int) const { dx[(size_t)m * ldx + n] = v; }
  // Direct engine (gemm_direct.h): dz [M][K] and W [N][K] rows.
  static constexpr bool kStrided = true;
  static constexpr bool kAVec = VEC, kBVec = VEC;
  __device__ gemm::StridedOp a_op() const { return {dz, (uint32_t)(4u * M * K), 4u * K, 4u}; }
  __device__ gemm::StridedOp b_op() const { return {w, (uint32_t)(4u * N * K), 4u * K, 4u}; }
};

// ------------------------------------------------------------------ duelling head
// DuellingMLP's two output layers (acme/tf/networks/duelling.py:37-57) as ONE skinny
// GEMM over the fused hidden layer h [rows][2H]: output column a < A is the advantage
// (weights wa on the advantage half of h), column A the value (wv on the value half).
// The block-diagonal B operand is synthesised by the loader from the two weight
// tensors.  Split-K partials go to a slab; duel_head_finish applies biases and
// q = v + (adv - mean(adv)).
struct DuelHeadFwd {
  static constexpr int A_MODE = KCONTIG, B_MODE = RCONTIG;
  int M, N, K, k_chunk;  // M = rows, N = A + 1, K = 2H
  int H, A;
  const float* h;
  const float* wv;  // [H]
  const float* wa;  // [H][A]
  float* slab;      // [splits][M][A + 1]
  struct ARow {
    const float* p;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int m) const { return ARow{m < M ? h + (size_t)m * K : nullptr}; }
  __device__ f32x4 a_load(const ARow& a, int k) const {
    if (!a.p) return zero4();
    return *reinterpret_cast<const f32x4*>(a.p + k);
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ float wt(int n, int k) const {
    if (n < A) return k >= H ? wa[(size_t)(k - H) * A + n] : 0.f;
    if (n == A) return k < H ? wv[k] : 0.f;
    return 0.f;
  }
  __device__ f32x4 b_load(const BRow& b, int k) const {
    return f32x4{wt(b.n, k), wt(b.n + 1, k), wt(b.n + 2, k), wt(b.n + 3, k)};
  }
  __device__ void store(int m, int n, float v, int split) const {
    slab[((size_t)split * M + m) * N + n] = v;
  }
};

// Head weight gradients: rows = hidden feature k (2H), columns = head outputs (A + 1),
// reduction over the batch: G[k][n] = sum_b h[b][k] dq_ext[b][n] with
// dq_ext[b][a < A] = g_b (1[a == a_b] - 1/A) (advantage, mean-subtracted) and
// dq_ext[b][A] = g_b (value).  The block-diagonal parts are the weight gradients and the
// column sums of dq_ext the bias gradients (colsum hook).
struct DuelHeadWgrad {
  static constexpr int A_MODE = RCONTIG, B_MODE = RCONTIG;
  static constexpr bool kColSum = true;
  int M, N, K, k_chunk;  // M = 2H, N = A + 1, K = batch
  int A;
  const float* h;        // [batch][2H]
  const float* g;        // [batch]
  const int32_t* act;    // [batch]
  float* slab;           // [splits][M + 1][N]
  struct ARow {
    int i;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int i) const { return ARow{i}; }
  __device__ f32x4 a_load(const ARow& a, int b) const {
    if (a.i >= M) return zero4();
    return *reinterpret_cast<const f32x4*>(h + (size_t)b * M + a.i);
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ f32x4 b_load(const BRow& r, int b) const {
    const float gb = g[b];
    const int ab = act[b];
    const float inv_a = 1.f / (float)A;
    f32x4 out;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = r.n + j;
      out[j] = n < A ? gb * ((n == ab ? 1.f : 0.f) - inv_a) : (n == A ? gb : 0.f);
    }
    return out;
  }
  __device__ void store(int i, int n, float v, int split) const {
    slab[((size_t)split * (M + 1) + i) * N + n] = v;
  }
  __device__ void store_colsum(int n, float v, int split) const {
    slab[((size_t)split * (M + 1) + M) * N + n] = v;
  }
};

}  // namespace conv
}  // namespace acme
