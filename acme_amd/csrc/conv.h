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
  __device__ static __forceinline__ f32x4 load4(const uint8_t* p) {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(p);
    // float32(x / 255.0): exact for all 256 byte values via the correctly rounded
    // f32 division (checked exhaustively, tests/test_oracle_cpu.py).
    return f32x4{__fdiv_rn((float)(w & 0xff), 255.f), __fdiv_rn((float)((w >> 8) & 0xff), 255.f),
                 __fdiv_rn((float)((w >> 16) & 0xff), 255.f), __fdiv_rn((float)(w >> 24), 255.f)};
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
  static constexpr int A_MODE = KCONTIG, B_MODE = RCONTIG;
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
    return *reinterpret_cast<const f32x4*>(w + (size_t)k * G::CO + b.n);
  }
  __device__ void store(int m, int n, float v, int) const {
    v += bias[n];
    y[(size_t)m * G::CO + n] = v > 0.f ? v : 0.f;
  }
};

// ------------------------------------------------------------------ weight grad
template <class G, class In>
struct ConvWgrad {
  static constexpr int A_MODE = RCONTIG, B_MODE = RCONTIG;
  int M, N, K, k_chunk;  // M = G::K rows (kh,kw,ci), N = CO, K = batch * OPIX
  const typename In::T* x;
  const float* dz;  // [batch * OPIX][CO]
  float* slab;      // [splits][M][N]
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
    slab[((size_t)split * M + i) * N + n] = v;
  }
};

// ------------------------------------------------------------------ input grad
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

enum Act { ACT_NONE = 0, ACT_RELU = 1 };

template <bool VEC, class In = InF32>
struct DenseFwd {
  static constexpr int A_MODE = KCONTIG, B_MODE = RCONTIG;
  int M, N, K, k_chunk;
  const typename In::T* x;
  const typename In::T* x2;
  int split_b;
  int ldx;
  const float* w;
  const float* bias;
  float* y;
  int act;
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
      for (int j = 0; j < 4; ++j) r[j] = (k + j < K) ? __fdiv_rn((float)a.p[k + j], 255.f) : 0.f;
      return r;
    } else {
      return load_row4<VEC>(reinterpret_cast<const float*>(a.p), k, K);
    }
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ f32x4 b_load(const BRow& b, int k) const {
    if (b.n >= N || k >= K) return zero4();
    return load_row4<VEC>(w + (size_t)k * N, b.n, N);
  }
  __device__ void store(int m, int n, float v, int) const {
    v += bias[n];
    if (act == ACT_RELU) v = v > 0.f ? v : 0.f;
    y[(size_t)m * N + n] = v;
  }
};

template <bool VEC, class In = InF32>
struct DenseWgrad {
  static constexpr int A_MODE = RCONTIG, B_MODE = RCONTIG;
  int M, N, K, k_chunk;  // M = Kin, N = Nout, K = rows (batch)
  const typename In::T* x;
  int ldx;
  const float* dz;  // [batch][N]
  float* out;       // [splits][M][N] (or the gradient buffer when splits == 1)
  struct ARow {
    int i;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int i) const { return ARow{i}; }
  __device__ f32x4 a_load(const ARow& a, int m) const {
    if (a.i >= M || m >= K) return zero4();
    if constexpr (sizeof(typename In::T) == 1) {
      const uint8_t* p = reinterpret_cast<const uint8_t*>(x) + (size_t)m * ldx;
      if (VEC) return In::load4(p + a.i);
      f32x4 r;
      for (int j = 0; j < 4; ++j) r[j] = (a.i + j < M) ? __fdiv_rn((float)p[a.i + j], 255.f) : 0.f;
      return r;
    } else {
      return load_row4<VEC>(reinterpret_cast<const float*>(x) + (size_t)m * ldx, a.i, M);
    }
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ f32x4 b_load(const BRow& b, int m) const {
    if (b.n >= N || m >= K) return zero4();
    return load_row4<VEC>(dz + (size_t)m * N, b.n, N);
  }
  __device__ void store(int i, int n, float v, int split) const {
    out[((size_t)split * M + i) * N + n] = v;
  }
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
    if (xprev) v = xprev[idx] > 0.f ? v : 0.f;
    dx[idx] = v;
  }
};

}  // namespace conv
}  // namespace acme
