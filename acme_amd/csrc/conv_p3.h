// Plane-operand implicit-GEMM problems of the Nature DQN network (gemm_p3.h engine).
//
// Same layers, conventions and TF SAME padding as conv.h (NHWC activations, HWIO
// weights, dZ = gradient w.r.t. a layer's pre-activation); the difference is storage:
// every f32 activation / gradient / weight operand is read from, and every activation /
// gradient result written to, scaled two-plane f16 form (gemm_p3.h; results are multiplied
// by the operands' read scales), and the uint8 Atari frames are read as ONE exact f16 plane
// (integers 0..255, converted once per step by launch_frames_f16 or the replay's fused
// gather) with the 1/255 scale applied to the f32 result
// (acme/wrappers/atari_wrapper.py:284-306 scales the frame before the first convolution;
// the scale commutes with the sum up to f32 rounding of the result).
//
// Operand orientation per GEMM (why each mode):
//   forward  A = im2col(X) KCONTIG (8 channels of a pixel)   B = W [K][CO] RCONTIG
//   wgrad    A = im2col(X)^T RCONTIG                         B = dZ [pix][CO] RCONTIG
//   dgrad    A = dZ gather KCONTIG (8 out-channels)          B = W^T KCONTIG (CO contiguous)
//
// Loaders return byte offsets (gemm_p3.h kOOB = zeros).  The stage's first reduction
// index k0 is a multiple of BK (<= 32) and every filter-tap row (KW * channels) is a
// multiple of 32, so a stage never crosses a kernel row: kh (and for >= 32 channels kw)
// derive from the wave-uniform k0 alone and stay in scalar registers.
#pragma once

#include "conv.h"
#include "gemm_p3.h"

namespace acme {
namespace conv {

using gemm::CPlanes;
using gemm::kOOB;
using gemm::Planes;
using gemm::PlaneSrc;

__device__ __forceinline__ uint32_t boff(int64_t elem) { return (uint32_t)(2 * elem); }
// A operand offsets: f16 elements, or bytes when A is the uint8 frames (gemm_p3.h AU8).
template <bool U8>
__device__ __forceinline__ uint32_t aoff(int64_t elem) {
  return U8 ? (uint32_t)elem : (uint32_t)(2 * elem);
}

using V8 = float[8];

// The two planes of 8 scaled values (v[j] * w) as packed f16 pairs; returns max |v|.
__device__ __forceinline__ float split8(const V8& v, float w, uint32_t (&h)[4], uint32_t (&l)[4]) {
  float mx = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint16_t h0, l0, h1, l1;
    gemm::split2_bits(v[2 * j] * w, h0, l0);
    gemm::split2_bits(v[2 * j + 1] * w, h1, l1);
    h[j] = (uint32_t)h0 | ((uint32_t)h1 << 16);
    l[j] = (uint32_t)l0 | ((uint32_t)l1 << 16);
    mx = gemm::amax_max(mx, gemm::amax_max(fabsf(v[2 * j]), fabsf(v[2 * j + 1])));
  }
  return mx;
}
// Planes of 8 consecutive values at element e (16-B aligned): two 16-byte stores; returns
// max |v| (the tensor's amax).
__device__ __forceinline__ float put8(const Planes& y, int64_t e, const V8& v) {
  uint32_t h[4], l[4];
  const float mx = split8(v, y.w(), h, l);
  *reinterpret_cast<uint4*>(y.p + e) = uint4{h[0], h[1], h[2], h[3]};
  *reinterpret_cast<uint4*>(y.p + y.stride + e) = uint4{l[0], l[1], l[2], l[3]};
  return mx;
}
// 8 f32 values at p (32-B aligned).
__device__ __forceinline__ void st8(float* p, const V8& v) {
  *reinterpret_cast<float4*>(p) = float4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<float4*>(p + 4) = float4{v[4], v[5], v[6], v[7]};
}
// The same with non-temporal stores: weight-gradient results (the conv split-K slabs, the
// dense weight gradient), which only the end-of-step Adam reads.  They stream to memory
// during the kernel instead of sitting dirty in the L2 until its end-of-kernel writeback:
// step 0.4920 -> 0.4895 ms over six alternating 300-step pairs (Adam, which reads them
// later, 51.6 -> 56.7 us; the weight gradients 2-4 us each faster; round 6,
// profiles/r06/schedule/ab_nt_wgrad_slabs.log).
__device__ __forceinline__ void st8_nt(float* p, const V8& v) {
  using f4 = __attribute__((ext_vector_type(4))) float;
  __builtin_nontemporal_store(f4{v[0], v[1], v[2], v[3]}, reinterpret_cast<f4*>(p));
  __builtin_nontemporal_store(f4{v[4], v[5], v[6], v[7]}, reinterpret_cast<f4*>(p + 4));
}
// ReLU mask of 8 stored activations (their f16 h plane; x > 0 <=> h > 0): dz where x > 0.
__device__ __forceinline__ void relu_mask8(const CPlanes& x, int64_t e, V8& v) {
  const uint4 w = *reinterpret_cast<const uint4*>(x.p + e);
  const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint16_t a = (uint16_t)(ws[j] & 0xffff), b = (uint16_t)(ws[j] >> 16);
    if (!(a != 0 && (a & 0x8000) == 0)) v[2 * j] = 0.f;
    if (!(b != 0 && (b & 0x8000) == 0)) v[2 * j + 1] = 0.f;
  }
}

// ------------------------------------------------------------------ forward
// NPA = 1: frames (the f16 copy of the uint8 values, or with U8 the uint8 frames themselves,
// widened exactly as they are staged), result scaled by 1/255; NPA = 2: f32 planes.
template <class G, int NPA, bool U8 = false>
struct P3ConvFwd {
  static_assert(!U8 || NPA == 1, "uint8 frames are one plane");
  static constexpr bool A_U8 = U8;
  static_assert(G::CI % 8 == 0 || (G::CI == 4 && G::KW % 2 == 0 && G::S % 2 == 0 &&
                                   G::PL % 2 == 0),
                "8-k units need 8 channels, or 4-channel pixel pairs that never straddle "
                "the image border");
  static_assert((G::KW * G::CI) % 32 == 0, "a filter-tap row must hold whole 32-k stages");
  static_assert(G::CO % 8 == 0, "output channels must be a multiple of 8");
  static constexpr int A_MODE = gemm::KCONTIG, B_MODE = gemm::RCONTIG;
  static constexpr int A_PLANES = NPA, B_PLANES = gemm::kPlanes;
  static constexpr bool kAmax = true;
  int M, N, K, k_chunk;  // M = frames * OPIX, N = CO, K = KH*KW*CI
  PlaneSrc a_src;        // [frames][IH][IW][CI]
  PlaneSrc b_src;        // W [K][CO]
  const float* bias;
  Planes y;              // [frames][OH][OW][CO]
  // U8 image-resident fill (gemm_p3i.h): frames >= a_split come from a_src2 (numbered from
  // 0 there), e.g. o_tm1 and o_t of a batch in two buffers.
  PlaneSrc a_src2{};
  int a_split = 1 << 30;
  uint64_t* stamps = nullptr;  // timing experiment (gemm_p3i.h phase stamps, HasStamps)
  __device__ gemm::PScale* amax_sc() const { return y.sc; }
  struct ARow {
    int pix;  // element offset of (frame, ih0, iw0)
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
    a.ih0 = oh * G::S - G::PT;
    a.iw0 = ow * G::S - G::PL;
    a.pix = (b * G::IPIX + a.ih0 * G::IW + a.iw0) * G::CI;
    return a;
  }
  __device__ uint32_t a_off(const ARow& a, int k0, int kk) const {
    constexpr int T = G::KW * G::CI;
    const int kh = k0 / T;
    const int r = k0 - kh * T + kk;
    const int kw = r / G::CI, ci = r - kw * G::CI;
    const bool ok = a.ok && (unsigned)(a.ih0 + kh) < (unsigned)G::IH &&
                    (unsigned)(a.iw0 + kw) < (unsigned)G::IW;
    return ok ? aoff<U8>(a.pix + (kh * G::IW + kw) * G::CI + ci) : kOOB;
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ uint32_t b_off(const BRow& b, int k0, int kk) const {
    return b.n < N ? boff((int64_t)(k0 + kk) * G::CO + b.n) : kOOB;
  }
  static constexpr bool kStore8 = true;
  // relu(acc r (/ 255) + b): the activation of 8 outputs (r = the operands' read scales).
  __device__ void act8(int n, const V8& acc, V8& v) const {
    const float rs = gemm::result_scale(a_src, b_src);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float x = acc[j] * rs;
      if constexpr (NPA == 1) x = x / 255.0f;
      x += bias[n + j];
      v[j] = x > 0.f ? x : 0.f;
    }
  }
  __device__ float store8(int m, int n, const V8& acc, int) const {
    V8 v;
    act8(n, acc, v);
    return put8(y, (int64_t)m * G::CO + n, v);
  }
  // The epilogue's constants for columns n..n+7, loaded before the k loop (gemm_p3.h EpiPre).
  struct Pre {
    float b[8];
    float rs, w;
    uint32_t* flag;
  };
  __device__ Pre pre(int n) const {
    Pre q;
    const int nn = n < N ? n : 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) q.b[j] = bias[nn + j];
    q.rs = gemm::result_scale(a_src, b_src);
    q.w = y.sc->w;
    q.flag = y.sc->flag;
    return q;
  }
  __device__ float store8p(int m, int n, const V8& acc, int, const Pre& q) const {
    V8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float x = acc[j] * q.rs;
      if constexpr (NPA == 1) x = x / 255.0f;
      x += q.b[j];
      v[j] = x > 0.f ? x : 0.f;
    }
    uint32_t h[4], l[4];
    const float mx = split8(v, q.w, h, l);
    const int64_t e = (int64_t)m * G::CO + n;
    *reinterpret_cast<uint4*>(y.p + e) = uint4{h[0], h[1], h[2], h[3]};
    *reinterpret_cast<uint4*>(y.p + y.stride + e) = uint4{l[0], l[1], l[2], l[3]};
    return mx;
  }
};

// ------------------------------------------------------------------ weight grad
template <class G, int NPA, bool U8 = false>
struct P3ConvWgrad {
  static_assert(!U8 || NPA == 1, "uint8 frames are one plane");
  static constexpr bool A_U8 = U8;
  static_assert(G::CI % 8 == 0 || (G::CI == 4 && G::KW % 2 == 0 && G::S % 2 == 0 &&
                                   G::PL % 2 == 0),
                "see P3ConvFwd");
  static_assert(G::OPIX >= 32, "a 32-k stage must span at most two frames");
  static constexpr int A_MODE = gemm::RCONTIG, B_MODE = gemm::RCONTIG;
  static constexpr int A_PLANES = NPA, B_PLANES = gemm::kPlanes;
  static constexpr bool kColSum = true;  // bias gradient = column sums of dZ
  // One accumulator per tile (gemm_p3.h P3Acc): each split-K partial is a short reduction
  // (B x pixels / splits rows), and the split accumulators cost conv3_wgrad 27.9 -> 34.9 us
  // for gradients already below the f32 engine's error either way (round 6: conv2 / conv3
  // weight gradients 4.3e-7 / 3.5e-7 against 4.0e-7 / 3.3e-7 split and 6.9e-7 / 5.6e-7 f32,
  // profiles/r06/accuracy/).
  static constexpr bool kNoSplitAcc = true;
  int M, N, K, k_chunk;  // M = G::K rows (kh,kw,ci), N = CO, K = frames * OPIX
  PlaneSrc a_src;        // X [frames][IH][IW][CI]
  PlaneSrc b_src;        // dZ [frames * OPIX][CO]
  float* slab;           // [splits][M + 1][N]; row M holds the split's bias-gradient partial
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
  __device__ uint32_t a_off(const ARow& a, int k0, int kk) const {
    const int b0 = k0 / G::OPIX;  // scalar
    int r = k0 - b0 * G::OPIX + kk;
    const bool wrap = r >= G::OPIX;
    const int b = b0 + (wrap ? 1 : 0);
    r -= wrap ? G::OPIX : 0;
    const int oh = r / G::OW, ow = r - oh * G::OW;
    const int ih = oh * G::S + a.dh, iw = ow * G::S + a.dw;
    const bool ok = a.ok && (unsigned)ih < (unsigned)G::IH && (unsigned)iw < (unsigned)G::IW;
    return ok ? aoff<U8>(((b * G::IPIX + ih * G::IW + iw) * G::CI) + a.ci) : kOOB;
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ uint32_t b_off(const BRow& b, int k0, int kk) const {
    return b.n < N ? boff((int64_t)(k0 + kk) * G::CO + b.n) : kOOB;
  }
  static constexpr bool kStore8 = true;
  __device__ float store8(int i, int n, const V8& acc, int split) const {
    const float rs = gemm::result_scale(a_src, b_src);
    V8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = NPA == 1 ? (acc[j] * rs) / 255.0f : acc[j] * rs;
    st8_nt(slab + ((size_t)split * (M + 1) + i) * N + n, v);
    return 0.f;
  }
  __device__ void store_colsum(int n, float v, int split) const {
    slab[((size_t)split * (M + 1) + M) * N + n] = v * gemm::read_scale(b_src.sc);
  }
};

// ------------------------------------------------------------------ input grad
// Stride-1 input gradient (conv3): dX[p][ci] = sum_{kh,kw,co} dZ[p + PT - kh, ...][co] W.
template <class G>
struct P3ConvDgrad {
  static_assert(G::S == 1, "strided input gradients use P3ConvDgradSubZ");
  static_assert(G::CO % 32 == 0 && G::CI % 8 == 0, "channel counts");
  static constexpr int A_MODE = gemm::KCONTIG, B_MODE = gemm::KCONTIG;
  static constexpr int A_PLANES = gemm::kPlanes, B_PLANES = gemm::kPlanes;
  static constexpr bool kAmax = true;
  int M, N, K, k_chunk;  // M = frames * IPIX, N = CI, K = KH*KW*CO
  PlaneSrc a_src;        // dZ [frames][OH][OW][CO]
  PlaneSrc b_src;        // W [KH][KW][CI][CO]
  CPlanes xprev;         // [frames][IH][IW][CI] post-ReLU activations of the previous layer
  Planes dx;             // [frames][IH][IW][CI] = dZ of the previous layer
  __device__ gemm::PScale* amax_sc() const { return dx.sc; }
  struct ARow {
    int pix;  // element offset of (frame, th0, tw0) in dZ
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
    a.th0 = ih + G::PT;
    a.tw0 = iw + G::PL;
    a.pix = (b * G::OPIX + a.th0 * G::OW + a.tw0) * G::CO;
    return a;
  }
  __device__ uint32_t a_off(const ARow& a, int k0, int kk) const {
    constexpr int T = G::KW * G::CO;
    const int kh = k0 / T;
    const int r = k0 - kh * T + kk;
    const int kw = r / G::CO, co = r - kw * G::CO;
    const bool ok = a.ok && (unsigned)(a.th0 - kh) < (unsigned)G::OH &&
                    (unsigned)(a.tw0 - kw) < (unsigned)G::OW;
    return ok ? boff(a.pix - (kh * G::OW + kw) * G::CO + co) : kOOB;
  }
  __device__ BRow b_row(int ci) const { return BRow{ci}; }
  __device__ uint32_t b_off(const BRow& b, int k0, int kk) const {
    constexpr int T = G::KW * G::CO;
    const int kh = k0 / T;
    const int r = k0 - kh * T + kk;
    const int kw = r / G::CO, co = r - kw * G::CO;
    return b.ci < N ? boff(((kh * G::KW + kw) * G::CI + b.ci) * G::CO + co) : kOOB;
  }
  static constexpr bool kStore8 = true;
  __device__ float store8(int m, int ci, const V8& acc, int) const {
    const int64_t idx = (int64_t)m * G::CI + ci;
    const float rs = gemm::result_scale(a_src, b_src);
    V8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = acc[j] * rs;
    relu_mask8(xprev, idx, v);
    return put8(dx, idx, v);
  }
};

// Strided input gradient by sub-pixel decomposition, all S*S parity classes in one
// launch (blockIdx.z = class): conv.h ConvDgradSubZ with plane operands.
template <class G>
struct P3ConvDgradSubZ {
  static_assert(G::KH % G::S == 0 && G::KW % G::S == 0, "kernel must be a multiple of stride");
  static_assert(G::CO % 32 == 0 && G::CI % 8 == 0, "channel counts");
  static constexpr int A_MODE = gemm::KCONTIG, B_MODE = gemm::KCONTIG;
  static constexpr int A_PLANES = gemm::kPlanes, B_PLANES = gemm::kPlanes;
  static constexpr bool kZClass = true;
  static constexpr bool kAmax = true;
  static constexpr int S = G::S;
  static constexpr int JH = G::KH / S, JW = G::KW / S;
  static constexpr int KR = JH * JW * G::CO;
  int M, N, K, k_chunk;  // M = rows of the largest class (grid), N = CI, K = KR
  int batch;
  PlaneSrc a_src, b_src;  // dZ, W
  CPlanes xprev;
  Planes dx;
  int ph = 0, pw = 0, rh = 0, rw = 0, nh = 1, nw = 1, mc = 0;  // set by for_z
  __device__ gemm::PScale* amax_sc() const { return dx.sc; }
  __device__ P3ConvDgradSubZ for_z(int z) const {
    P3ConvDgradSubZ q = *this;
    q.ph = z / S;
    q.pw = z % S;
    q.rh = ((q.ph - G::PT) % S + S) % S;
    q.rw = ((q.pw - G::PL) % S + S) % S;
    q.nh = (G::IH - q.rh + S - 1) / S;
    q.nw = (G::IW - q.rw + S - 1) / S;
    q.mc = batch * q.nh * q.nw;
    return q;
  }
  static int max_rows(int batch) { return ConvDgradSubZ<G>::max_rows(batch); }
  struct ARow {
    int pix;  // element offset of (frame, oh0, ow0) in dZ
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
    a.oh0 = (ih + G::PT - ph) / S;
    a.ow0 = (iw + G::PL - pw) / S;
    a.pix = (b * G::OPIX + a.oh0 * G::OW + a.ow0) * G::CO;
    return a;
  }
  __device__ uint32_t a_off(const ARow& a, int k0, int kk) const {
    constexpr int T = JW * G::CO;
    const int jh = k0 / T;
    const int r = k0 - jh * T + kk;
    const int jw = r / G::CO, co = r - jw * G::CO;
    const bool ok = a.ok && (unsigned)(a.oh0 - jh) < (unsigned)G::OH &&
                    (unsigned)(a.ow0 - jw) < (unsigned)G::OW;
    return ok ? boff(a.pix - (jh * G::OW + jw) * G::CO + co) : kOOB;
  }
  __device__ BRow b_row(int ci) const { return BRow{ci}; }
  __device__ uint32_t b_off(const BRow& b, int k0, int kk) const {
    constexpr int T = JW * G::CO;
    const int jh = k0 / T;
    const int r = k0 - jh * T + kk;
    const int jw = r / G::CO, co = r - jw * G::CO;
    const int kh = ph + S * jh, kw = pw + S * jw;
    return b.ci < N ? boff(((kh * G::KW + kw) * G::CI + b.ci) * G::CO + co) : kOOB;
  }
  static constexpr bool kStore8 = true;
  __device__ float store8(int m, int ci, const V8& acc, int) const {
    if (m >= mc) return 0.f;
    int b, ih, iw;
    decode(m, b, ih, iw);
    const int64_t idx = ((int64_t)b * G::IPIX + ih * G::IW + iw) * G::CI + ci;
    const float rs = gemm::result_scale(a_src, b_src);
    V8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = acc[j] * rs;
    relu_mask8(xprev, idx, v);
    return put8(dx, idx, v);
  }
};

// ------------------------------------------------------------------ dense layers
// Y = X W (+ bias, act in the split-K reduction): X [rows][ldx] planes, W [K][N] planes.
struct P3DenseFwd {
  static constexpr int A_MODE = gemm::KCONTIG, B_MODE = gemm::RCONTIG;
  static constexpr int A_PLANES = gemm::kPlanes, B_PLANES = gemm::kPlanes;
  static constexpr bool kNoSplitAcc = true;  // gemm_p3.h P3Acc
  int M, N, K, k_chunk;
  PlaneSrc a_src;  // X
  int ldx;
  PlaneSrc b_src;  // W
  float* slab;     // [splits][M][N] partial sums (already read-scaled; finalised by the
                   // slab reduction)
  uint64_t* stamps = nullptr;  // timing experiment (gemm_p3.h HasStamps)
  struct ARow {
    int off;
    bool ok;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int m) const { return ARow{m * ldx, m < M}; }
  __device__ uint32_t a_off(const ARow& a, int k0, int kk) const {
    return a.ok ? boff(a.off + k0 + kk) : kOOB;
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ uint32_t b_off(const BRow& b, int k0, int kk) const {
    return b.n < N ? boff((int64_t)(k0 + kk) * N + b.n) : kOOB;
  }
  static constexpr bool kStore8 = true;
  __device__ float store8(int m, int n, const V8& acc, int split) const {
    const float rs = gemm::result_scale(a_src, b_src);
    V8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = acc[j] * rs;
    st8(slab + ((size_t)split * M + m) * N + n, v);
    return 0.f;
  }
};

// dW = X^T dZ (reduction over the batch), db = column sums of dZ.
struct P3DenseWgrad {
  static constexpr int A_MODE = gemm::RCONTIG, B_MODE = gemm::RCONTIG;
  static constexpr int A_PLANES = gemm::kPlanes, B_PLANES = gemm::kPlanes;
  static constexpr bool kNoSplitAcc = true;  // gemm_p3.h P3Acc
  static constexpr bool kColSum = true;
  int M, N, K, k_chunk;  // M = Kin, N = Nout, K = rows (batch)
  PlaneSrc a_src;        // X [rows][ldx]
  int ldx;
  PlaneSrc b_src;        // dZ [rows][N]
  float* out;
  float* bias_out;
  struct ARow {
    int i;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int i) const { return ARow{i}; }
  __device__ uint32_t a_off(const ARow& a, int k0, int kk) const {
    return a.i < M ? boff((int64_t)(k0 + kk) * ldx + a.i) : kOOB;
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ uint32_t b_off(const BRow& b, int k0, int kk) const {
    return b.n < N ? boff((int64_t)(k0 + kk) * N + b.n) : kOOB;
  }
  static constexpr bool kStore8 = true;
  __device__ float store8(int i, int n, const V8& acc, int) const {
    const float rs = gemm::result_scale(a_src, b_src);
    V8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = acc[j] * rs;
    st8_nt(out + (size_t)i * N + n, v);
    return 0.f;
  }
  __device__ void store_colsum(int n, float v, int) const {
    bias_out[n] = v * gemm::read_scale(b_src.sc);
  }
};

// dX = dZ W^T masked by the previous layer's ReLU: dZ [rows][K] planes, W [N][K] planes
// (the layer's [Kin][Nout] weight: Nout = K is contiguous).
struct P3DenseDgrad {
  static constexpr int A_MODE = gemm::KCONTIG, B_MODE = gemm::KCONTIG;
  static constexpr int A_PLANES = gemm::kPlanes, B_PLANES = gemm::kPlanes;
  static constexpr bool kAmax = true;
  int M, N, K, k_chunk;  // M = rows, N = Kin, K = Nout
  PlaneSrc a_src;        // dZ
  PlaneSrc b_src;        // W
  CPlanes xprev;         // [rows][ldx]
  int ldx;
  Planes dx;             // [rows][ldx]
  __device__ gemm::PScale* amax_sc() const { return dx.sc; }
  struct ARow {
    int off;
    bool ok;
  };
  struct BRow {
    int n;
  };
  __device__ ARow a_row(int m) const { return ARow{m * K, m < M}; }
  __device__ uint32_t a_off(const ARow& a, int k0, int kk) const {
    return a.ok ? boff(a.off + k0 + kk) : kOOB;
  }
  __device__ BRow b_row(int n) const { return BRow{n}; }
  __device__ uint32_t b_off(const BRow& b, int k0, int kk) const {
    return b.n < N ? boff((int64_t)b.n * K + k0 + kk) : kOOB;
  }
  static constexpr bool kStore8 = true;
  __device__ float store8(int m, int n, const V8& acc, int) const {
    const int64_t idx = (int64_t)m * ldx + n;
    const float rs = gemm::result_scale(a_src, b_src);
    V8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = acc[j] * rs;
    relu_mask8(xprev, idx, v);
    return put8(dx, idx, v);
  }
};

}  // namespace conv
}  // namespace acme
