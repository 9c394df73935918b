// AtariTorso forward / backward launches (see torso.h).  Tile shapes come from the
// round-1 A/B sweep on MI355X (profiles/r01): 128x32 (4 waves 4x1) for conv1's 32 output
// channels, 128x64 (2x2) for conv2/conv3 forward, split-K weight gradients reduced by one
// deterministic slab pass, and the stride-2 conv2 input gradient as four sub-pixel GEMMs.
#include "torso.h"

#include <algorithm>

#include "common.h"
#include "conv_p3.h"
#include "gemm.h"
#include "gemm_p3.h"
#include "gemm_p3i.h"
#include "gemm_p3s.h"
#include "gemm_p3c12.h"
#include "gemm_x6.h"
#include "kernels.h"
#include "profiler.h"

namespace acme {
namespace torso {

using namespace acme::conv;
using acme::gemm::launch_gemm;

namespace {

constexpr int kConv1WgradSplits = 256, kConv2WgradSplits = 64, kConv3WgradSplits = 64;

inline int chunk_for(int K, int splits) {
  int c = (int)ceil_div(K, splits);
  return (int)ceil_div(c, 32) * 32;
}

#define TORSO_GEMM(name, BM, BN, WM, WN, prob, splits)                                        \
  TORSO_GEMM_F(name, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, BM, BN, WM, \
               WN, prob, splits)
#define TORSO_GEMM_F(name, flops, BM, BN, WM, WN, prob, splits)                               \
  do {                                                                                        \
    ACME_PROF_PEAK(name, st, flops, 0.0, (gemm::matmul_peak_tflops<1, decltype(prob)>()));      \
    hipError_t _e = gemm::launch_matmul<BM, BN, WM, WN, 16>(prob, splits, st);                 \
    if (_e != hipSuccess) {                                                                   \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                    \
    }                                                                                         \
  } while (0)

// Conv weight + bias gradient: split-K over the batch pixels into [splits][K+1][CO] slabs
// (row K = bias partial from the GEMM's colsum hook), then one deterministic reduction
// writes dW and db.
template <class G, class In, int BM, int BN, int WM, int WN>
int conv_wgrad(const typename In::T* x, const float* dz, int rows, int splits, float* slab,
               float* dw, float* db, const char* name, const char* rname, hipStream_t st) {
  ConvWgrad<G, In> p;
  p.M = G::K; p.N = G::CO; p.K = rows * G::OPIX; p.k_chunk = chunk_for(p.K, splits);
  p.x = x; p.dz = dz; p.slab = slab;
  TORSO_GEMM(name, BM, BN, WM, WN, p, splits);
  const int64_t count = (int64_t)(p.M + 1) * p.N;
  ACME_PROF(rname, st, 0.0, 4.0 * (double)(splits + 1) * (double)count);
  return launch_slab_reduce(slab, splits, count, dw, (int64_t)p.M * p.N, db, nullptr, 0, 0, st);
}

}  // namespace

int64_t wgrad_slab_floats() {
  return std::max<int64_t>({(int64_t)kConv1WgradSplits * (G1::K + 1) * G1::CO,
                            (int64_t)kConv2WgradSplits * (G2::K + 1) * G2::CO,
                            (int64_t)kConv3WgradSplits * (G3::K + 1) * G3::CO});
}

int forward(const Weights& w, bool u8, const void* obs_a, const void* obs_b, int split, int rows,
            const Acts& a, hipStream_t st) {
  if (u8) {
    ConvFwd<G1, InU8> p;
    p.M = rows * G1::OPIX; p.N = G1::CO; p.K = G1::K; p.k_chunk = G1::K;
    p.x = static_cast<const uint8_t*>(obs_a); p.x2 = static_cast<const uint8_t*>(obs_b);
    p.split_b = split; p.w = w.w1; p.bias = w.b1; p.y = a.x1;
    TORSO_GEMM("conv1_fwd", 128, 32, 4, 1, p, 1);
  } else {
    ConvFwd<G1, InF32> p;
    p.M = rows * G1::OPIX; p.N = G1::CO; p.K = G1::K; p.k_chunk = G1::K;
    p.x = static_cast<const float*>(obs_a); p.x2 = static_cast<const float*>(obs_b);
    p.split_b = split; p.w = w.w1; p.bias = w.b1; p.y = a.x1;
    TORSO_GEMM("conv1_fwd", 128, 32, 4, 1, p, 1);
  }
  {
    ConvFwd<G2, InF32> p;
    p.M = rows * G2::OPIX; p.N = G2::CO; p.K = G2::K; p.k_chunk = G2::K;
    p.x = a.x1; p.x2 = a.x1; p.split_b = rows; p.w = w.w2; p.bias = w.b2; p.y = a.x2;
    TORSO_GEMM("conv2_fwd", 128, 64, 2, 2, p, 1);
  }
  {
    ConvFwd<G3, InF32> p;
    p.M = rows * G3::OPIX; p.N = G3::CO; p.K = G3::K; p.k_chunk = G3::K;
    p.x = a.x2; p.x2 = a.x2; p.split_b = rows; p.w = w.w3; p.bias = w.b3; p.y = a.x3;
    TORSO_GEMM("conv3_fwd", 128, 64, 2, 2, p, 1);
  }
  return ACME_OK;
}

int backward(const Weights& w, const Grads& g, bool u8, const void* obs, int rows, const Acts& a,
             const float* dz3, float* dz2, float* dz1, float* slab, hipStream_t st) {
  int rc;
  // conv3
  if ((rc = conv_wgrad<G3, InF32, 64, 64, 2, 2>(a.x2, dz3, rows, kConv3WgradSplits, slab, g.w3,
                                                g.b3, "conv3_wgrad", "conv3_wgrad_reduce", st)))
    return rc;
  {
    ConvDgrad<G3> p;
    p.M = rows * G3::IPIX; p.N = G3::CI; p.K = G3::KH * G3::KW * G3::CO; p.k_chunk = p.K;
    p.dz = dz3; p.w = w.w3; p.xprev = a.x2; p.dx = dz2;
    TORSO_GEMM("conv3_dgrad", 128, 64, 2, 2, p, 1);
  }
  // conv2
  if ((rc = conv_wgrad<G2, InF32, 64, 64, 2, 2>(a.x1, dz2, rows, kConv2WgradSplits, slab, g.w2,
                                                g.b2, "conv2_wgrad", "conv2_wgrad_reduce", st)))
    return rc;
  {  // Stride-2 input gradient: the four sub-pixel parity classes as one launch (z = class).
    ConvDgradSubZ<G2> p;
    p.M = ConvDgradSubZ<G2>::max_rows(rows); p.N = G2::CI; p.K = ConvDgradSubZ<G2>::KR;
    p.k_chunk = p.K; p.batch = rows;
    p.dz = dz2; p.w = w.w2; p.xprev = a.x1; p.dx = dz1;
    // Useful FLOPs: every input pixel once, K = KR per class.
    TORSO_GEMM_F("conv2_dgrad", 2.0 * rows * G2::IPIX * G2::CI * (double)p.K, 256, 32, 4, 1, p,
                 G2::S * G2::S);
  }
  // conv1 (no input gradient needed)
  if (u8)
    return conv_wgrad<G1, InU8, 128, 32, 4, 1>(static_cast<const uint8_t*>(obs), dz1, rows,
                                               kConv1WgradSplits, slab, g.w1, g.b1,
                                               "conv1_wgrad", "conv1_wgrad_reduce", st);
  return conv_wgrad<G1, InF32, 128, 32, 4, 1>(static_cast<const float*>(obs), dz1, rows,
                                              kConv1WgradSplits, slab, g.w1, g.b1, "conv1_wgrad",
                                              "conv1_wgrad_reduce", st);
}

// ---------------------------------------------------------------- plane path
namespace {

// Weight-gradient K splits; kP3MaxWgradSplits sizes the slab.
constexpr int kP3Conv1WgradSplits = 512, kP3Conv2WgradSplits = 128, kP3Conv3WgradSplits = 128;
constexpr int kP3MaxWgradSplits = 512;

#define P3_GEMM_F(name, flops, BM, BN, WM, WN, BK, prob, splits)                             \
  do {                                                                                        \
    ACME_PROF_PEAK(name, st, flops, 0.0, gemm::p3_peak_tflops<decltype(prob)>());             \
    hipError_t _e = gemm::launch_gemm_p3<BM, BN, WM, WN, BK>(prob, splits, st);               \
    if (_e != hipSuccess) {                                                                   \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                    \
    }                                                                                         \
  } while (0)
// Warp-specialised form (gemm_p3ws_kernel, fragment reads one k16 step ahead; BK = 32).
#define P3WS_GEMM(name, BM, BN, WM, WN, prob, splits)                                        \
  do {                                                                                        \
    ACME_PROF_PEAK(name, st, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, 0.0, \
                   gemm::p3_peak_tflops<decltype(prob)>());                                   \
    hipError_t _e = gemm::launch_gemm_p3ws<BM, BN, WM, WN, 32, true>(prob, splits, st);      \
    if (_e != hipSuccess) {                                                                   \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                    \
    }                                                                                         \
  } while (0)
#define P3_GEMM(name, BM, BN, WM, WN, BK, prob, splits)                                      \
  P3_GEMM_F(name, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, BM, BN, WM, \
            WN, BK, prob, splits)
// Image-resident convolution (gemm_p3i.h): FPB frames per block, WM x WN waves of 32*MT
// rows; `frames` images.
using I1F = gemm::ImgGeomPairs<G1>;
using I2F = gemm::ImgGeom<G2, false>;
using I3F = gemm::ImgGeom<G3, false>;
using I3D = gemm::ImgGeom<G3, true>;
#define P3I_GEMM(name, GI, FPB, BN, WM, WN, MT, prob, frames)                                 \
  do {                                                                                        \
    ACME_PROF_PEAK(name, st, 2.0 * (double)(prob).M * (double)(prob).N * (double)(prob).K, 0.0, \
                   gemm::p3_peak_tflops<decltype(prob)>());                                   \
    hipError_t _e = gemm::launch_gemm_p3i<GI, FPB, BN, WM, WN, MT>(prob, frames, st);         \
    if (_e != hipSuccess) {                                                                   \
      set_error("gemm launch failed: %s (%s:%d)", hipGetErrorString(_e), __FILE__, __LINE__); \
      return ACME_ERR_HIP;                                                                    \
    }                                                                                         \
  } while (0)

inline CPlanes cp(const Plane& x) { return CPlanes{x.p, x.stride, x.sc}; }
inline Planes pl(const Plane& x) { return Planes{x.p, x.stride, x.sc}; }
// Operand source over the first `elems` elements of each plane.
inline PlaneSrc src(const Plane& x, int64_t elems) {
  return PlaneSrc{x.p, x.stride, (int32_t)(2 * elems), x.sc};
}
inline PlaneSrc frames_src(const Frames& f, int rows) {
  return PlaneSrc{static_cast<const uint16_t*>(f.p), 0,
                  (int32_t)((f.u8 ? 1 : 2) * (int64_t)rows * G1::IPIX * G1::CI)};
}

// conv1 forward (image-resident) over `rows` frames into y, f16 or uint8 frames.
template <bool U8>
int conv1_fwd_p3(const PWeights& w, const Frames& frames, int rows, const Planes& y,
                 hipStream_t st, uint64_t* stamps = nullptr) {
  P3ConvFwd<G1, 1, U8> p;
  p.stamps = stamps;
  p.M = rows * G1::OPIX; p.N = G1::CO; p.K = G1::K; p.k_chunk = G1::K;
  const int n1 = U8 ? std::min(rows, frames.split) : rows;
  p.a_src = frames_src(frames, n1); p.b_src = src(w.w1, G1::K * G1::CO);
  if (U8 && n1 < rows) {
    p.a_src2 = frames_src(frames.rows_from(n1), rows - n1);
    p.a_split = n1;
  }
  p.bias = w.b1; p.y = y;
  // Image-resident frames (gemm_p3i.h pixel pairs): 39.6 -> 33.7 us vs the best im2col
  // tiling.
  P3I_GEMM("conv1_fwd", I1F, 1, 32, 7, 1, 2, p, rows);
  return ACME_OK;
}

// The fused conv1 -> conv2 forward (gemm_p3c12.h) over frames [nsep, rows).
template <bool U8>
int conv12_fwd_p3(const PWeights& w, const Frames& frames, int rows, int nsep, const PActs& a,
                  hipStream_t st) {
  const int nf = rows - nsep;
  const Frames fr = frames.rows_from(nsep);
  if (U8 && fr.split < nf)
    return (set_error("the fused conv1 -> conv2 forward reads its frames from one buffer"),
            ACME_ERR_INVALID);
  P3ConvFwd<G1, 1, U8> p1;
  p1.M = nf * G1::OPIX; p1.N = G1::CO; p1.K = G1::K; p1.k_chunk = G1::K;
  p1.a_src = frames_src(fr, nf); p1.b_src = src(w.w1, G1::K * G1::CO);
  p1.bias = w.b1;
  p1.y = Planes{a.x1.p + (int64_t)nsep * kX1, a.x1.stride, a.x1.sc};
  P3ConvFwd<G2, gemm::kPlanes> p2;
  p2.M = nf * G2::OPIX; p2.N = G2::CO; p2.K = G2::K; p2.k_chunk = G2::K;
  p2.a_src = src(a.x1, (int64_t)rows * kX1); p2.b_src = src(w.w2, G2::K * G2::CO);
  p2.bias = w.b2;
  p2.y = Planes{a.x2.p + (int64_t)nsep * kFlat, a.x2.stride, a.x2.sc};
  const double fl = 2.0 * p1.M * p1.N * (double)p1.K + 2.0 * p2.M * p2.N * (double)p2.K;
  ACME_PROF_PEAK("conv12_fwd", st, fl, 0.0, gemm::p3_peak_tflops<decltype(p2)>());
  hipError_t e = gemm::launch_gemm_p3c12(p1, p2, nf, 0, st);
  if (e != hipSuccess) return (set_error("gemm launch failed: %s", hipGetErrorString(e)), ACME_ERR_HIP);
  return ACME_OK;
}

// conv1's weight + bias gradient (split-K slabs) from the frames of rows [0, rows).
template <bool U8>
int conv1_wgrad_p3(const Frames& frames, int rows, const Plane& dz1, float* slab, int splits,
                   bool single_role, P3ConvWgrad<G1, 1, U8>& p, hipStream_t st) {
  if (U8 && frames.split < rows)
    return (set_error("conv1's weight gradient reads its frames from one buffer"),
            ACME_ERR_INVALID);
  P3ConvWgrad<G1, 1, U8> q;
  q.M = G1::K; q.N = G1::CO; q.K = rows * G1::OPIX;
  q.k_chunk = chunk_for(q.K, splits);
  q.a_src = frames_src(frames, rows); q.b_src = src(dz1, (int64_t)rows * kX1);
  q.slab = slab;
  // Producer / consumer waves (gemm_p3ws_kernel): 28.5 -> 25.0 us, the same bits.
  if (single_role) P3_GEMM("conv1_wgrad", 256, 32, 4, 1, 32, q, splits);
  else P3WS_GEMM("conv1_wgrad", 256, 32, 4, 1, q, splits);
  p = q;
  return ACME_OK;
}

template <class P>
int p3_wgrad_reduce(const P& p, int splits, float* slab, float* dw, float* db, const char* rname,
                    hipStream_t st) {
  const int64_t count = (int64_t)(p.M + 1) * p.N;
  ACME_PROF(rname, st, 0.0, 4.0 * (double)(splits + 1) * (double)count);
  return launch_slab_reduce(slab, splits, count, dw, (int64_t)p.M * p.N, db, nullptr, 0, 0, st);
}

}  // namespace

uint64_t* g_stamps_conv[3] = {nullptr, nullptr, nullptr};

int64_t wgrad_slab_floats_p3() {
  return std::max<int64_t>({(int64_t)kP3MaxWgradSplits * (G1::K + 1) * G1::CO,
                            (int64_t)kP3MaxWgradSplits * (G2::K + 1) * G2::CO,
                            (int64_t)kP3MaxWgradSplits * (G3::K + 1) * G3::CO});
}

int forward_p3(const PWeights& w, const Frames& frames, int rows, const PActs& a,
               hipStream_t st, int keep_x1) {
  // Frames [0, nsep) run conv1 then conv2 with x1 in HBM (the backward reads it); frames
  // [nsep, rows) the fused conv1 -> conv2 kernel (gemm_p3c12.h), whose x1 stays in LDS.
  // The target forward (keep_x1 == 0, on the side stream) is fused throughout: 0.716 ->
  // 0.713 ms per step when it was introduced.  The online forward runs unfused: fusing its
  // o_t rows (x1 kept for the o_tm1 rows only) measured 0.545 -> 0.603 ms per step with
  // the f16 planes (the fused kernel's one block per CU beside the other stream).
  const int nsep = keep_x1 == 0 ? 0 : rows;
  int rc;
  if (nsep < rows &&
      (rc = frames.u8 ? conv12_fwd_p3<true>(w, frames, rows, nsep, a, st)
                      : conv12_fwd_p3<false>(w, frames, rows, nsep, a, st)) != ACME_OK)
    return rc;
  if (nsep > 0 && (rc = frames.u8 ? conv1_fwd_p3<true>(w, frames, nsep, pl(a.x1), st, g_stamps_conv[0])
                                  : conv1_fwd_p3<false>(w, frames, nsep, pl(a.x1), st, g_stamps_conv[0])) != ACME_OK)
    return rc;
  if (nsep > 0) {
    P3ConvFwd<G2, gemm::kPlanes> p;
    p.M = nsep * G2::OPIX; p.N = G2::CO; p.K = G2::K; p.k_chunk = G2::K;
    p.a_src = src(a.x1, (int64_t)nsep * kX1); p.b_src = src(w.w2, G2::K * G2::CO);
    p.bias = w.b2; p.y = pl(a.x2);
    p.stamps = g_stamps_conv[1];
    // Image-resident x1 (gemm_p3i.h; two frames, 8 x 2 waves per block): with two f16
    // planes a frame's x1 image is 56 KB, so two frames and the weight ring fit one CU.
    // Step 0.573 -> 0.551 ms against the producer / consumer im2col kernel (two alternating
    // runs each, one box; one frame per block: 0.571).
    P3I_GEMM("conv2_fwd", I2F, 2, 64, 8, 2, 1, p, nsep);
  }
  {
    P3ConvFwd<G3, gemm::kPlanes> p;
    p.M = rows * G3::OPIX; p.N = G3::CO; p.K = G3::K; p.k_chunk = G3::K;
    p.a_src = src(a.x2, (int64_t)rows * kFlat); p.b_src = src(w.w3, G3::K * G3::CO);
    p.bias = w.b3; p.y = pl(a.x3);
    if (keep_x1 != 0) p.stamps = g_stamps_conv[2];  // the online forward's
    // Image-resident, 4 x 2 waves (measured 50.1 -> 43.5 us vs the 128x64 im2col engine;
    // two frames per block measured slower on the step, 0.550 -> 0.568-0.618 ms).
    P3I_GEMM("conv3_fwd", I3F, 1, 64, 4, 2, 1, p, rows);
  }
  return ACME_OK;
}

int backward_p3(const PWeights& w, const Grads& g, const Frames& frames, int rows,
                const PActs& a, const Plane& dz3, const Plane& dz2, const Plane& dz1, float* slab,
                hipStream_t st_main, const Side& sd) {
  int rc;
  // Weight gradients of conv3 and conv2 go to the side stream (when given): each only
  // waits for its layer's dZ, and runs beside the next input gradient on the main stream
  // (two forks; one fork after conv3_dgrad for both saved an event record but measured
  // 0.754 -> 0.767 ms per step: the lost overlap costs more).
  const bool fork = sd.side != nullptr;
  const bool defer = sd.defer != nullptr;
  if (defer && !(sd.slab && sd.slab2))
    return (set_error("deferred weight gradients need two side slabs"), ACME_ERR_INVALID);
  hipStream_t st = fork ? sd.side : st_main;
  float* wslab = fork || defer ? sd.slab : slab;
  {  // conv3 weight + bias gradient
    if (fork) {
      ACME_HIP_TRY(hipEventRecord(sd.e[0], st_main));
      ACME_HIP_TRY(hipStreamWaitEvent(sd.side, sd.e[0], 0));
    }
    P3ConvWgrad<G3, gemm::kPlanes> p;
    p.M = G3::K; p.N = G3::CO; p.K = rows * G3::OPIX;
    const int splits = kP3Conv3WgradSplits;
    p.k_chunk = chunk_for(p.K, splits);
    p.a_src = src(a.x2, (int64_t)rows * kFlat); p.b_src = src(dz3, (int64_t)rows * kFlat);
    p.slab = wslab;
    P3_GEMM("conv3_wgrad", 128, 64, 2, 2, 32, p, splits);
    if (defer) sd.defer[2] = WgradSlab{wslab, splits, (int64_t)p.M * p.N, p.N};
    else if ((rc = p3_wgrad_reduce(p, splits, wslab, g.w3, g.b3, "conv3_wgrad_reduce", st)))
      return rc;
  }
  st = st_main;
  {
    P3ConvDgrad<G3> p;
    p.M = rows * G3::IPIX; p.N = G3::CI; p.K = G3::KH * G3::KW * G3::CO; p.k_chunk = p.K;
    p.a_src = src(dz3, (int64_t)rows * kFlat); p.b_src = src(w.w3, G3::K * G3::CO);
    p.xprev = cp(a.x2); p.dx = pl(dz2);
    // Image-resident dZ, two frames x 8 x 2 waves: 37.4 us (128x64 im2col) -> 31.2 us.
    P3I_GEMM("conv3_dgrad", I3D, 2, 64, 8, 2, 1, p, rows);
  }
  if (fork) {
    ACME_HIP_TRY(hipEventRecord(sd.e[1], st_main));
    ACME_HIP_TRY(hipStreamWaitEvent(sd.side, sd.e[1], 0));
    st = sd.side;
  }
  {  // conv2
    P3ConvWgrad<G2, gemm::kPlanes> p;
    p.M = G2::K; p.N = G2::CO; p.K = rows * G2::OPIX;
    const int splits = kP3Conv2WgradSplits;
    p.k_chunk = chunk_for(p.K, splits);
    p.a_src = src(a.x1, (int64_t)rows * kX1); p.b_src = src(dz2, (int64_t)rows * kFlat);
    float* slab2 = defer ? sd.slab2 : wslab;
    p.slab = slab2;
    P3_GEMM("conv2_wgrad", 128, 64, 2, 2, 32, p, splits);
    if (defer) sd.defer[1] = WgradSlab{slab2, splits, (int64_t)p.M * p.N, p.N};
    else if ((rc = p3_wgrad_reduce(p, splits, slab2, g.w2, g.b2, "conv2_wgrad_reduce", st)))
      return rc;
    if (fork) ACME_HIP_TRY(hipEventRecord(sd.e[2], sd.side));
  }
  st = st_main;
  {  // stride-2 input gradient, four sub-pixel classes in one launch
    P3ConvDgradSubZ<G2> p;
    p.M = P3ConvDgradSubZ<G2>::max_rows(rows); p.N = G2::CI; p.K = P3ConvDgradSubZ<G2>::KR;
    p.k_chunk = p.K; p.batch = rows;
    p.a_src = src(dz2, (int64_t)rows * kFlat); p.b_src = src(w.w2, G2::K * G2::CO);
    p.xprev = cp(a.x1); p.dx = pl(dz1);
    // Image-resident dZ, two frames x four classes per block (16 waves, gemm_p3s.h):
    // 57.7 us (128x32 im2col) -> 38.0 (one frame per block) -> 34.7 us.
    const double fl = 2.0 * rows * G2::IPIX * G2::CI * (double)p.K;
    ACME_PROF_PEAK("conv2_dgrad", st, fl, 0.0, gemm::p3_peak_tflops<decltype(p)>());
    hipError_t e = gemm::launch_gemm_p3s<G2, 2>(p, rows, st);
    if (e != hipSuccess) return (set_error("gemm launch failed: %s", hipGetErrorString(e)), ACME_ERR_HIP);
  }
  {  // conv1 (no input gradient)
    const int splits = kP3Conv1WgradSplits;
    int64_t wcount;
    int M1, N1;
    if (frames.u8) {
      P3ConvWgrad<G1, 1, true> p;
      if ((rc = conv1_wgrad_p3<true>(frames, rows, dz1, slab, splits, sd.conv1_single, p, st)))
        return rc;
      M1 = p.M, N1 = p.N;
      if (!defer && (rc = p3_wgrad_reduce(p, splits, slab, g.w1, g.b1, "conv1_wgrad_reduce", st)))
        return rc;
    } else {
      P3ConvWgrad<G1, 1> p;
      if ((rc = conv1_wgrad_p3<false>(frames, rows, dz1, slab, splits, sd.conv1_single, p, st)))
        return rc;
      M1 = p.M, N1 = p.N;
      if (!defer && (rc = p3_wgrad_reduce(p, splits, slab, g.w1, g.b1, "conv1_wgrad_reduce", st)))
        return rc;
    }
    wcount = (int64_t)M1 * N1;
    if (defer) sd.defer[0] = WgradSlab{slab, splits, wcount, N1};
  }
  if (sd.tail && (rc = sd.tail(sd.tail_ctx, st_main)) != ACME_OK) return rc;
  if (fork) ACME_HIP_TRY(hipStreamWaitEvent(st_main, sd.e[2], 0));  // join
  return ACME_OK;
}

}  // namespace torso
}  // namespace acme
