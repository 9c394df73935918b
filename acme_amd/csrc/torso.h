// AtariTorso (acme/tf/networks/atari.py:36-50: Conv2D(32, 8, 4) -> ReLU -> Conv2D(64, 4, 2)
// -> ReLU -> Conv2D(64, 3, 1) -> ReLU -> Flatten, Sonnet SAME padding, NHWC) as implicit-GEMM
// MFMA launches, shared by the DQN learner (DQNAtariNetwork) and the IMPALA learner
// (IMPALAAtariNetwork's OAR embedding torso).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "conv.h"

namespace acme {
namespace gemm {
struct PScale;  // gemm_p3.h
}
namespace torso {

using G1 = conv::Geom<84, 84, 4, 21, 21, 32, 8, 8, 4, 2, 2>;
using G2 = conv::Geom<21, 21, 32, 11, 11, 64, 4, 4, 2, 1, 1>;
using G3 = conv::Geom<11, 11, 64, 11, 11, 64, 3, 3, 1, 1, 1>;
constexpr int kFlat = 11 * 11 * 64;  // 7744 features per frame
constexpr int kObsBytes = 84 * 84 * 4;
constexpr int kX1 = G1::OPIX * G1::CO;  // conv1 output floats per frame (14112)

struct Weights {
  const float *w1, *b1, *w2, *b2, *w3, *b3;
};
struct Grads {
  float *w1, *b1, *w2, *b2, *w3, *b3;
};
// Post-ReLU activations, [rows][...] NHWC: x1 [rows][kX1], x2 / x3 [rows][kFlat].
struct Acts {
  float *x1, *x2, *x3;
};

// Floats of split-K workspace the weight-gradient launches need.
int64_t wgrad_slab_floats();

// Forward over `rows` frames; frames [0, split) come from obs_a, the rest from obs_b
// (uint8 scaled by 1/255 inside conv1 when u8, else float32).
int forward(const Weights& w, bool u8, const void* obs_a, const void* obs_b, int split, int rows,
            const Acts& a, hipStream_t st);

// Backward over `rows` frames from dz3 = dLoss/d(conv3 pre-activation) [rows][kFlat]
// (already masked by conv3's ReLU).  dz2 [rows][kFlat] and dz1 [rows][kX1] are scratch;
// slab holds at least wgrad_slab_floats() floats.  No input gradient for the frames.
int backward(const Weights& w, const Grads& g, bool u8, const void* obs, int rows, const Acts& a,
             const float* dz3, float* dz2, float* dz1, float* slab, hipStream_t st);

// ---- Plane path (gemm_p3.h engine, uint8 frames): activations, gradients and weights
// as scaled two-plane f16 tensors (Plane::p[i * stride + e] = plane i of element e; sc =
// the tensor's scale record).
struct Plane {
  uint16_t* p;
  int64_t stride;
  gemm::PScale* sc;
};
struct PWeights {
  Plane w1, w2, w3;  // views into the flat parameter planes
  const float *b1, *b2, *b3;
};
// Timing experiment (ACME_V_STAMPS=1, tools/gemm_stamps.py): when set, the online
// forward's conv1 / conv2 / conv3 launches stamp their workgroups' phases here
// ([workgroups][8] u64 each, gemm_p3i.h).
extern uint64_t* g_stamps_conv[3];

struct PActs {
  Plane x1, x2, x3;
};
int64_t wgrad_slab_floats_p3();
// conv1's input, rows of 84*84*4: the f16 copy of the uint8 frames (launch_frames_f16), or
// with u8 the uint8 frames themselves (widened exactly where conv1's kernels stage them),
// rows [0, split) at p and the rest at p2 (a batch's o_tm1 and o_t in two buffers).
struct Frames {
  const void* p;
  bool u8 = false;
  const void* p2 = nullptr;
  int split = 1 << 30;
  Frames rows_from(int r) const {
    if (!u8) return Frames{static_cast<const uint8_t*>(p) + (size_t)r * kObsBytes * 2};
    if (r >= split)
      return Frames{static_cast<const uint8_t*>(p2) + (size_t)(r - split) * kObsBytes, true};
    return Frames{static_cast<const uint8_t*>(p) + (size_t)r * kObsBytes, true, p2, split - r};
  }
};
// frames: f16 copies of the uint8 frames [rows][84*84*4] (launch_frames_f16), or u8 frames.
// keep_x1: frames [0, keep_x1) get their conv1 output x1 in HBM (the backward reads it);
// -1: all.  With the fused conv1 -> conv2 kernel (gemm_p3c12.h, used when
// keep_x1 == 0) x1 only lives in LDS.
int forward_p3(const PWeights& w, const Frames& frames, int rows, const PActs& a,
               hipStream_t st, int keep_x1 = -1);
// Optional second stream for the weight gradients: conv3 / conv2 weight gradients run on
// `side` (with their own split-K slab) beside the input gradients on the main stream;
// events e[0..2] are scratch (hipEventDisableTiming).  side == nullptr: one stream.
// A weight gradient left as its split-K slab: `splits` rows of (wcount + bcount) floats,
// the weights' then the bias's partial sums (launch_slab_reduce's input).
struct WgradSlab {
  const float* slab = nullptr;
  int splits = 0;
  int64_t wcount = 0, bcount = 0;
};
struct Side {
  hipStream_t side = nullptr;
  float* slab = nullptr;
  hipEvent_t e[3] = {nullptr, nullptr, nullptr};
  // defer (optional, [3] = conv1, conv2, conv3): the weight gradients are not reduced but
  // described here for the consumer (the fused step's Adam, launch_adam_slabs).  conv3 and
  // conv2 then use `slab` and `slab2` (both needed, with or without the side stream).
  float* slab2 = nullptr;
  WgradSlab* defer = nullptr;
  // Optional work for the main stream after its last kernel, before the join (the DQN
  // step's priority write-back, which balances the two streams' backward).
  int (*tail)(void* ctx, hipStream_t st) = nullptr;
  void* tail_ctx = nullptr;
  // conv1's weight gradient on the single-role kernel instead of the producer / consumer one
  // (the same bits; tests, ACME_V_WSN=1 at the learner's creation).
  bool single_role = false;
  bool conv1_single = false;  // conv1's weight gradient on the single-role kernel (the DQN step)
};
// dz3: conv3's dZ planes [rows][kFlat] (masked); dz2 / dz1 plane scratch.
int backward_p3(const PWeights& w, const Grads& g, const Frames& frames, int rows,
                const PActs& a, const Plane& dz3, const Plane& dz2, const Plane& dz1, float* slab,
                hipStream_t st, const Side& side = Side());

}  // namespace torso
}  // namespace acme
