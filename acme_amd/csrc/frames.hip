// Frame-deduplicated Atari observations.
//
// The reference stores every transition's two stacked observations whole
// (adders/reverb/transition.py:147-152: o_t and o_{t+n}, each [84, 84, 4] uint8 built by
// wrappers/frame_stacking.py:78-83 as np.stack(last 4 frames, axis=-1)), 56,448 bytes per
// transition.  Consecutive stacks share 3 of their 4 frames and the n-step o_{t+n} is a
// later stack of the same episode, so a frame table (replay/__init__.py FrameTable) keeps
// each distinct frame once in an HBM ring [num_frames][H*W] and every transition as 2 x S
// frame indices.  This kernel rebuilds the stacked observations of a sampled batch:
//   out[b][p * S + s] = frames[idx[b][s]][p]        (HWC, stack on the last axis)
// For S = 4 one thread takes 4 pixels: a 4-byte load from each of the 4 frames, a byte
// transpose (v_perm_b32), one 16-byte store.  Reads 4 * H*W and writes S * H*W bytes per
// observation: the same HBM bytes as gathering the stored stack.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"
#include "profiler.h"

using namespace acme;

namespace {

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}

// S = 4: grid (ceil(px / 4 / 256), batch); px % 4 == 0.
__global__ void __launch_bounds__(256) expand4_kernel(const uint8_t* __restrict__ frames,
                                                       int64_t num_frames, int64_t px,
                                                       const int32_t* __restrict__ idx,
                                                       uint8_t* __restrict__ out) {
  const int64_t b = blockIdx.y;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // pixel quad
  if (q * 4 >= px) return;
  uint32_t w[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    int64_t f = idx[b * 4 + s];
    f = f < 0 ? 0 : (f >= num_frames ? num_frames - 1 : f);  // host-validated; clamp anyway
    w[s] = *reinterpret_cast<const uint32_t*>(frames + f * px + q * 4);
  }
  // Pixel j of the quad -> bytes (w0.j, w1.j, w2.j, w3.j).
  const uint32_t a01lo = perm(w[1], w[0], 0x05010400u);  // w0.0 w1.0 w0.1 w1.1
  const uint32_t a23lo = perm(w[3], w[2], 0x05010400u);
  const uint32_t a01hi = perm(w[1], w[0], 0x07030602u);  // w0.2 w1.2 w0.3 w1.3
  const uint32_t a23hi = perm(w[3], w[2], 0x07030602u);
  uint4 v;
  v.x = perm(a23lo, a01lo, 0x05040100u);  // pixel 0: w0.0 w1.0 w2.0 w3.0
  v.y = perm(a23lo, a01lo, 0x07060302u);  // pixel 1
  v.z = perm(a23hi, a01hi, 0x05040100u);  // pixel 2
  v.w = perm(a23hi, a01hi, 0x07060302u);  // pixel 3
  *reinterpret_cast<uint4*>(out + b * px * 4 + q * 16) = v;
}

// Any S: one thread per output byte.
__global__ void expand_generic_kernel(const uint8_t* __restrict__ frames, int64_t num_frames,
                                      int64_t px, int stack, const int32_t* __restrict__ idx,
                                      uint8_t* __restrict__ out) {
  const int64_t b = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= px * stack) return;
  const int64_t p = e / stack, s = e - p * stack;
  int64_t f = idx[b * stack + s];
  f = f < 0 ? 0 : (f >= num_frames ? num_frames - 1 : f);
  out[b * px * stack + e] = frames[f * px + p];
}

}  // namespace

extern "C" {

int acme_frames_expand(const uint8_t* frames, int64_t num_frames, int64_t frame_bytes,
                       int32_t stack, const int32_t* idx, int64_t batch, uint8_t* out,
                       void* stream) {
  ACME_CHECK_ARG(frames && idx && out, "null argument");
  ACME_CHECK_ARG(num_frames >= 1 && frame_bytes >= 1 && stack >= 1 && batch >= 1 &&
                     batch <= 65535,
                 "bad frame expansion shape");
  hipStream_t st = as_stream(stream);
  ACME_PROF("frames_expand", st, 0.0, 2.0 * (double)batch * stack * frame_bytes);
  if (stack == 4 && frame_bytes % 4 == 0 && (reinterpret_cast<uintptr_t>(frames) & 3) == 0 &&
      (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
    const int64_t quads = frame_bytes / 4;
    expand4_kernel<<<dim3((unsigned)ceil_div(quads, 256), (unsigned)batch), 256, 0, st>>>(
        frames, num_frames, frame_bytes, idx, out);
  } else {
    expand_generic_kernel<<<dim3((unsigned)ceil_div(frame_bytes * stack, 256), (unsigned)batch),
                            256, 0, st>>>(frames, num_frames, frame_bytes, stack, idx, out);
  }
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

}  // extern "C"
