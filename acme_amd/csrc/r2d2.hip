// R2D2 prioritized sequence replay helpers: the two pieces of
// R2D2Learner._step (acme/agents/tf/r2d2/learning.py) that connect the learner to the
// prioritized sequence table, as device kernels so the write-back path never leaves HBM.
//
//   compute_priority (learning.py:230-236): p_b = eta * max_t |e[t][b]| +
//       (1 - eta) * mean_t |e[t][b]|, float32 (eta and 1 - eta rounded from double) (tf.reduce_max / tf.reduce_mean over axis 0;
//       the mean sums t = 0..T-1 in order, then divides by T), cast to float64 for
//       update_priorities (learning.py:196-199).
//   importance weights (learning.py:178-183): w = (1 / (N * P))^beta / max(w) in float64
//       (N = max_replay_size, P = the sampled item's probability), cast to float32.  Reverb
//       streams a sequence as T timesteps that all carry their item's probability, so the
//       reference's [T, B] weights are this [B] vector broadcast over time.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "common.h"
#include "profiler.h"

using namespace acme;

namespace {

__global__ void r2d2_priority_kernel(const float* __restrict__ err, int T, int B, float eta,
                                     float one_minus_eta, double* __restrict__ out) {
#pragma clang fp contract(off)
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float mx = 0.f, sum = 0.f;
  for (int t = 0; t < T; ++t) {
    const float a = fabsf(err[(int64_t)t * B + b]);
    mx = fmaxf(mx, a);
    sum = sum + a;
  }
  const float mean = sum / (float)T;
  out[b] = (double)(eta * mx + one_minus_eta * mean);
}

// One workgroup: w_b = (1 / (N p_b))^beta, then / max_b w_b (f64), stored as f32.
__global__ void __launch_bounds__(1024) r2d2_is_weights_kernel(const double* __restrict__ prob,
                                                               int B, double n, double beta,
                                                               float* __restrict__ out) {
  __shared__ double red[1024];
  double mx = 0.0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) mx = fmax(mx, pow(1.0 / (n * prob[b]), beta));
  red[threadIdx.x] = mx;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  const double m = red[0];
  for (int b = threadIdx.x; b < B; b += blockDim.x)
    out[b] = (float)(pow(1.0 / (n * prob[b]), beta) / m);
}

}  // namespace

extern "C" {

int acme_r2d2_priorities(const float* errors, int32_t T, int32_t B, double eta, double* out,
                         void* stream) {
  ACME_CHECK_ARG(errors && out, "null argument");
  ACME_CHECK_ARG(T >= 1 && B >= 1, "errors must be [T >= 1, B >= 1]");
  hipStream_t st = as_stream(stream);
  ACME_PROF("r2d2_priorities", st, 0.0, 4.0 * T * B + 8.0 * B);
  // alpha and 1 - alpha are Python floats in the reference, each cast to f32 by TF.
  r2d2_priority_kernel<<<(unsigned)ceil_div(B, 256), 256, 0, st>>>(
      errors, T, B, (float)eta, (float)(1.0 - eta), out);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int acme_r2d2_importance_weights(const double* probabilities, int32_t B,
                                 int64_t max_replay_size, double beta, float* out,
                                 void* stream) {
  ACME_CHECK_ARG(probabilities && out, "null argument");
  ACME_CHECK_ARG(B >= 1 && max_replay_size >= 1, "bad batch / replay size");
  hipStream_t st = as_stream(stream);
  r2d2_is_weights_kernel<<<1, 1024, 0, st>>>(probabilities, B, (double)max_replay_size, beta,
                                              out);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

}  // extern "C"
