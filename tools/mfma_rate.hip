// Issue rate of the f16 / bf16 MFMAs the plane engine uses: every SIMD of the chip runs one
// wave of N back-to-back MFMAs on 4 independent accumulators; prints the chip's rate and,
// from the shader clock (s_memtime), cycles per MFMA.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_rate.hip -o tools/mfma_rate && tools/mfma_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int KIND>
__global__ void __launch_bounds__(256) mfma_loop(int n, float* out, long long* cyc) {
  f16x8 a, b, a2, b2;
  bf16x8 c, d;
  for (int j = 0; j < 8; ++j) {
    a[j] = (_Float16)(threadIdx.x * 1e-3f + j);
    b[j] = (_Float16)(j * 1e-3f);
    a2[j] = (_Float16)(threadIdx.x * 2e-3f - j);
    b2[j] = (_Float16)(j * -1e-3f);
    c[j] = (__bf16)(threadIdx.x * 1e-3f + j);
    d[j] = (__bf16)(j * 1e-3f);
  }
  f32x16 acc[4];
  f32x4 acc4[4];
  for (int q = 0; q < 4; ++q)
    for (int v = 0; v < 16; ++v) acc[q][v] = 0.f;
  for (int q = 0; q < 4; ++q)
    for (int v = 0; v < 4; ++v) acc4[q][v] = 0.f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (KIND == 0) acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[q], 0, 0, 0);
      if constexpr (KIND == 1) acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c, d, acc[q], 0, 0, 0);
      if constexpr (KIND == 2) acc4[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc4[q], 0, 0, 0);
      if constexpr (KIND == 3) {  // the plane engine's pattern: 3 dependent terms per accumulator
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[q], 0, 0, 0);
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b2, acc[q], 0, 0, 0);
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a2, b, acc[q], 0, 0, 0);
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int q = 0; q < 4; ++q) s += KIND == 2 ? acc4[q][0] : acc[q][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int KIND>
void run(const char* name, double flops_per) {
  const int blocks = 256, threads = 256, n = 4096;  // 4 waves per CU: one per SIMD
  float* out;
  long long* cyc;
  (void)hipMalloc(&out, blocks * threads * sizeof(float));
  (void)hipMalloc(&cyc, sizeof(long long));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  mfma_loop<KIND><<<blocks, threads>>>(16, out, cyc);  // warm-up
  (void)hipEventRecord(e0);
  mfma_loop<KIND><<<blocks, threads>>>(n, out, cyc);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  long long c = 0;
  (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  const int per = KIND == 3 ? 12 : 4;  // MFMAs per loop iteration
  const double total = (double)blocks * 4 * n * per * flops_per;  // waves x MFMAs x flops
  printf("%-28s %8.3f ms  %7.1f TFLOP/s  %6.1f memtime-ticks per MFMA (one wave)\n", name, ms,
         total / (ms * 1e-3) / 1e12, (double)c / ((double)per * n));
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  run<0>("v_mfma_f32_32x32x16_f16", 2.0 * 32 * 32 * 16);
  run<1>("v_mfma_f32_32x32x16_bf16", 2.0 * 32 * 32 * 16);
  run<2>("v_mfma_f32_16x16x32_f16", 2.0 * 16 * 16 * 32);
  run<3>("32x32x16_f16 3-term chains", 2.0 * 32 * 32 * 16);
  return 0;
}
