// Cost of stream-order markers on MI355X: back-to-back small kernels on one stream with
// (0) nothing between them, (1) hipEventRecord after each, (2) the event attached to each
// kernel's dispatch (hipExtLaunchKernelGGL stop event); (3) a dependency check: a second
// stream waits on the attached event and must see the first stream's write.  Kernel gaps
// come from a rocprofv3 kernel trace (tools/event_cost.py-style analysis by marker kernel).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

__global__ void tick(int* x, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) x[0] = v;
}
__global__ void spin(long long cycles) {
  long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
}
__global__ void check(const int* x, int v, int* bad) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && x[0] != v) bad[0] += 1;
}

int main() {
  int *x, *bad;
  hipMalloc(&x, 64);
  hipMalloc(&bad, 64);
  hipMemset(bad, 0, 64);
  hipStream_t s, s2;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  for (int timing = 0; timing < 2; ++timing) {
    hipEvent_t ev[4];
    for (auto& e : ev) hipEventCreateWithFlags(&e, timing ? 0 : hipEventDisableTiming);
    for (int mode = 0; mode < 4; ++mode) {
      hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 400000000LL);
      for (int i = 0; i < 400; ++i) {
        if (mode == 2) {
          hipExtLaunchKernelGGL(tick, dim3(1), dim3(64), 0, s, nullptr, ev[i % 4], 0, x, i);
        } else if (mode == 3) {
          hipExtLaunchKernelGGL(tick, dim3(1), dim3(64), 0, s, nullptr, ev[i % 4], 0, x, i);
          hipStreamWaitEvent(s2, ev[i % 4], 0);
          hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, s2, (const int*)x, i, bad);
          // s must not overwrite x before s2's check: s waits on s2's progress via a
          // second attached event every iteration.
          hipExtLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s2, nullptr, ev[(i + 2) % 4], 0, 0LL);
          hipStreamWaitEvent(s, ev[(i + 2) % 4], 0);
        } else {
          hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, s, x, i);
          if (mode == 1) hipEventRecord(ev[i % 4], s);
        }
      }
      hipDeviceSynchronize();
    }
  }
  int hb = -1;
  hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  printf("dependency violations: %d (%s)\n", hb, hipGetErrorString(hipGetLastError()));
  return 0;
}
