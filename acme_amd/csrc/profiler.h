// Per-section kernel timing with HIP events recorded on the stream the kernels are
// launched on (bench.py's live roofline numbers; cross-checked against rocprofv3).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace acme {
namespace prof {

bool enabled();
// Opens a section: records a start event on `st`.  Returns a token (or -1 if disabled).
// `peak`: the TFLOP/s ceiling of the arithmetic path the section runs on (its MFMA engine;
// 0 = not a GEMM section), reported with the section for the roofline.
int begin(const char* name, hipStream_t st, double flops, double bytes, double peak = 0);
void end(int token, hipStream_t st);

struct Scope {
  int tok;
  hipStream_t st;
  Scope(const char* name, hipStream_t s, double flops = 0, double bytes = 0, double peak = 0)
      : tok(enabled() ? begin(name, s, flops, bytes, peak) : -1), st(s) {}
  ~Scope() {
    if (tok >= 0) end(tok, st);
  }
};

}  // namespace prof
}  // namespace acme

#define ACME_PROF(name, st, flops, bytes) ::acme::prof::Scope _acme_prof_scope_(name, st, flops, bytes)
#define ACME_PROF_PEAK(name, st, flops, bytes, peak) \
  ::acme::prof::Scope _acme_prof_scope_(name, st, flops, bytes, peak)

// Dense MFMA peaks (MI355X_MICROARCH.md): f32 v_mfma_f32_32x32x2_f32 and bf16 (dense).
constexpr double kPeakF32MfmaTflops = 157.3;
constexpr double kPeakBf16MfmaTflops = 2500.0;
