// Per-section kernel timing with HIP events recorded on the stream the kernels are
// launched on (bench.py's live roofline numbers; cross-checked against rocprofv3).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace acme {
namespace prof {

bool enabled();
// Opens a section: records a start event on `st`.  Returns a token (or -1 if disabled).
int begin(const char* name, hipStream_t st, double flops, double bytes);
void end(int token, hipStream_t st);

struct Scope {
  int tok;
  hipStream_t st;
  Scope(const char* name, hipStream_t s, double flops = 0, double bytes = 0)
      : tok(enabled() ? begin(name, s, flops, bytes) : -1), st(s) {}
  ~Scope() {
    if (tok >= 0) end(tok, st);
  }
};

}  // namespace prof
}  // namespace acme

#define ACME_PROF(name, st, flops, bytes) ::acme::prof::Scope _acme_prof_scope_(name, st, flops, bytes)
