// Shared helpers for the acme_amd HIP library (gfx950 / CDNA4 only).
//
// Error model of the C-ABI (include/acme_hip.h): every entry point returns
// ACME_OK (0) or a negative acme_status and records a human-readable message
// in a thread-local buffer readable through acme_last_error().  The Python
// shims map the status to ValueError / RuntimeError, mirroring how the
// reference surfaces failures as Python exceptions.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "../../include/acme_hip.h"

namespace acme {

void set_error(const char* fmt, ...);

// Tile / schedule variant for tuning runs: ACME_V_<KEY>=<n> in the environment (read once
// per key); 0 is the shipped default.
int tune_variant(const char* key);
void tune_set(const char* key, int value);
// Incremented by every tune_set: cached launch plans (captured graphs) keyed on it.
int tune_generation();

// An event that orders work between streams of this device (no timing, device-scope
// fence: the host may test it for completion but must not read device-written memory on
// its strength), instead of a system-scope one.  DQN step 0.5299 -> 0.5270 ms (three
// alternating runs each, one box: within noise).  An event record or wait still costs its
// stream 5-9 us (the step's kernel trace); doorbell kernels in their place (a one-wave
// signal kernel, a one-wave spinning wait kernel) measured 2.5 us per step slower.
hipError_t make_order_event(hipEvent_t* ev);

#define ACME_HIP_TRY(expr)                                                   \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess) {                                                  \
      ::acme::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                        __FILE__, __LINE__);                                 \
      return ACME_ERR_HIP;                                                   \
    }                                                                        \
  } while (0)

#define ACME_CHECK_ARG(cond, ...)                                            \
  do {                                                                       \
    if (!(cond)) {                                                           \
      ::acme::set_error(__VA_ARGS__);                                        \
      return ACME_ERR_INVALID;                                               \
    }                                                                        \
  } while (0)

#define ACME_LAUNCH_CHECK()                                                  \
  do {                                                                       \
    hipError_t _e = hipGetLastError();                                       \
    if (_e != hipSuccess) {                                                  \
      ::acme::set_error("kernel launch failed: %s (%s:%d)",                  \
                        hipGetErrorString(_e), __FILE__, __LINE__);          \
      return ACME_ERR_HIP;                                                   \
    }                                                                        \
  } while (0)

static inline hipStream_t as_stream(void* s) {
  return reinterpret_cast<hipStream_t>(s);
}

static inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

constexpr int kWave = 64;  // CDNA wavefront width; never 32.

}  // namespace acme
