// Error state + version entry points of libacme_hip.so.
#include "common.h"

#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

namespace acme {

static thread_local char g_last_error[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

namespace {
std::mutex g_tune_mu;
std::vector<std::pair<std::string, int>> g_tune;  // key -> value (env, or acme_tune_set)
int g_tune_gen = 0;
}  // namespace

int tune_generation() {
  std::lock_guard<std::mutex> lock(g_tune_mu);
  return g_tune_gen;
}

int tune_variant(const char* key) {
  std::lock_guard<std::mutex> lock(g_tune_mu);
  for (auto& kv : g_tune)
    if (kv.first == key) return kv.second;
  const char* v = getenv((std::string("ACME_V_") + key).c_str());
  const int x = v ? atoi(v) : 0;
  g_tune.emplace_back(key, x);
  return x;
}

void tune_set(const char* key, int value) {
  std::lock_guard<std::mutex> lock(g_tune_mu);
  ++g_tune_gen;
  for (auto& kv : g_tune)
    if (kv.first == key) {
      kv.second = value;
      return;
    }
  g_tune.emplace_back(key, value);
}

namespace gemm {

// Matmul engine: 1 = three-plane bf16 MFMA (gemm_x6.h, f32-equivalent), 0 = f32 MFMA
// (gemm.h).  Initialised from ACME_MATMUL ("f32" or "x6"), default x6.
static int g_engine = -1;

bool use_x6() {
  if (g_engine < 0) {
    const char* e = getenv("ACME_MATMUL");
    g_engine = (e && strcmp(e, "f32") == 0) ? ACME_MATMUL_F32 : ACME_MATMUL_X6;
  }
  return g_engine == ACME_MATMUL_X6;
}

}  // namespace gemm

hipError_t make_order_event(hipEvent_t* ev) {
  // Device-scope release: no system-scope cache writeback / invalidation when the event
  // is recorded or waited on (nothing on the host reads device memory on their strength).
  return hipEventCreateWithFlags(ev, hipEventDisableTiming | hipEventDisableSystemFence);
}

}  // namespace acme

extern "C" {

int acme_set_matmul_engine(int32_t engine) {
  ACME_CHECK_ARG(engine == ACME_MATMUL_F32 || engine == ACME_MATMUL_X6, "unknown matmul engine %d",
                 engine);
  acme::gemm::g_engine = engine;
  return ACME_OK;
}

int32_t acme_matmul_engine(void) { return acme::gemm::use_x6() ? ACME_MATMUL_X6 : ACME_MATMUL_F32; }

const char* acme_last_error(void) { return acme::g_last_error; }

int acme_tune_set(const char* key, int32_t value) {
  ACME_CHECK_ARG(key, "null key");
  acme::tune_set(key, value);
  return ACME_OK;
}

const char* acme_version(void) { return "acme_amd 0.1.0 (" __DATE__ " " __TIME__ ")"; }

const char* acme_target_arch(void) { return "gfx950"; }

int acme_event_create(void** ev) {
  ACME_CHECK_ARG(ev, "null argument");
  hipEvent_t e = nullptr;
  ACME_HIP_TRY(acme::make_order_event(&e));
  *ev = e;
  return ACME_OK;
}

int acme_event_destroy(void* ev) {
  if (ev) ACME_HIP_TRY(hipEventDestroy(static_cast<hipEvent_t>(ev)));
  return ACME_OK;
}

int acme_event_record(void* ev, void* stream) {
  ACME_CHECK_ARG(ev, "null event");
  ACME_HIP_TRY(hipEventRecord(static_cast<hipEvent_t>(ev), acme::as_stream(stream)));
  return ACME_OK;
}

int acme_stream_wait_event(void* stream, void* ev) {
  ACME_CHECK_ARG(ev, "null event");
  ACME_HIP_TRY(hipStreamWaitEvent(acme::as_stream(stream), static_cast<hipEvent_t>(ev), 0));
  return ACME_OK;
}

int acme_event_query(void* ev) {
  ACME_CHECK_ARG(ev, "null event");
  const hipError_t e = hipEventQuery(static_cast<hipEvent_t>(ev));
  if (e == hipSuccess) return 1;
  if (e == hipErrorNotReady) return 0;
  ACME_HIP_TRY(e);
  return ACME_ERR_HIP;
}

int acme_event_synchronize(void* ev) {
  ACME_CHECK_ARG(ev, "null event");
  ACME_HIP_TRY(hipEventSynchronize(static_cast<hipEvent_t>(ev)));
  return ACME_OK;
}

}  // extern "C"
