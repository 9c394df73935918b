// Section profiler (see profiler.h) + its C ABI (acme_profile_*).
#include "profiler.h"

#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"

namespace acme {
namespace prof {
namespace {

struct Rec {
  int section;
  hipEvent_t a, b;
  double flops, bytes;
  bool closed;
};

struct Section {
  std::string name;
  double ms = 0, flops = 0, bytes = 0, peak = 0;
  int64_t count = 0;
};

std::mutex g_mu;
bool g_enabled = false;
std::vector<Rec> g_open;
std::vector<hipEvent_t> g_pool;
std::vector<Section> g_sections;
std::map<std::string, int> g_index;

hipEvent_t get_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  (void)hipEventCreate(&e);
  return e;
}

// Resolve all recorded pairs into the per-section totals (synchronises on the events).
void drain() {
  for (Rec& r : g_open) {
    float ms = 0.f;
    if (r.closed && hipEventSynchronize(r.b) == hipSuccess &&
        hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
      Section& s = g_sections[r.section];
      s.ms += ms;
      s.flops += r.flops;
      s.bytes += r.bytes;
      s.count += 1;
    }
    g_pool.push_back(r.a);
    g_pool.push_back(r.b);
  }
  g_open.clear();
}

}  // namespace

bool enabled() { return g_enabled; }

int begin(const char* name, hipStream_t st, double flops, double bytes, double peak) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_index.find(name);
  int sec;
  if (it == g_index.end()) {
    sec = (int)g_sections.size();
    g_sections.push_back(Section{name});
    g_index[name] = sec;
  } else {
    sec = it->second;
  }
  if (peak > 0) g_sections[sec].peak = peak;
  if (g_open.size() > 100000 && g_open.back().closed) drain();  // bound the backlog
  Rec r{sec, get_event(), get_event(), flops, bytes, false};
  (void)hipEventRecord(r.a, st);
  g_open.push_back(r);
  return (int)g_open.size() - 1;
}

void end(int token, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (token < 0 || token >= (int)g_open.size()) return;
  (void)hipEventRecord(g_open[token].b, st);
  g_open[token].closed = true;
}

}  // namespace prof
}  // namespace acme

extern "C" {

int acme_profile_enable(int32_t on) {
  std::lock_guard<std::mutex> lk(acme::prof::g_mu);
  acme::prof::g_enabled = on != 0;
  return ACME_OK;
}

int acme_profile_reset(void) {
  std::lock_guard<std::mutex> lk(acme::prof::g_mu);
  acme::prof::drain();
  for (auto& s : acme::prof::g_sections) s.ms = s.flops = s.bytes = 0, s.count = 0;
  return ACME_OK;
}

int32_t acme_profile_num_sections(void) {
  std::lock_guard<std::mutex> lk(acme::prof::g_mu);
  acme::prof::drain();
  return (int32_t)acme::prof::g_sections.size();
}

int acme_profile_query(int32_t i, const char** name, double* total_ms, int64_t* count,
                       double* flops, double* bytes) {
  std::lock_guard<std::mutex> lk(acme::prof::g_mu);
  acme::prof::drain();
  ACME_CHECK_ARG(i >= 0 && i < (int32_t)acme::prof::g_sections.size(), "section out of range");
  const auto& s = acme::prof::g_sections[i];
  if (name) *name = s.name.c_str();
  if (total_ms) *total_ms = s.ms;
  if (count) *count = s.count;
  if (flops) *flops = s.flops;
  if (bytes) *bytes = s.bytes;
  return ACME_OK;
}

int acme_profile_query_peak(int32_t i, double* peak_tflops) {
  std::lock_guard<std::mutex> lk(acme::prof::g_mu);
  ACME_CHECK_ARG(i >= 0 && i < (int32_t)acme::prof::g_sections.size(), "section out of range");
  if (peak_tflops) *peak_tflops = acme::prof::g_sections[i].peak;
  return ACME_OK;
}

}  // extern "C"
