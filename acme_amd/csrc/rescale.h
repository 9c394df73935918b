// The plane scale records' rescale (gemm_p3.h PScale) as one workgroup's work, so that it can
// run as its own launch (launch_plane_rescale) or as an extra workgroup of a launch already on
// the stream (the DQN step's priority write-back: one kernel boundary fewer on the critical
// path).  Records [0, nt) are transient (written and read within a step: the next step writes
// and reads at the new scale), [nt, n) persistent (parameter planes, rewritten by every Adam
// pass at w and read in the next step: r becomes the wi their writer used, and w moves when
// an amax was taken).  copy_to >= 0 (outside [0, n)): record copy_to took a plane copy of
// record copy_from's latest write (r = its wi).  Records in [skip_lo, skip_hi) are left alone
// (rescaled on the stream that writes them).  A transient record whose amax is 0 keeps its
// scale.  A record whose maximum is not finite (planes computed from overflowed planes) takes
// the largest scale reduction of the group's overflowed records with a finite maximum (its
// inputs shrink by that factor at their new scale), else 2^-16.  overflow |= 1 when a write
// exceeded f16's range (amax w >= 65520) or was not finite.
//
// defer_r: the transient records' read scale r is NOT moved (w, wi and rl are): consumers
// still running on another stream read the planes stored now at r; the step's Adam launch
// then commits r = wi (adam_commit_read_scales) once every consumer has finished.
#pragma once

#include <hip/hip_runtime.h>

#include "gemm_p3.h"
#include "kernels.h"

namespace acme {

// Timing experiment (replay.hip prio_update_fused_kernel phase stamps, 8 per workgroup):
// non-null while a DQN learner created with ACME_V_STAMPS=1 lives.
extern uint64_t* g_update_stamps;

struct RescaleJob {
  gemm::PScale* s = nullptr;  // null: no job
  int nt = 0, n = 0, copy_from = -1, copy_to = -1;
  int* overflow = nullptr;
  int skip_lo = -1, skip_hi = -1;
  int defer_r = 0;
  RescaleGuard rg{};
};

// The power of two w that puts a (> 0, finite) at 2^7 <= a w < 2^8 (gemm_p3.h); exponent
// clamped so w and 1 / w stay normal f32.
__device__ __forceinline__ int rescale_exp(float a) {
  int k;
  (void)frexpf(a, &k);  // a = m 2^k, m in [0.5, 1)
  const int e = 8 - k;
  return e < -100 ? -100 : (e > 100 ? 100 : e);
}

// One workgroup of blockDim.x = 64 W threads (W >= 1) does the whole job; every thread of
// the workgroup calls.  All loads are issued before the first store.
__device__ __forceinline__ void rescale_block(const RescaleJob& j) {
  constexpr int kMax = 16;
  __shared__ uint32_t s_a[kMax];  // each record's maximum (f32 bits)
  __shared__ int s_shift[kMax];
  __shared__ int s_bad;
  gemm::PScale* s = j.s;
  const int n = j.n;
  const int nw = blockDim.x >> 6, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool last = threadIdx.x == blockDim.x - 1;
  const RescaleGuard& rg = j.rg;
  // Every load in one round, before any LDS store (the records are reached through generic
  // pointers, which the compiler must order against LDS stores): each wave's records' slots,
  // thread i's record i, and the guard's inputs in the last thread.  The slots were written
  // by atomics from every XCD, so each round trip goes past the local L2; one record per
  // wave round (four rounds at 15 records) made this workgroup 6 us long and the priority
  // write-back waited on its verdict (profiles/r06/replay/update_stamps.log).
  constexpr int kPerWave = kMax;  // >= records per wave at any wave count
  uint32_t av[kPerWave];
#pragma unroll
  for (int k = 0; k < kPerWave; ++k) {
    const int i = wv + k * nw;
    av[k] = i < n ? s[i].slot[lane].v : 0u;
  }
  const int ti = threadIdx.x;
  float w0 = 0.f, r0 = 0.f, wi0 = 0.f;
  if (ti < n) {
    w0 = s[ti].w;
    r0 = s[ti].r;
    wi0 = s[ti].wi;
  }
  uint32_t gv[6] = {0u, 0u, 0u, 0u, 0u, 0u};
  int64_t cnt[2] = {0, 0};
  float dpv = 0.f, cwi = 0.f;
  if (last) {
    cwi = j.copy_to >= 0 ? s[j.copy_from].wi : 0.f;
    if (rg.g) {
      gv[0] = rg.g->on;
      gv[1] = rg.g->tt;
      gv[2] = rg.g->t[rg.gate.par & 1];
      gv[3] = rg.g->prm;
      gv[4] = rg.g->hold;
      gv[5] = rg.tmo ? rg.tmo[0] : 0u;
      cnt[0] = rg.g->applied;
      cnt[1] = rg.g->skipped;
      if (rg.gate.dp) dpv = *rg.gate.dp;
    }
  }
  // Phase 1: every record's slot maximum (a wave per record, records strided over waves).
#pragma unroll
  for (int k = 0; k < kPerWave; ++k) {
    const int i = wv + k * nw;
    if (i >= n) break;
    uint32_t a = av[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a = max(a, (uint32_t)__shfl_xor((int)a, o, 64));
    if (lane == 0) s_a[i] = a;
  }
  if (threadIdx.x == 0) s_bad = 0;
  __syncthreads();
  // Phase 2: per record, the overflow shift and the bad flag.
  if (threadIdx.x < n) {
    const int i = threadIdx.x;
    const float a = __builtin_bit_cast(float, s_a[i]);
    const bool live = !(i >= j.skip_lo && i < j.skip_hi);
    const bool finite = a <= 3.0e38f;
    int wexp;
    (void)frexpf(w0, &wexp);  // w0 = 2^(wexp - 1)
    const float aw = a * w0;
    s_shift[i] = live && finite && a > 0.f && !(aw < 65520.f) ? rescale_exp(a) - (wexp - 1) : 0;
    // Overflowed (max w >= 65520, or not finite) or underflowed (0 < max w < 1: the
    // largest element's low plane is subnormal, so the planes carry less than an f32
    // rounding's precision relative to the tensor's maximum).
    if (live && a != 0.f && (!(aw < 65520.f) || aw < 1.f)) atomicOr(&s_bad, 1);
  }
  __syncthreads();
  // Phase 3: stores.  Slots cleared by the record's wave; the record by thread i; the copy
  // and the guard by the last thread.
#pragma unroll
  for (int k = 0; k < kMax; ++k) {
    const int i = wv + k * nw;
    if (i >= n) break;
    if (!(i >= j.skip_lo && i < j.skip_hi)) s[i].slot[lane].v = 0u;
  }
  if (threadIdx.x < n && !(threadIdx.x >= j.skip_lo && threadIdx.x < j.skip_hi)) {
    const int i = threadIdx.x;
    const float a = __builtin_bit_cast(float, s_a[i]);
    const bool persistent = i >= j.nt;
    const float stored = persistent ? wi0 : r0;  // the read scale of the planes stored now
    gemm::PScale* rec = s + i;
    if (a == 0.f) {  // no maximum taken: the scale stays
      if (persistent) rec->r = rec->rl = stored;
      else rec->rl = stored;
    } else {
      if (!(a * w0 < 65520.f) && j.overflow) atomicOr(j.overflow, 1);
      const bool finite = a <= 3.0e38f;
      int shift = -16;  // not finite: the largest reduction of the group, else 2^-16
      if (!finite) {
        int mn = 0;
        for (int k = 0; k < n && k < kMax; ++k) mn = min(mn, s_shift[k]);
        if (mn < 0) shift = mn;
      }
      const int e = finite ? rescale_exp(a) : 0;
      const float w = finite ? ldexpf(1.f, e) : ldexpf(w0, shift);
      const float wi = finite ? ldexpf(1.f, -e) : ldexpf(wi0, -shift);
      rec->w = w;
      rec->wi = wi;
      rec->rl = stored;
      if (persistent) rec->r = stored;
      else if (!j.defer_r) rec->r = wi;
    }
  }
  if (last) {
    if (j.copy_to >= 0) {
      s[j.copy_to].r = cwi;
      s[j.copy_to].rl = cwi;
    }
    StepGuard* g = rg.g;
    const uint32_t bad = s_bad ? 1u : 0u;
    if (g && rg.mode == kRgTarget) {
      g->t[rg.gate.par & 1] = gv[1] | bad;
      g->tt = 0u;
    } else if (g && rg.mode == kRgQValues) {
      g->qv = gv[1] | bad;
      g->tt = 0u;
    } else if (g && rg.mode == kRgFlag) {
      if (bad) g->on = 1u;
    } else if (g && rg.mode == kRgStep) {
      // The flags (on, prm) are cleared by the step's Adam launch, after every reader.
      const bool timed_out = rg.tmo && gv[5] != 0u;
      const bool skip =
          (gv[0] | gv[2] | gv[4] | bad) != 0u || dpv > 0.f || timed_out;
      // The verdict first (the same launch's update workgroups wait for it), then the
      // counts from the values read up front: no load between the decision and the store.
      const uint32_t v = (rg.seq << 1) | (skip ? 1u : 0u);
      __hip_atomic_store(&g->vseq, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (rg.host_verdicts)
        __hip_atomic_store(rg.host_verdicts + (rg.seq & 63u), v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      if (timed_out) {
        rg.tmo[0] = 0u;
        rg.tmo[1] += 1u;
      }
      g->last = skip ? 1u : 0u;
      if (skip) {
        const int64_t k = cnt[1] + 1;
        g->skipped = k;
        if (rg.host_skipped) *rg.host_skipped = k;
        if (rg.sticky) g->hold = 1u;
      } else {
        g->applied = cnt[0] + 1;
      }
    } else if (g && rg.mode == kRgClear) {
      g->hold = 0u;
      g->on = g->tt = g->prm = g->last = g->qv = 0u;
      g->t[0] = g->t[1] = 0u;
    }
  }
}

}  // namespace acme
