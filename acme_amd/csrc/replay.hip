// GPU-resident replay table: the MI355X replacement for the Reverb table the agents
// build (acme/agents/tf/dqn/agent.py:95-102, acme/agents/tf/d4pg/agent.py:96-102).
//
// Layout in HBM (one hipMalloc per array, struct-of-arrays):
//   field[f]     [capacity, field_bytes[f]]   item payloads (u8 Atari frames, f32 ...)
//   keys         [capacity] u64               key of the item in each ring slot
//   raw_prio     [capacity] f64               priority as given by adder / learner
//   level[0]     [S0] f64                     sum-tree leaves = raw_prio^alpha
//   level[l]     [S_l] f64                    64-ary sum tree: level[l][j] =
//                                             wave_scan_total(level[l-1][64j..64j+63])
// S0 = roundup(capacity, 64); S_{l+1} = roundup(S_l / 64, 64) until S_l == 64 (the top
// level has exactly 64 entries; the root total is recomputed by the sampling wave).
// When the top level has at most kTopComputed entries with children (1M slots: 4), readers
// compute them from their children (the same wave scans, so the same bits) instead of
// reading the stored top, and the one-launch priority update does not maintain it: the
// top was the one level many workgroups of that launch write into, which cost it a
// last-workgroup hand-off (round 5).
//
// The fan-out is the wavefront width: one wave reads the 64 children of a node in one
// coalesced 512-B load, prefix-sums them with a 6-step shuffle scan, and picks the child
// with a ballot.  A 1 M-slot table is 4 levels, so a draw is 4 dependent 512-B reads
// instead of the 20 dependent 8-B reads of a binary tree.
//
// Sampling (Reverb Prioritized(alpha)): target t = u * total, u = Philox4x32-10 53-bit
// uniform of counter (j, step); descend choosing the first child whose inclusive prefix
// exceeds t.  Uniform(): slot = floor(u * size).  FIFO remover: slot = key % capacity.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "common.h"
#include "detmath.h"
#include "kernels.h"
#include "profiler.h"
#include "rescale.h"

namespace acme {
// Timing experiment hook (rescale.h): the DQN learner sets it while ACME_V_STAMPS=1.
uint64_t* g_update_stamps = nullptr;
}  // namespace acme

using namespace acme;

// Host inserts (the actor side, adders/reverb/transition.py:119-165 -> one item per env
// step) go through a ring of pinned staging chunks and the table's own non-blocking side
// stream: the caller's thread packs items into a pinned chunk (or writes them there
// directly, acme_replay_stage), acme_replay_commit issues the H2D copies and the tree
// refresh on the side stream and returns without waiting.  A chunk is reused only after
// its copies completed (its event), so the host blocks only when PCIe falls 4 chunks behind.
//
// Ordering (no per-step event cost on the learner stream):
//  * every device operation on a caller stream (sample, gather, update_priorities, ...)
//    first waits on the latest insert's event if that stream has not yet waited for it, so
//    a sample sees every committed item;
//  * the streams those operations ran on are remembered; a commit records an event on each
//    of them (and on the committing caller's stream) and makes the side stream wait, so an
//    insert never overwrites a slot an earlier-issued gather still reads, nor rescans the
//    tree concurrently with an earlier priority update.
// Streams passed to a table must stay alive while the table does (torch streams do).
constexpr int kStageChunks = 4;
constexpr int64_t kStageBytes = 32ll << 20;  // per chunk
constexpr int kMaxReaders = 8;
constexpr int kMaxPipes = 8;

struct acme_replay {
  acme_replay_config cfg;
  int nlevels = 0;
  int64_t level_size[8] = {};
  double* levels[8] = {};
  double* raw_prio = nullptr;
  uint64_t* keys = nullptr;
  int32_t* winner = nullptr;  // per-slot scratch for last-wins priority updates
  uint32_t* upd_done = nullptr;  // the fused update's finished-workgroup count (0 between launches)
  int64_t* upd_slots = nullptr;  // per-update scratch (resolved slot)
  int32_t* upd_valid = nullptr;  // per-update scratch (key still present)
  int64_t upd_cap = 0;
  uint8_t* fields[ACME_MAX_FIELDS] = {};
  int64_t inserted = 0;  // total items ever inserted (host side; = next key)
  std::mutex mu;
  // Insert path.
  hipStream_t side = nullptr;
  hipStream_t upload = nullptr;  // H2D of staged chunks into their device mirrors
  hipEvent_t insert_event = nullptr;  // recorded on `side` after each commit
  uint64_t insert_seq = 0;            // commits so far
  int64_t stage_items = 0;            // items per staging chunk
  int64_t stage_off[ACME_MAX_FIELDS + 3] = {};  // field rows, then keys, raw prio, leaves
  uint8_t* stage[kStageChunks] = {};
  uint8_t* stage_dev[kStageChunks] = {};  // device mirror of each chunk (upload target)
  hipEvent_t stage_up[kStageChunks] = {};  // the chunk's upload to its mirror completed
  hipEvent_t stage_done[kStageChunks] = {};
  bool stage_used[kStageChunks] = {};
  int stage_next = 0;
  int staged = -1;  // chunk handed out by acme_replay_stage, not yet committed
  int64_t staged_n = 0;
  std::thread::id staged_by;         // the thread that must commit it
  std::condition_variable stage_cv;  // other threads wait here for the commit
  struct Reader {
    hipStream_t s;
    hipEvent_t ev;
    uint64_t waited;  // insert_seq this stream last waited for
    bool dirty;       // has table work issued since the last commit
  } readers[kMaxReaders] = {};
  int nreaders = 0;
  std::mutex order_mu;
  // Pipelined readers (acme_replay_sample_gather_pipe): each holds at most one drawn batch
  // whose rows are not copied yet.  Every operation that writes rows issues those copies
  // first (flush_pipes), so a pending batch always gets the rows of its drawn keys.
  struct Pipe {
    bool open, pending;
    hipEvent_t ev;  // orders a new stream after copies flushed on the pipe's previous one
    hipStream_t st;
    int64_t batch;
    const int64_t* slots;
    void* out[ACME_MAX_FIELDS];
  } pipes[kMaxPipes] = {};
};

namespace {

// Inclusive Hillis-Steele scan over the 64 lanes of a wave, f64.  The order of the
// additions is fixed (round d adds the value d lanes below), which the oracle
// restates exactly (oracle/replay_oracle.c: wave_scan64).
__device__ __forceinline__ double wave_scan64(double x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    double y = __shfl_up(x, d, 64);
    if (lane >= d) x = y + x;
  }
  return x;
}

// The scan's total (its lane-63 value) in every lane, with the same bits: lane 63 of the
// scan adds aligned blocks pairwise (round d: the block of d lanes ending at 63 - d to the one
// ending at 63), and so does this butterfly (each round adds the aligned neighbour block of
// the same size; f64 addition is commutative).  DPP moves for blocks of 1..8 lanes, a swizzle
// for 16 and two lane reads for 32 replace six rounds of LDS permutes.  The whole wave must
// be active (as for wave_scan64).
template <int Ctrl>
__device__ __forceinline__ double dpp_f64(double x) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, Ctrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), Ctrl, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ double wave_total64(double x) {
  x = x + dpp_f64<0xB1>(x);   // quad_perm [1,0,3,2]: pairs
  x = x + dpp_f64<0x4E>(x);   // quad_perm [2,3,0,1]: quads
  x = x + dpp_f64<0x141>(x);  // row_half_mirror: blocks of 8
  x = x + dpp_f64<0x140>(x);  // row_mirror: blocks of 16
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const int lo = __builtin_amdgcn_ds_swizzle((int)(uint32_t)u, 0x401F);  // lane ^ 16
  const int hi = __builtin_amdgcn_ds_swizzle((int)(uint32_t)(u >> 32), 0x401F);
  x = x + __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  const uint64_t v = __builtin_bit_cast(uint64_t, x);
  const uint32_t a0 = __builtin_amdgcn_readlane((int)(uint32_t)v, 31);
  const uint32_t a1 = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 31);
  const uint32_t b0 = __builtin_amdgcn_readlane((int)(uint32_t)v, 63);
  const uint32_t b1 = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
  return __builtin_bit_cast(double, ((uint64_t)a1 << 32) | a0) +
         __builtin_bit_cast(double, ((uint64_t)b1 << 32) | b0);
}

__device__ __forceinline__ int select_child(double v, double s, double t) {
  const uint64_t le = __ballot(s <= t);
  const uint64_t nz = __ballot(v > 0.0);
  int idx = __popcll(le);
  const int last = nz ? 63 - __clzll(nz) : 0;
  if (idx > last) idx = last;
  return idx;
}

// One wave per draw.  levels passed top-first in a small struct by value.  top_nodes > 0:
// the top level's first top_nodes entries are computed from level nlevels - 2 (the rest are
// zero), not read.
constexpr int kTopComputed = 16;
struct TreeView {
  const double* level[8];
  int nlevels;
  int top_nodes = 0;
};

// The top level's entry `lane` as its writers store it: the scan total of its 64 children
// (tree.top_nodes > 0), else the stored entry.  All children loads issue before the scans.
__device__ __forceinline__ double top_entry(const double* const* level, int nlevels,
                                            int top_nodes) {
  const int lane = threadIdx.x & 63;
  if (top_nodes <= 0) return level[nlevels - 1][lane];
  const double* c = level[nlevels - 2];
  double ch[kTopComputed];
#pragma unroll
  for (int g = 0; g < kTopComputed; ++g) ch[g] = g < top_nodes ? c[g * 64 + lane] : 0.0;
  double v = 0.0;
#pragma unroll
  for (int g = 0; g < kTopComputed; ++g) {
    if (g >= top_nodes) break;  // wave-uniform
    const double t = wave_total64(ch[g]);
    if (lane == g) v = t;
  }
  return v;
}

// Draw j of a prioritized sample by one wave (every lane returns the same slot and
// probability): the descent the oracle restates (oracle/replay_oracle.c).
__device__ __forceinline__ void draw_prioritized(const TreeView& tree, int64_t size,
                                                 uint64_t seed, uint64_t step, int64_t j,
                                                 int64_t* slot_out, double* prob_out) {
  const int lane = threadIdx.x & 63;
  const double u = sample_uniform(seed, step, (uint32_t)j);

  int64_t node = 0;
  double t = 0.0, total = 0.0, leaf_value = 0.0;
  // A computed top level's children rows (level nlevels - 2) are already in registers when
  // the descent reaches that level: its row is taken from them instead of loaded again (one
  // dependent round trip fewer per draw, round 6).
  const int top = tree.nlevels - 1;
  double ch[kTopComputed];
  for (int l = top; l >= 0; --l) {
    const int64_t base = node * 64;
    double v;
    if (l == top) {
      if (tree.top_nodes > 0) {
        const double* c = tree.level[top - 1];
#pragma unroll
        for (int g = 0; g < kTopComputed; ++g) ch[g] = g < tree.top_nodes ? c[g * 64 + lane] : 0.0;
        v = 0.0;
#pragma unroll
        for (int g = 0; g < kTopComputed; ++g) {
          if (g >= tree.top_nodes) break;  // wave-uniform
          const double tt = wave_total64(ch[g]);
          if (lane == g) v = tt;
        }
      } else {
        v = tree.level[top][lane];
      }
    } else if (l == top - 1 && tree.top_nodes > 0) {
      v = 0.0;  // row `node` (< top_nodes) of level top - 1: ch[node]
#pragma unroll
      for (int g = 0; g < kTopComputed; ++g)
        if (g == node) v = ch[g];
    } else {
      v = tree.level[l][base + lane];
    }
    const double s = wave_scan64(v);
    if (l == tree.nlevels - 1) {
      total = __shfl(s, 63, 64);
      if (!(total > 0.0)) break;
      t = u * total;
    }
    const int idx = select_child(v, s, t);
    const double excl = idx > 0 ? __shfl(s, idx - 1, 64) : 0.0;
    leaf_value = __shfl(v, idx, 64);
    t = t - excl;
    node = base + idx;
  }
  int64_t slot;
  double prob;
  if (!(total > 0.0)) {  // every priority is zero: uniform fallback
    slot = (int64_t)(u * (double)size);
    if (slot >= size) slot = size - 1;
    prob = 1.0 / (double)size;
  } else {
    slot = node;
    prob = leaf_value / total;
  }
  *slot_out = slot;
  *prob_out = prob;
}

__global__ void __launch_bounds__(256) sample_prioritized_kernel(
    TreeView tree, const double* __restrict__ raw_prio, const uint64_t* __restrict__ keys,
    int64_t batch, int64_t size, uint64_t seed, uint64_t step, double prob_scale,
    int64_t* out_slots, uint64_t* out_keys, double* out_probs, int64_t* out_size,
    double* out_prio) {
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (j >= batch) return;  // wave-uniform
  int64_t slot;
  double prob;
  draw_prioritized(tree, size, seed, step, j, &slot, &prob);
  prob *= prob_scale;  // 1 (exact) unless this table is one shard of a global draw
  if (lane == 0) {
    out_slots[j] = slot;
    if (out_keys) out_keys[j] = keys[slot];
    if (out_probs) out_probs[j] = prob;
    if (out_size) out_size[j] = size;
    if (out_prio) out_prio[j] = raw_prio[slot];
  }
}

__global__ void sample_uniform_kernel(const double* __restrict__ raw_prio,
                                      const uint64_t* __restrict__ keys, int64_t batch,
                                      int64_t size, uint64_t seed, uint64_t step,
                                      double prob_scale, int64_t* out_slots, uint64_t* out_keys,
                                      double* out_probs, int64_t* out_size,
                                      double* out_prio) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= batch) return;
  const double u = sample_uniform(seed, step, (uint32_t)j);
  int64_t slot = (int64_t)(u * (double)size);
  if (slot >= size) slot = size - 1;
  out_slots[j] = slot;
  if (out_keys) out_keys[j] = keys[slot];
  if (out_probs) out_probs[j] = (1.0 / (double)size) * prob_scale;
  if (out_size) out_size[j] = size;
  if (out_prio) out_prio[j] = raw_prio[slot];
}

// The top level's entries with children, when few enough for readers to compute them
// (TreeView::top_nodes), else 0 (read the stored top).
int computed_top_nodes(const acme_replay* r) {
  if (r->nlevels < 2) return 0;
  const int64_t n = r->level_size[r->nlevels - 2] / 64;
  return n <= kTopComputed ? (int)n : 0;
}
TreeView tree_view(const acme_replay* r) {
  TreeView tv;
  for (int l = 0; l < 8; ++l) tv.level[l] = r->levels[l];
  tv.nlevels = r->nlevels;
  tv.top_nodes = computed_top_nodes(r);
  return tv;
}

// Sampling mass of the table (one wave): the prioritized root total with the sampler's own
// scan (same bits as `total` in sample_prioritized_kernel), or the item count (uniform).
__global__ void total_kernel(TreeView tree, int prioritized, int64_t size,
                             double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  if (!prioritized) {
    if (lane == 0) *out = (double)size;
    return;
  }
  const double s = wave_total64(top_entry(tree.level, tree.nlevels, tree.top_nodes));
  if (lane == 63) *out = s;
}

// Row gather of every field in ONE launch: one workgroup per (row, field).  Rows that
// are 16-B multiples (the 28,224-B Atari frames, 96-B control observations) move as
// 16-B vectors with up to 8 loads in flight per thread; other rows as 4-B words or bytes.
struct GatherArgs {
  const uint8_t* src[ACME_MAX_FIELDS];
  uint8_t* dst[ACME_MAX_FIELDS];
  int64_t bytes[ACME_MAX_FIELDS];
};

__global__ void __launch_bounds__(256) gather_fields_kernel(GatherArgs g,
                                                            const int64_t* __restrict__ slots) {
  const int f = blockIdx.y;
  const int64_t row = blockIdx.x;
  const int64_t slot = slots[row];
  const int64_t nb = g.bytes[f];
  const uint8_t* s8 = g.src[f] + slot * nb;
  uint8_t* d8 = g.dst[f] + row * nb;
  if ((nb & 15) == 0 && ((reinterpret_cast<uintptr_t>(d8) | reinterpret_cast<uintptr_t>(s8)) & 15) == 0) {
    const int64_t nvec = nb >> 4;
    const uint4* __restrict__ s = reinterpret_cast<const uint4*>(s8);
    uint4* __restrict__ d = reinterpret_cast<uint4*>(d8);
    for (int64_t i0 = threadIdx.x; i0 < nvec; i0 += 8 * blockDim.x) {
      uint4 r[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int64_t i = i0 + (int64_t)k * blockDim.x;
        if (i < nvec) r[k] = s[i];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int64_t i = i0 + (int64_t)k * blockDim.x;
        if (i < nvec) d[i] = r[k];
      }
    }
  } else if ((nb & 3) == 0 && ((reinterpret_cast<uintptr_t>(d8) | reinterpret_cast<uintptr_t>(s8)) & 3) == 0) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(s8);
    uint32_t* d = reinterpret_cast<uint32_t*>(d8);
    for (int64_t i = threadIdx.x; i < (nb >> 2); i += blockDim.x) d[i] = s[i];
  } else {
    for (int64_t i = threadIdx.x; i < nb; i += blockDim.x) d8[i] = s8[i];
  }
}

// Row gather as wave-sized pieces.  A piece is what one wave-instruction moves: 64 lanes x
// 16 B = 1 KiB of ONE row of one field (pieces never cross rows, so the row, its slot and
// the field are wave-uniform scalars).  Rows of at least 1 KiB (the 28,224-B Atari frames:
// 28 pieces, the last one 576 B) are split into pieces, field-major then row then piece;
// each wave takes K consecutive pieces, issues all K loads, then the K stores, and strides
// over the rest.  Smaller rows (a, r, d) are copied 64 rows per wave by 4-B words after the
// big fields.  Source rows are read once, so they are loaded non-temporal.
struct PieceArgs {
  const uint8_t* src[ACME_MAX_FIELDS];
  uint8_t* dst[ACME_MAX_FIELDS];
  int32_t bytes[ACME_MAX_FIELDS];
  int32_t ppr[ACME_MAX_FIELDS];    // pieces per row of a big field (0: small field)
  int32_t first[ACME_MAX_FIELDS + 1];  // first piece of each big field; first[nbig] = total
  int32_t big[ACME_MAX_FIELDS];    // field indices of the big fields, then the small ones
  int32_t nbig, nsmall;
};

using vu4 = __attribute__((ext_vector_type(4))) uint32_t;

template <int K>
__global__ void __launch_bounds__(256) gather_pieces_kernel(PieceArgs args,
                                                            const int64_t* __restrict__ slots,
                                                            int32_t batch) {
  __shared__ PieceArgs a;  // LDS copy of the tables (see gather_row_kernel)
  if (threadIdx.x == 0) a = args;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int32_t nwaves = gridDim.x * 4;
  const int32_t total = a.first[a.nbig];
  for (int32_t p0 = wave * K; p0 < total; p0 += nwaves * K) {
    vu4 v[K];
    uint8_t* dst[K];
    bool ok[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int32_t p = p0 + k;
      ok[k] = false;
      dst[k] = nullptr;
      if (p >= total) continue;
      int i = 0;
      while (i + 1 < a.nbig && p >= a.first[i + 1]) ++i;
      const int f = a.big[i];
      const int32_t local = p - a.first[i];
      const int32_t r = local / a.ppr[i];
      const int32_t q = local - r * a.ppr[i];
      const int32_t off = q * 1024 + lane * 16;
      ok[k] = off < a.bytes[f];
      const int64_t slot = slots[r];
      const vu4* s = reinterpret_cast<const vu4*>(a.src[f] + slot * a.bytes[f] + off);
      dst[k] = a.dst[f] + (int64_t)r * a.bytes[f] + off;
      if (ok[k]) v[k] = __builtin_nontemporal_load(s);
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (ok[k]) *reinterpret_cast<vu4*>(dst[k]) = v[k];
  }
  // Small fields: wave w copies rows [64 w', 64 w' + 64) of small field s, 4 B per step.
  const int32_t per = (batch + 63) / 64;
  for (int32_t w = wave; w < a.nsmall * per; w += nwaves) {
    const int f = a.big[a.nbig + w / per];
    const int32_t r = (w % per) * 64 + lane;
    if (r >= batch) continue;
    const int64_t slot = slots[r];
    const uint32_t* s = reinterpret_cast<const uint32_t*>(a.src[f] + slot * a.bytes[f]);
    uint32_t* d = reinterpret_cast<uint32_t*>(a.dst[f] + (int64_t)r * a.bytes[f]);
    for (int j = 0; j < a.bytes[f] / 4; ++j) d[j] = s[j];
  }
}

// The transition layout (two equal big rows o_tm1 / o_t, small a / r / d): one workgroup per
// sampled row moves both big rows (2 x nvec 16-B chunks, up to MAXC per thread, all loads
// issued before the first store) and the small rows.  Every address comes from kernel
// arguments and the row's slot, so the loads are global loads with nothing between them
// that waits on memory.
struct SmallFields {
  const uint8_t* src[ACME_MAX_FIELDS];
  uint8_t* dst[ACME_MAX_FIELDS];
  int32_t words[ACME_MAX_FIELDS];
  int32_t n;
};

template <int T, int MAXC, bool NT>
__global__ void __launch_bounds__(T) gather_pair_kernel(const uint8_t* __restrict__ s0,
                                                        const uint8_t* __restrict__ s1,
                                                        uint8_t* __restrict__ d0,
                                                        uint8_t* __restrict__ d1, int32_t nvec,
                                                        SmallFields sm,
                                                        const int64_t* __restrict__ slots) {
  const int64_t r = blockIdx.x;
  const int64_t slot = slots[r];
  const int64_t rb = (int64_t)nvec * 16;
  const vu4* a0 = reinterpret_cast<const vu4*>(s0 + slot * rb);
  const vu4* a1 = reinterpret_cast<const vu4*>(s1 + slot * rb);
  vu4* b0 = reinterpret_cast<vu4*>(d0 + r * rb);
  vu4* b1 = reinterpret_cast<vu4*>(d1 + r * rb);
  vu4 v[MAXC];
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    // Unconditional loads (a lane past the end re-reads the last chunk): a load under a
    // branch gets a full vmcnt(0) wait at the join, which would serialise the row.
    const int32_t c = min(threadIdx.x + k * T, 2 * nvec - 1);
    const vu4* p = c < nvec ? a0 + c : a1 + (c - nvec);
    v[k] = NT ? __builtin_nontemporal_load(p) : *p;
  }
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int32_t c = threadIdx.x + k * T;
    vu4* p = c < nvec ? b0 + c : b1 + (c - nvec);
    if (c < 2 * nvec) *p = v[k];
  }
#pragma unroll
  for (int q = 0; q < ACME_MAX_FIELDS; ++q) {
    if (q >= sm.n) break;
    for (int w = threadIdx.x; w < sm.words[q]; w += T)
      reinterpret_cast<uint32_t*>(sm.dst[q] + r * 4 * sm.words[q])[w] =
          reinterpret_cast<const uint32_t*>(sm.src[q] + slot * 4 * sm.words[q])[w];
  }
}

// Sample + gather fused for the transition layout: workgroup j's first wave draws item j
// (prioritized descent or uniform, the same arithmetic as the sampling kernels) and writes
// the sample record; then the workgroup copies the item's rows as gather_pair_kernel does.
// One launch instead of two, and no slot round trip through memory.
template <bool PRIO, int T, int MAXC>
__global__ void __launch_bounds__(T) sample_gather_pair_kernel(
    TreeView tree, const double* __restrict__ raw_prio, const uint64_t* __restrict__ keys,
    int64_t size, uint64_t seed, uint64_t step, double prob_scale, int64_t* out_slots,
    uint64_t* out_keys, double* out_probs, int64_t* out_size, double* out_prio,
    const uint8_t* __restrict__ s0, const uint8_t* __restrict__ s1, uint8_t* __restrict__ d0,
    uint8_t* __restrict__ d1, int32_t nvec, SmallFields sm, uint16_t* __restrict__ fb) {
  __shared__ int64_t s_slot;
  const int64_t r = blockIdx.x;
  if (threadIdx.x < 64) {
    int64_t slot;
    double prob;
    if (PRIO) {
      draw_prioritized(tree, size, seed, step, r, &slot, &prob);
    } else {
      const double u = sample_uniform(seed, step, (uint32_t)r);
      slot = (int64_t)(u * (double)size);
      if (slot >= size) slot = size - 1;
      prob = 1.0 / (double)size;
    }
    prob *= prob_scale;
    if (threadIdx.x == 0) {
      s_slot = slot;
      out_slots[r] = slot;
      if (out_probs) out_probs[r] = prob;
      if (out_size) out_size[r] = size;
    }
  }
  __syncthreads();
  const int64_t slot = s_slot;
  // The record's key and priority after the barrier: their loads ride with the row copy's
  // instead of delaying it by one round trip (the barrier waits for outstanding loads).
  if (threadIdx.x == 64) {
    if (out_keys) out_keys[r] = keys[slot];
    if (out_prio) out_prio[r] = raw_prio[slot];
  }
  const int64_t rb = (int64_t)nvec * 16;
  const vu4* a0 = reinterpret_cast<const vu4*>(s0 + slot * rb);
  const vu4* a1 = reinterpret_cast<const vu4*>(s1 + slot * rb);
  vu4* b0 = reinterpret_cast<vu4*>(d0 + r * rb);
  vu4* b1 = reinterpret_cast<vu4*>(d1 + r * rb);
  vu4 v[MAXC];
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int32_t c = min(threadIdx.x + k * T, 2 * nvec - 1);
    const vu4* p = c < nvec ? a0 + c : a1 + (c - nvec);
    v[k] = __builtin_nontemporal_load(p);
  }
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int32_t c = threadIdx.x + k * T;
    vu4* p = c < nvec ? b0 + c : b1 + (c - nvec);
    if (c < 2 * nvec) *p = v[k];
  }
  if (fb) {  // the learner's exact f16 copy of both frames: rows [0, B) o_tm1, [B, 2B) o_t
    const int64_t B = gridDim.x;
#pragma unroll
    for (int k = 0; k < MAXC; ++k) {
      const int32_t c = threadIdx.x + k * T;
      if (c >= 2 * nvec) continue;
      const int64_t row = c < nvec ? r : B + r;
      const int32_t cc = c < nvec ? c : c - nvec;
      vu4* q = reinterpret_cast<vu4*>(fb + (row * nvec + cc) * 16);
      // f16(byte) is exact (8 significant bits).
      auto cvt = [](uint32_t x, int sh) {
        return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)(uint16_t)((x >> sh) & 0xffu));
      };
      vu4 lo, hi;
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        lo[2 * w] = cvt(v[k][w], 0) | (cvt(v[k][w], 8) << 16);
        lo[2 * w + 1] = cvt(v[k][w], 16) | (cvt(v[k][w], 24) << 16);
        hi[2 * w] = cvt(v[k][w + 2], 0) | (cvt(v[k][w + 2], 8) << 16);
        hi[2 * w + 1] = cvt(v[k][w + 2], 16) | (cvt(v[k][w + 2], 24) << 16);
      }
      q[0] = lo;
      q[1] = hi;
    }
  }
#pragma unroll
  for (int q = 0; q < ACME_MAX_FIELDS; ++q) {
    if (q >= sm.n) break;
    for (int w = threadIdx.x; w < sm.words[q]; w += T)
      reinterpret_cast<uint32_t*>(sm.dst[q] + r * 4 * sm.words[q])[w] =
          reinterpret_cast<const uint32_t*>(sm.src[q] + slot * 4 * sm.words[q])[w];
  }
}

// Pipelined draw + gather (round 6; acme_replay_sample_gather_pipe): workgroup j's first wave
// draws item j of the NEW batch (the sampling arithmetic above) and writes its record, while
// waves 1-3 copy row j of the batch the previous launch drew (its slots already in memory,
// one load away).  The descent's chain of dependent tree loads thus runs under the previous
// batch's row copy instead of in front of it, and no barrier ties the two together.
template <bool PRIO, int MAXC>
__global__ void __launch_bounds__(256) sample_gather_pipe_kernel(
    TreeView tree, const double* __restrict__ raw_prio, const uint64_t* __restrict__ keys,
    int64_t size, uint64_t seed, uint64_t step, int64_t batch, int64_t* out_slots,
    uint64_t* out_keys, double* out_probs, int64_t* out_size, double* out_prio,
    const int64_t* __restrict__ pend_slots, int64_t pend_batch, const uint8_t* __restrict__ s0,
    const uint8_t* __restrict__ s1, uint8_t* __restrict__ d0, uint8_t* __restrict__ d1,
    int32_t nvec, SmallFields sm) {
  constexpr int T = 192;  // copy threads (waves 1-3)
  const int64_t r = blockIdx.x;
  if (threadIdx.x < 64) {
    if (r >= batch) return;  // wave-uniform
    int64_t slot;
    double prob;
    if (PRIO) {
      draw_prioritized(tree, size, seed, step, r, &slot, &prob);
    } else {
      const double u = sample_uniform(seed, step, (uint32_t)r);
      slot = (int64_t)(u * (double)size);
      if (slot >= size) slot = size - 1;
      prob = 1.0 / (double)size;
    }
    if (threadIdx.x == 0) {
      out_slots[r] = slot;
      if (out_probs) out_probs[r] = prob;
      if (out_size) out_size[r] = size;
      if (out_keys) out_keys[r] = keys[slot];
      if (out_prio) out_prio[r] = raw_prio[slot];
    }
    return;
  }
  if (r >= pend_batch) return;  // workgroup-uniform
  const int t = threadIdx.x - 64;
  const int64_t slot = pend_slots[r];
  const int64_t rb = (int64_t)nvec * 16;
  const vu4* a0 = reinterpret_cast<const vu4*>(s0 + slot * rb);
  const vu4* a1 = reinterpret_cast<const vu4*>(s1 + slot * rb);
  vu4* b0 = reinterpret_cast<vu4*>(d0 + r * rb);
  vu4* b1 = reinterpret_cast<vu4*>(d1 + r * rb);
  vu4 v[MAXC];
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int32_t c = min(t + k * T, 2 * nvec - 1);  // unconditional (see gather_pair_kernel)
    const vu4* p = c < nvec ? a0 + c : a1 + (c - nvec);
    v[k] = __builtin_nontemporal_load(p);
  }
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int32_t c = t + k * T;
    vu4* p = c < nvec ? b0 + c : b1 + (c - nvec);
    // Non-temporal: a prefetching reader's learner reads these rows steps later (six
    // alternating 300-step pairs, DQN 0.4701 -> 0.4679 ms; round 6,
    // profiles/r06/replay/ab_nt_row_stores.log).
    if (c < 2 * nvec) __builtin_nontemporal_store(v[k], p);
  }
#pragma unroll
  for (int q = 0; q < ACME_MAX_FIELDS; ++q) {
    if (q >= sm.n) break;
    for (int w = t; w < sm.words[q]; w += T)
      reinterpret_cast<uint32_t*>(sm.dst[q] + r * 4 * sm.words[q])[w] =
          reinterpret_cast<const uint32_t*>(sm.src[q] + slot * 4 * sm.words[q])[w];
  }
}
constexpr int kPipeChunks = 19;  // 16-B chunks per copy thread: rows up to 192 x 19 x 8 B

// Sample + gather fused for rows of small fields only (the control-suite transitions:
// every field under 1 KB): one wave per sampled row draws it (the sampling kernels'
// arithmetic) and copies its fields, 4 rows per workgroup, no block barrier.
template <bool PRIO>
__global__ void __launch_bounds__(256) sample_gather_small_kernel(
    TreeView tree, const double* __restrict__ raw_prio, const uint64_t* __restrict__ keys,
    int64_t batch, int64_t size, uint64_t seed, uint64_t step, double prob_scale,
    int64_t* out_slots, uint64_t* out_keys, double* out_probs, int64_t* out_size,
    double* out_prio, SmallFields sm) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= batch) return;  // wave-uniform
  int64_t slot;
  double prob;
  if (PRIO) {
    draw_prioritized(tree, size, seed, step, r, &slot, &prob);
  } else {
    const double u = sample_uniform(seed, step, (uint32_t)r);
    slot = (int64_t)(u * (double)size);
    if (slot >= size) slot = size - 1;
    prob = 1.0 / (double)size;
  }
  prob *= prob_scale;
  if (lane == 0) {
    out_slots[r] = slot;
    if (out_keys) out_keys[r] = keys[slot];
    if (out_probs) out_probs[r] = prob;
    if (out_size) out_size[r] = size;
    if (out_prio) out_prio[r] = raw_prio[slot];
  }
#pragma unroll
  for (int q = 0; q < ACME_MAX_FIELDS; ++q) {
    if (q >= sm.n) break;
    for (int w = lane; w < sm.words[q]; w += 64)
      reinterpret_cast<uint32_t*>(sm.dst[q] + r * 4 * sm.words[q])[w] =
          reinterpret_cast<const uint32_t*>(sm.src[q] + slot * 4 * sm.words[q])[w];
  }
}

// Recompute level[l] nodes from their 64 children (one wave per node).
// Mode A: contiguous node range [node_begin, node_begin + count).
// Mode B: node = slots[j] >> (6 l) for j < count (duplicates recompute identically).
__global__ void __launch_bounds__(256) level_update_kernel(
    const double* __restrict__ child, double* __restrict__ parent, int64_t node_begin,
    int64_t count, const int64_t* __restrict__ slots, const int32_t* __restrict__ valid,
    int shift) {
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (j >= count) return;
  int64_t node;
  if (slots) {
    if (valid && !valid[j]) return;
    node = slots[j] >> shift;
  } else {
    node = node_begin + j;
  }
  const double v = child[node * 64 + lane];
  const double s = wave_total64(v);
  if (lane == 63) parent[node] = s;
}

// Priority updates from the learner (device keys).  Pass 1: resolve slots, check the
// key still lives in its slot, and elect the LAST update of each slot with atomicMax.
__global__ void prio_resolve_kernel(const uint64_t* __restrict__ upd_keys, int64_t n,
                                    const uint64_t* __restrict__ keys, int64_t capacity,
                                    int64_t* __restrict__ out_slots,
                                    int32_t* __restrict__ valid, int32_t* __restrict__ winner) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t k = upd_keys[j];
  const int64_t slot = (int64_t)(k % (uint64_t)capacity);
  const int ok = keys[slot] == k;
  out_slots[j] = slot;
  valid[j] = ok;
  if (ok) atomicMax(&winner[slot], (int32_t)j);
}

// Pass 2: the elected update writes raw priority and leaf = p^alpha.
__global__ void prio_write_kernel(const double* __restrict__ prios, int64_t n,
                                  const int64_t* __restrict__ slots,
                                  const int32_t* __restrict__ valid,
                                  const int32_t* __restrict__ winner, double alpha,
                                  double* __restrict__ raw_prio, double* __restrict__ leaves,
                                  const Gate gate) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || !valid[j] || gate_skip(gate)) return;
  const int64_t slot = slots[j];
  if (winner[slot] != (int32_t)j) return;
  const double p = prios[j];
  raw_prio[slot] = p;
  leaves[slot] = det_pow_priority(p, alpha);
}

// Pass 3 (after all writes): reset the election scratch.
__global__ void prio_reset_kernel(const int64_t* __restrict__ slots,
                                  const int32_t* __restrict__ valid, int64_t n,
                                  int32_t* __restrict__ winner) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || !valid[j]) return;
  winner[slots[j]] = -1;
}

// update_priorities in ONE launch.  Updates are partitioned over the workgroups by their
// ancestor at level h = nlevels - 2 (owner = slot >> 6h, workgroup owner % G), so every
// update of a slot, and every touched node of levels 1..h, belongs to exactly one workgroup:
// it elects the last valid update per slot in LDS (largest j wins, Reverb's in-order
// application) and computes its leaves p^alpha and its nodes of levels 1..h.  The children
// of those nodes are loaded up front (one round of loads issued together right after the
// keys are resolved), the new values substituted in LDS and each node rescanned from LDS, so
// no store has to be read back.  The top level (whose children many workgroups write) is
// rescanned by the LAST workgroup to finish: the level-h values are stored write-through
// (agent-scope atomic stores, drained before the workgroup counts itself) and read back by
// agent-scope atomic loads, the hand-off form that needs no L2 writeback or invalidate
// (cdna_hip_programming.md G16), so the update is one launch instead of two (round 4: a
// 10.2 us kernel + a 5.2 us one-workgroup launch for the top level).
constexpr int kFusedUpdateMax = 4096;
constexpr int kFusedUpdateBlocks = 256;
constexpr int kUpdPairs = 32;  // (level, node) pairs a workgroup prefetches; else read back
struct FusedUpdateArgs {
  const uint64_t* upd_keys;
  const double* prios;
  int n;
  int64_t capacity;
  const uint64_t* keys;
  double alpha;
  double* raw_prio;
  double* level[8];
  int64_t top_nodes;  // nodes of level nlevels - 2 (the top level's entries that have children)
  int top_computed;   // readers compute the top level (computed_top_nodes > 0): not stored
  int nlevels;
  uint32_t* done;     // workgroups finished (the last one rescans the top; it resets the count)
  Gate gate;  // a learner step that was skipped writes no priority
  // job.s: the learner step's rescale, run by workgroup 0 (the update workgroups are 1..G).
  // With a step verdict (kRgStep) the update workgroups wait for it (StepGuard::vseq) and
  // write nothing when the step was skipped, for every reason the rescale decides
  // (overflow, underflow, a timed-out unroll, the sticky hold, another rank's skip).
  RescaleJob job;
  // Timing experiment (ACME_V_STAMPS=1 in the DQN learner, tools/update_stamps.py): thread 0 of
  // each workgroup stores s_memrealtime (100 MHz) at its phase boundaries, 8 slots per
  // workgroup: entry, keys resolved (workgroup 0: rescale done), node list, verdict, leaves,
  // levels, exit.
  uint64_t* stamps = nullptr;
};
// Waits (bounded) for the verdict with sequence number seq; true when that step is skipped
// (or the wait timed out: no priority is written, and the timeout is counted in
// g->vtimeout, which the host reads: acme_dqn_verdict_timeouts).  Workgroup 0 of the same
// launch publishes it and was dispatched first, so it is resident or done.
// `first`: thread 0's load of g->vseq issued earlier (its latency overlapped the caller's LDS
// work); polled again only when it did not yet hold this step's verdict.
__device__ __forceinline__ bool wait_verdict_skip(StepGuard* g, uint32_t seq, uint32_t first) {
  __shared__ uint32_t s_v;
  if (threadIdx.x == 0) {
    uint32_t v = first;
    for (int it = 0; it < (1 << 22) && (v >> 1) != (seq & 0x7fffffffu); ++it) {
      __builtin_amdgcn_s_sleep(2);
      v = __hip_atomic_load(&g->vseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const bool got = (v >> 1) == (seq & 0x7fffffffu);
    if (!got) atomicAdd(&g->vtimeout, 1u);
    s_v = got ? (v & 1u) : 1u;
  }
  __syncthreads();
  return s_v != 0u;
}
// A workgroup barrier that orders LDS only: outstanding global loads stay in flight across it
// (__syncthreads also waits for every vector memory operation of the wave).
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// A level-h value other workgroups' top rescan reads: write-through.
__device__ __forceinline__ void store_shared_level(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// R: updates per thread the launch holds (n <= 256 R).  The small form (R = 2, up to 512
// updates: a DQN batch) takes 21 KB of LDS and few registers, so its workgroups fit beside
// the next step's target forward (gemm_p3c12_kernel, 121 KB of LDS per CU), which the
// early start runs at the same time on the side stream; at R = 16 (49 KB, 200 VGPRs) they
// waited for its blocks to retire (24 us in the two-stream trace against 12 us alone,
// profiles/r06/schedule/).
template <int R>
__global__ void __launch_bounds__(256) prio_update_fused_kernel(FusedUpdateArgs a) {
  static_assert(R * 256 <= kFusedUpdateMax, "update capacity");
  __shared__ int64_t s_slot[R * 256];
  __shared__ int s_len, s_np, s_ovf, s_last;
  __shared__ double s_ch[kUpdPairs][64];  // children of each prefetched node
  __shared__ int64_t s_node[kUpdPairs];
  __shared__ int s_lvl[kUpdPairs];
  __shared__ int64_t s_nk[kUpdPairs];  // node << 3 | level: one LDS read per match test
  __shared__ double s_val[kUpdPairs];
  const int first = a.job.s ? 1 : 0;
  auto stamp = [&](int ph) {
    if (a.stamps && threadIdx.x == 0)
      a.stamps[8 * (int64_t)blockIdx.x + ph] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  if (a.job.s && blockIdx.x == 0) {
    rescale_block(a.job);
    stamp(1);
    return;
  }
  const bool verdict = a.job.s && a.job.rg.g && a.job.rg.mode == kRgStep;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wave = tid >> 6, nw = nt >> 6;
  const int G = kFusedUpdateBlocks, bid = (int)blockIdx.x - first;
  const int h = a.nlevels >= 2 ? a.nlevels - 2 : 0;
  bool skip = !verdict && gate_skip(a.gate);
  if (tid == 0) s_len = 0;
  __syncthreads();
  // Round 1: every update's key and priority (all workgroups read all of them; L2-resident
  // after the first), its slot and owner; this workgroup's updates join the list in atomic
  // order, and the thread that read an update keeps it (key, priority, list entry) in
  // registers.  Its stale-key check shares round 2 with the children rows, and its leaf
  // p^alpha is computed while those loads are in flight (round 6: three dependent rounds of
  // global loads became two, and the f64 power left the critical path).
  uint64_t kv[R];
  double pr[R];
  int64_t sl[R];
  int my_e[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    my_e[i] = -1;
    kv[i] = 0;
    pr[i] = 0.0;
    sl[i] = 0;
  }
  if (!skip) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (i * nt >= a.n) break;  // workgroup-uniform
      const int j = tid + i * nt;
      const int jc = j < a.n ? j : a.n - 1;
      kv[i] = a.upd_keys[jc];
      pr[i] = a.prios[jc];
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (i * nt >= a.n) break;
      const int j = tid + i * nt;
      const int64_t slot = (int64_t)(kv[i] % (uint64_t)a.capacity);
      if (j < a.n && (int)((slot >> (6 * h)) % G) == bid) {
        const int e = atomicAdd(&s_len, 1);
        s_slot[e] = slot;
        my_e[i] = e;
        sl[i] = slot;
      }
    }
  }
  __syncthreads();
  stamp(1);
  const int len = s_len;
  if (len > 0) {
    // The distinct nodes of levels 1..h this workgroup recomputes: a thread per (level,
    // update) keeps the node if no earlier update of the list has the same ancestor at that
    // level (a serial scan by one thread took up to 7 us on the workgroup with the most
    // updates, profiles/r05/update_stamps/).  The list's order is the threads' (atomic slot
    // order); every use below matches nodes by (level, node), so the result does not depend
    // on it.  A node whose updates all turn out stale is rescanned from unchanged children:
    // the same value it holds.
    if (tid == 0) {
      s_np = 0;
      s_ovf = 0;
    }
    __syncthreads();
    for (int idx = tid; idx < h * len; idx += nt) {
      const int l = 1 + idx / len, e = idx - (l - 1) * len;
      const int64_t node = s_slot[e] >> (6 * l);
      bool first = true;
      for (int f = 0; f < e && first; ++f) first = (s_slot[f] >> (6 * l)) != node;
      if (!first) continue;
      const int q = atomicAdd(&s_np, 1);
      if (q < kUpdPairs) {
        s_lvl[q] = l;
        s_node[q] = node;
        s_nk[q] = (node << 3) | l;
      } else {
        s_ovf = 1;
      }
    }
    __syncthreads();
    if (tid == 0 && s_np > kUpdPairs) s_np = kUpdPairs;  // (with s_ovf: the read-back path)
    __syncthreads();
    stamp(2);
    const int np = s_np;
    const bool pre = !s_ovf;
    // Round 2, one batch of loads: the stored key of each of this thread's updates (the stale
    // check) and each node's 64 children (a wave per node); the leaves computed meanwhile.
    // (Loops over a thread's updates stop at the workgroup-uniform count, so nothing is
    // evaluated for the unused register slots: the f64 power below for all 16 measured
    // 17 us.)
    uint64_t kt[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (i * nt >= a.n) break;
      kt[i] = my_e[i] >= 0 ? a.keys[sl[i]] : 0;
    }
    if (pre) {
      for (int q = wave; q < np; q += nw)
        s_ch[q][lane] = a.level[s_lvl[q] - 1][s_node[q] * 64 + lane];
    }
    double leafv[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (i * nt >= a.n) break;
      leafv[i] = 0.0;
      if (my_e[i] >= 0) leafv[i] = det_pow_priority(pr[i], a.alpha);
    }
    // Each entry repacked in place as slot << 13 | valid << 12 | j (the node list is built,
    // so s_slot's plain form is no longer read): the election below reads one word per entry.
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (i * nt >= a.n) break;
      if (my_e[i] >= 0)  // valid: the key still lives in its slot (evicted since sampled: ignored)
        s_slot[my_e[i]] = (sl[i] << 13) | ((kt[i] == kv[i] ? 1 : 0) << 12) | (tid + i * nt);
    }
    __syncthreads();
    stamp(4);
    // The verdict's first poll now (thread 0), landing while the LDS work below runs: the
    // barriers below order LDS only, so they do not wait for it.
    uint32_t vfirst = 0;
    if (verdict && tid == 0)
      vfirst = __hip_atomic_load(&a.job.rg.g->vseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // Everything but the stores before the verdict: the last valid update of each slot wins
    // (substituted into its level-1 node's children) and, on the prefetched path, every
    // node's new value rescanned level by level in LDS.
    bool winv[R];
#pragma unroll
    for (int i = 0; i < R; ++i) winv[i] = false;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (i * nt >= a.n) break;
      const int e = my_e[i];
      bool win = e >= 0 && kt[i] == kv[i];
      const int j = tid + i * nt;
      const int64_t me = (sl[i] << 1) | 1;  // same slot, valid
#pragma unroll 4
      for (int f = 0; f < len; ++f) {
        const int64_t x = s_slot[f];
        if ((x >> 12) == me && (int)(x & 4095) > j) win = false;
      }
      winv[i] = win;
    }
    // (The children rows were filled by wave q % nw before the barrier above, so the
    // substitutions below by any wave follow them: ADVICE r5's race.)
    if (pre) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        if (i * nt >= a.n) break;
        if (!winv[i]) continue;
        const int64_t k1 = ((sl[i] >> 6) << 3) | 1;
#pragma unroll 4
        for (int q = 0; q < np; ++q)
          if (s_nk[q] == k1) s_ch[q][sl[i] & 63] = leafv[i];
      }
    }
    lds_barrier();
    if (pre) {
      for (int l = 1; l <= h; ++l) {
        for (int q = wave; q < np; q += nw) {
          if (s_lvl[q] != l) continue;
          const double v = wave_total64(s_ch[q][lane]);
          if (lane == 63) s_val[q] = v;
        }
        lds_barrier();
        if (tid < np && s_lvl[tid] == l) {  // into the parent's children
          const int64_t kp = ((s_node[tid] >> 6) << 3) | (l + 1);
#pragma unroll 4
          for (int q = 0; q < np; ++q)
            if (s_nk[q] == kp) s_ch[q][s_node[tid] & 63] = s_val[tid];
        }
        lds_barrier();
      }
    }
    // The step's verdict (published by workgroup 0's rescale while this workgroup resolved
    // its keys, loaded and computed), before the first store.
    stamp(7);
    if (verdict) skip = wait_verdict_skip(a.job.rg.g, a.job.rg.seq, vfirst);
    stamp(3);
    if (!skip) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        if (i * nt >= a.n) break;
        if (!winv[i]) continue;
        a.raw_prio[sl[i]] = pr[i];
        if (h == 0 && !a.top_computed) store_shared_level(a.level[0] + sl[i], leafv[i]);
        else a.level[0][sl[i]] = leafv[i];
      }
      if (pre) {
        for (int q = tid; q < np; q += nt) {
          const int l = s_lvl[q];
          if (l == h && !a.top_computed) store_shared_level(a.level[l] + s_node[q], s_val[q]);
          else a.level[l][s_node[q]] = s_val[q];
        }
      } else {
        __syncthreads();
        for (int l = 1; l <= h; ++l) {  // read back what this workgroup stored (levels below are its own)
          for (int e = wave; e < len; e += nw) {
            const int64_t node = (s_slot[e] >> 13) >> (6 * l);
            const double v = wave_total64(a.level[l - 1][node * 64 + lane]);
            if (lane == 63) {
              if (l == h && !a.top_computed) store_shared_level(a.level[l] + node, v);
              else a.level[l][node] = v;
            }
          }
          __syncthreads();
        }
      }
      stamp(5);
    }
  }
  stamp(6);
  if (a.nlevels < 2 || a.top_computed) return;  // readers compute the top (TreeView)
  // Count this workgroup finished once its level-h stores are released at agent scope (every
  // thread's own release fence, then the workgroup barrier, then a release increment), and
  // the last one acquires them (the increment's acquire side and an agent-scope acquire fence
  // in every thread) before it rescans the top level (a waitcnt is no fence).
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (tid == 0)
    s_last = __hip_atomic_fetch_add(a.done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
             (uint32_t)(G - 1);
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const int top = a.nlevels - 1;
  for (int64_t node = wave; node < a.top_nodes; node += nw) {
    const double c = __hip_atomic_load(a.level[top - 1] + node * 64 + lane, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    const double v = wave_total64(c);
    if (lane == 63) a.level[top][node] = v;
  }
  if (tid == 0) __hip_atomic_store(a.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}



__global__ void fill_i32_kernel(int32_t* p, int64_t n, int32_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// Synthetic item generator (bench / tests): Philox stream per 16-B chunk.
__device__ __forceinline__ u32x4 fill_rand(uint64_t seed, uint64_t item, uint32_t chunk,
                                          uint32_t field) {
  u32x4 c = {chunk, (uint32_t)item, (uint32_t)(item >> 32) ^ (field << 24), kFillTag};
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

__global__ void __launch_bounds__(256) fill_bytes_kernel(uint8_t* __restrict__ field,
                                                         int64_t row_bytes, int64_t capacity,
                                                         int64_t first_key, int64_t n,
                                                         uint64_t seed, uint32_t field_id) {
  const int64_t nvec = row_bytes >> 4;
  const int64_t total = n * nvec;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t item = i / nvec, v = i - item * nvec;
    const int64_t key = first_key + item;
    const int64_t slot = key % capacity;
    const u32x4 r = fill_rand(seed, (uint64_t)key, (uint32_t)v, field_id);
    uint4 w = {r.x, r.y, r.z, r.w};
    reinterpret_cast<uint4*>(field + slot * row_bytes)[v] = w;
  }
}

__global__ void fill_f32_normal_kernel(float* __restrict__ field, int64_t row_floats,
                                       int64_t capacity, int64_t first_key, int64_t n,
                                       uint64_t seed, uint32_t field_id, float lo, float hi,
                                       int uniform) {
  const int64_t total = n * row_floats;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t item = i / row_floats, c = i - item * row_floats;
    const int64_t key = first_key + item;
    const u32x4 r = fill_rand(seed, (uint64_t)key, (uint32_t)c, field_id);
    const double u1 = u01_53(r.x, r.y), u2 = u01_53(r.z, r.w);
    float x;
    if (uniform) {
      x = lo + (hi - lo) * (float)u1;
    } else {
      x = (float)(sqrt(-2.0 * log(1.0 - u1)) * cos(6.283185307179586 * u2));
    }
    field[(key % capacity) * row_floats + c] = x;
  }
}

// Scalar fields of the synthetic transition (action, reward, discount) + keys/prio.
__global__ void fill_scalars_kernel(int32_t* __restrict__ action, float* __restrict__ reward,
                                    float* __restrict__ discount, int reward_uniform,
                                    float p_zero_discount, float nonzero_discount,
                                    int32_t num_actions, int64_t capacity, int64_t first_key,
                                    int64_t n, uint64_t seed, uint64_t* __restrict__ keys,
                                    double* __restrict__ raw_prio, double* __restrict__ leaves) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t key = first_key + i;
  const int64_t slot = key % capacity;
  const u32x4 r = fill_rand(seed, (uint64_t)key, 0xFFFFu, 0xFFu);
  if (action) action[slot] = (int32_t)(r.x % (uint32_t)num_actions);
  const double u1 = u01_53(r.y, r.z);
  const double u2 = u01_53(r.w, r.x);
  if (reward_uniform) {
    reward[slot] = (float)(5.0 * u1);
  } else {
    reward[slot] = (float)(sqrt(-2.0 * log(1.0 - u1)) * cos(6.283185307179586 * u2));
  }
  const double u3 = u01_53(r.z ^ 0x9E3779B9u, r.w ^ 0x7F4A7C15u);
  discount[slot] = u3 < (double)p_zero_discount ? 0.0f : nonzero_discount;
  keys[slot] = (uint64_t)key;
  raw_prio[slot] = 1.0;
  leaves[slot] = 1.0;
}

// Checkpoint restore: leaves from the restored raw priorities (zero past the live range).
__global__ void restore_leaves_kernel(const double* __restrict__ raw, double* __restrict__ leaves,
                                      int64_t live, int64_t n, int prioritized, double alpha) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  leaves[i] = i < live ? (prioritized ? det_pow_priority(raw[i], alpha) : 1.0) : 0.0;
}

// Recompute all internal levels over the slot range touched by an insert.
// The landing of a committed chunk: its device mirror's blocks (field rows, keys, raw
// priorities, leaf weights) copied into the table's ring slots, every block in at most two
// ring segments, in one launch of 4-byte words.
constexpr int kMaxScatterSegs = 2 * (ACME_MAX_FIELDS + 3);
struct ScatterSegs {
  const uint32_t* src[kMaxScatterSegs];
  uint32_t* dst[kMaxScatterSegs];
  int64_t end[kMaxScatterSegs];  // cumulative words
  int n;
};

__global__ void __launch_bounds__(256) stage_scatter_kernel(ScatterSegs s) {
  const int64_t total = s.end[s.n - 1];
  for (int64_t i = blockIdx.x * int64_t(256) + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * 256) {
    int k = 0;
    while (i >= s.end[k]) ++k;
    const int64_t w = i - (k ? s.end[k - 1] : 0);
    s.dst[k][w] = s.src[k][w];
  }
}

int refresh_range(acme_replay* r, int64_t first_key, int64_t n, hipStream_t st) {
  const int64_t C = r->cfg.capacity;
  if (n <= 0) return ACME_OK;
  if (n > C) {
    first_key += n - C;
    n = C;
  }
  const int64_t s0 = first_key % C;
  // Up to two contiguous slot segments.
  int64_t seg_begin[2] = {s0, 0};
  int64_t seg_len[2] = {std::min(n, C - s0), n - std::min(n, C - s0)};
  for (int l = 1; l < r->nlevels; ++l) {
    const int shift = 6 * l;
    for (int s = 0; s < 2; ++s) {
      if (seg_len[s] <= 0) continue;
      const int64_t nb = seg_begin[s] >> shift;
      const int64_t ne = (seg_begin[s] + seg_len[s] - 1) >> shift;
      const int64_t count = ne - nb + 1;
      level_update_kernel<<<(unsigned)ceil_div(count, 4), 256, 0, st>>>(
          r->levels[l - 1], r->levels[l], nb, count, nullptr, nullptr, 0);
      ACME_LAUNCH_CHECK();
    }
  }
  return ACME_OK;
}

// Records `st` as a stream that touched the table; the slot is created on first use.  With
// every slot taken, the oldest stream's work so far is fenced into the side stream now and
// its slot reused (a correct, slightly earlier fence).
int reader_slot(acme_replay* r, hipStream_t st, acme_replay::Reader** out) {
  for (int i = 0; i < r->nreaders; ++i)
    if (r->readers[i].s == st) {
      *out = &r->readers[i];
      return ACME_OK;
    }
  acme_replay::Reader* rd;
  if (r->nreaders < kMaxReaders) {
    rd = &r->readers[r->nreaders++];
    ACME_HIP_TRY(hipEventCreateWithFlags(&rd->ev, hipEventDisableTiming));
  } else {
    rd = &r->readers[0];
    if (rd->dirty) {
      ACME_HIP_TRY(hipEventRecord(rd->ev, rd->s));
      ACME_HIP_TRY(hipStreamWaitEvent(r->side, rd->ev, 0));
    }
    const hipEvent_t ev = rd->ev;
    std::memmove(&r->readers[0], &r->readers[1], sizeof(acme_replay::Reader) * (kMaxReaders - 1));
    rd = &r->readers[kMaxReaders - 1];
    rd->ev = ev;
  }
  rd->s = st;
  rd->waited = 0;
  rd->dirty = false;
  *out = rd;
  return ACME_OK;
}

// Prologue of every device operation on a caller stream: wait for the latest committed
// insert (once per stream per commit) and remember the stream for the next commit.
// size_out (optional): the table size this operation may use (items whose copies it waits for).
int order_after_inserts(acme_replay* r, hipStream_t st, int64_t* size_out = nullptr) {
  std::lock_guard<std::mutex> lock(r->order_mu);
  if (size_out) *size_out = std::min(r->inserted, r->cfg.capacity);
  if (!r->side) return ACME_OK;  // no host insert has run yet
  acme_replay::Reader* rd;
  int rc = reader_slot(r, st, &rd);
  if (rc != ACME_OK) return rc;
  if (rd->waited < r->insert_seq) {
    ACME_HIP_TRY(hipStreamWaitEvent(st, r->insert_event, 0));
    rd->waited = r->insert_seq;
  }
  rd->dirty = true;
  return ACME_OK;
}

// Issues pipe p's pending row copies now, on its stream (the caller holds r->mu).
int flush_pipe(acme_replay* r, acme_replay::Pipe& p) {
  if (!p.pending) return ACME_OK;
  p.pending = false;
  return acme_replay_gather(r, p.slots, p.batch, p.out, p.st);
}

// Before any operation that writes rows: every pipe's pending copies (the caller holds r->mu).
// A commit fences the copies' streams as readers; the setup-time writers (synthetic fill,
// checkpoint restore) pass wait = true and the host waits for the copies instead.
int flush_pipes(acme_replay* r, bool wait = false) {
  for (auto& p : r->pipes) {
    const bool had = p.pending;
    const int rc = flush_pipe(r, p);
    if (rc != ACME_OK) return rc;
    if (had && wait) ACME_HIP_TRY(hipStreamSynchronize(p.st));
  }
  return ACME_OK;
}

// Byte layout of a staging chunk of n items: each field's rows, then keys, raw priorities
// and leaf weights (8 B per item each), every block 256-B aligned.  Returns the chunk bytes.
int64_t stage_layout(const acme_replay_config& cfg, int64_t n, int64_t* off) {
  int64_t o = 0;
  for (int f = 0; f < cfg.num_fields; ++f) {
    off[f] = o;
    o += (n * cfg.field_bytes[f] + 255) / 256 * 256;
  }
  for (int k = 0; k < 3; ++k) {
    off[ACME_MAX_FIELDS + k] = o;
    o += (n * 8 + 255) / 256 * 256;
  }
  return o;
}

// Side stream, staging chunks and events, created on the first host insert.
int ensure_insert_path(acme_replay* r) {
  if (r->side) return ACME_OK;
  int64_t item = 0;
  for (int f = 0; f < r->cfg.num_fields; ++f) item += (r->cfg.field_bytes[f] + 255) / 256 * 256;
  item += 3 * 8;
  int64_t n = std::max<int64_t>(1, kStageBytes / std::max<int64_t>(item, 1));
  n = std::min(n, r->cfg.capacity);
  const int64_t off = stage_layout(r->cfg, n, r->stage_off);
  for (int c = 0; c < kStageChunks; ++c) {
    if (hipHostMalloc(reinterpret_cast<void**>(&r->stage[c]), off, hipHostMallocDefault) !=
        hipSuccess) {
      set_error("hipHostMalloc of a %lld-byte insert staging chunk failed", (long long)off);
      return ACME_ERR_OOM;
    }
    if (hipMalloc(reinterpret_cast<void**>(&r->stage_dev[c]), off) != hipSuccess) {
      set_error("hipMalloc of a %lld-byte insert staging mirror failed", (long long)off);
      return ACME_ERR_OOM;
    }
    ACME_HIP_TRY(hipEventCreateWithFlags(&r->stage_done[c], hipEventDisableTiming));
    ACME_HIP_TRY(hipEventCreateWithFlags(&r->stage_up[c], hipEventDisableTiming));
  }
  ACME_HIP_TRY(hipEventCreateWithFlags(&r->insert_event, hipEventDisableTiming));
  r->stage_items = n;
  ACME_HIP_TRY(hipStreamCreateWithFlags(&r->upload, hipStreamNonBlocking));
  ACME_HIP_TRY(hipStreamCreateWithFlags(&r->side, hipStreamNonBlocking));
  return ACME_OK;
}

// Next staging chunk, once the copies that last used it have completed.
int acquire_chunk(acme_replay* r, int* out) {
  const int c = r->stage_next;
  r->stage_next = (c + 1) % kStageChunks;
  if (r->stage_used[c]) ACME_HIP_TRY(hipEventSynchronize(r->stage_done[c]));
  *out = c;
  return ACME_OK;
}

// A pinned staging chunk: the table's ring (r->stage[c]) or an n-step writer's own.
struct Chunk {
  uint8_t* base;
  const int64_t* off;  // stage_layout offsets
  hipEvent_t done;     // recorded after the chunk's copies
  uint8_t* dev;        // its device mirror
  hipEvent_t up;       // recorded after the upload into the mirror
  int64_t cap;         // items the layout holds
};

Chunk ring_chunk(acme_replay* r, int c) {
  return {r->stage[c], r->stage_off, r->stage_done[c], r->stage_dev[c], r->stage_up[c],
          r->stage_items};
}

// Issues the n items staged in chunk ch: keys, raw priorities and leaf weights into the
// chunk; the chunk's used blocks uploaded (H2D, upload stream) into its device mirror with
// no ordering against the table's readers (the mirror is private); then on the side stream,
// fenced after the upload, `after` and every stream that touched the table, the landing
// (one scatter launch into the ring slots) and the tree refresh.  The fence thus holds only
// the few-microsecond landing, not the PCIe transfer, between the readers' earlier work and
// their next draw.  Caller holds r->mu.
//
// dev (optional): device rows of the n items; then the copies run on `after` itself (the
// caller's stream, which owns those buffers) instead of the side stream.  skip: keys
// consumed before these items (an over-capacity insert).
int commit_chunk(acme_replay* r, const Chunk& ch, int64_t n, const double* priorities,
                 uint64_t* out_keys, hipStream_t after, const void* const* dev = nullptr,
                 int64_t skip = 0) {
  const int64_t C = r->cfg.capacity;
  const int64_t first_key = r->inserted + skip;
  uint8_t* base = ch.base;
  uint64_t* hkeys = reinterpret_cast<uint64_t*>(base + ch.off[ACME_MAX_FIELDS]);
  double* hprio = reinterpret_cast<double*>(base + ch.off[ACME_MAX_FIELDS + 1]);
  double* hleaf = reinterpret_cast<double*>(base + ch.off[ACME_MAX_FIELDS + 2]);
  for (int64_t i = 0; i < n; ++i) {
    const double p = priorities ? priorities[i] : 1.0;
    if (!(p >= 0.0)) {
      set_error("priority %g at item %lld must be >= 0", p, (long long)i);
      return ACME_ERR_INVALID;
    }
    hkeys[i] = (uint64_t)(first_key + i);
    hprio[i] = p;
    hleaf[i] = r->cfg.sampler == ACME_SAMPLER_PRIORITIZED
                   ? det_pow_priority(p, r->cfg.priority_exponent)
                   : 1.0;
  }
  if (out_keys) std::memcpy(out_keys, hkeys, n * sizeof(uint64_t));
  const int frc = flush_pipes(r);
  if (frc != ACME_OK) return frc;
  {
    std::lock_guard<std::mutex> lock(r->order_mu);
    acme_replay::Reader* rd;
    int rc = reader_slot(r, after, &rd);
    if (rc != ACME_OK) return rc;
    hipStream_t st = dev ? after : r->side;
    if (dev) {  // the caller's stream first catches up with earlier host inserts
      if (rd->waited < r->insert_seq) ACME_HIP_TRY(hipStreamWaitEvent(st, r->insert_event, 0));
    } else {
      rd->dirty = true;  // the committing caller's own earlier work (e.g. frame uploads)
    }
    for (int i = 0; i < r->nreaders; ++i) {
      acme_replay::Reader& x = r->readers[i];
      if (!x.dirty || x.s == st) continue;
      ACME_HIP_TRY(hipEventRecord(x.ev, x.s));
      ACME_HIP_TRY(hipStreamWaitEvent(st, x.ev, 0));
      x.dirty = false;
    }
  }
  hipStream_t st = dev ? after : r->side;
  const int nf = r->cfg.num_fields;
  if (!dev) {
    // Upload: one copy when the chunk is full, else one per used block.
    const int64_t full = ch.off[ACME_MAX_FIELDS + 2] + n * 8;
    if (n == ch.cap) {
      ACME_HIP_TRY(hipMemcpyAsync(ch.dev, base, full, hipMemcpyHostToDevice, r->upload));
    } else {
      for (int f = 0; f < nf; ++f)
        ACME_HIP_TRY(hipMemcpyAsync(ch.dev + ch.off[f], base + ch.off[f],
                                    n * r->cfg.field_bytes[f], hipMemcpyHostToDevice,
                                    r->upload));
      for (int k = 0; k < 3; ++k)
        ACME_HIP_TRY(hipMemcpyAsync(ch.dev + ch.off[ACME_MAX_FIELDS + k],
                                    base + ch.off[ACME_MAX_FIELDS + k], n * 8,
                                    hipMemcpyHostToDevice, r->upload));
    }
    ACME_HIP_TRY(hipEventRecord(ch.up, r->upload));
    ACME_HIP_TRY(hipStreamWaitEvent(st, ch.up, 0));
  }
  ScatterSegs segs{};
  int64_t words = 0;
  auto seg = [&](const uint8_t* src, uint8_t* dst, int64_t bytes) {
    segs.src[segs.n] = reinterpret_cast<const uint32_t*>(src);
    segs.dst[segs.n] = reinterpret_cast<uint32_t*>(dst);
    words += bytes / 4;
    segs.end[segs.n++] = words;
  };
  int64_t done = 0;
  while (done < n) {
    const int64_t slot = (first_key + done) % C;
    const int64_t len = std::min(n - done, C - slot);
    for (int f = 0; f < nf; ++f) {
      const int64_t b = r->cfg.field_bytes[f];
      if (dev)
        ACME_HIP_TRY(hipMemcpyAsync(r->fields[f] + slot * b,
                                    static_cast<const uint8_t*>(dev[f]) + done * b, len * b,
                                    hipMemcpyDeviceToDevice, st));
      else
        seg(ch.dev + ch.off[f] + done * b, r->fields[f] + slot * b, len * b);
    }
    if (dev) {
      ACME_HIP_TRY(hipMemcpyAsync(r->keys + slot, hkeys + done, len * sizeof(uint64_t),
                                  hipMemcpyHostToDevice, st));
      ACME_HIP_TRY(hipMemcpyAsync(r->raw_prio + slot, hprio + done, len * sizeof(double),
                                  hipMemcpyHostToDevice, st));
      ACME_HIP_TRY(hipMemcpyAsync(r->levels[0] + slot, hleaf + done, len * sizeof(double),
                                  hipMemcpyHostToDevice, st));
    } else {
      const int64_t o = done * 8;
      seg(ch.dev + ch.off[ACME_MAX_FIELDS] + o, reinterpret_cast<uint8_t*>(r->keys + slot),
          len * 8);
      seg(ch.dev + ch.off[ACME_MAX_FIELDS + 1] + o,
          reinterpret_cast<uint8_t*>(r->raw_prio + slot), len * 8);
      seg(ch.dev + ch.off[ACME_MAX_FIELDS + 2] + o,
          reinterpret_cast<uint8_t*>(r->levels[0] + slot), len * 8);
    }
    done += len;
  }
  if (!dev) {
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(words, 256 * 4), 2048);
    stage_scatter_kernel<<<std::max(grid, 1u), 256, 0, st>>>(segs);
    ACME_LAUNCH_CHECK();
  }
  int rc = refresh_range(r, first_key, n, st);
  if (rc != ACME_OK) return rc;
  ACME_HIP_TRY(hipEventRecord(ch.done, st));
  {
    std::lock_guard<std::mutex> lock(r->order_mu);
    ACME_HIP_TRY(hipEventRecord(r->insert_event, st));
    r->insert_seq += 1;
    r->inserted += skip + n;
    if (dev) {  // the caller's stream is ordered after this insert already
      acme_replay::Reader* rd;
      int rc2 = reader_slot(r, st, &rd);
      if (rc2 != ACME_OK) return rc2;
      rd->waited = r->insert_seq;
      rd->dirty = true;
    }
  }
  return ACME_OK;
}

}  // namespace

extern "C" {

int acme_replay_create(const acme_replay_config* cfg, acme_replay** out) {
  ACME_CHECK_ARG(cfg && out, "null argument");
  ACME_CHECK_ARG(cfg->capacity > 0 && cfg->capacity < (int64_t(1) << 40),
                 "capacity must be in [1, 2^40), got %lld", (long long)cfg->capacity);
  ACME_CHECK_ARG(cfg->sampler == ACME_SAMPLER_UNIFORM || cfg->sampler == ACME_SAMPLER_PRIORITIZED,
                 "unknown sampler %d", cfg->sampler);
  ACME_CHECK_ARG(cfg->num_fields >= 0 && cfg->num_fields <= ACME_MAX_FIELDS,
                 "num_fields must be in [0, %d]", ACME_MAX_FIELDS);
  ACME_CHECK_ARG(cfg->priority_exponent >= 0.0, "priority_exponent must be >= 0");
  for (int f = 0; f < cfg->num_fields; ++f)
    ACME_CHECK_ARG(cfg->field_bytes[f] > 0 && cfg->field_bytes[f] % 4 == 0,
                   "field %d: bytes per item must be a positive multiple of 4", f);

  acme_replay* r = new acme_replay();
  r->cfg = *cfg;
  // Level sizes.
  int64_t s = ceil_div(cfg->capacity, 64) * 64;
  r->level_size[0] = s;
  r->nlevels = 1;
  while (s > 64) {
    s = ceil_div(s / 64, 64) * 64;
    r->level_size[r->nlevels++] = s;
  }
  auto fail = [&](const char* what) {
    acme_replay_destroy(r);
    set_error("hipMalloc failed for %s", what);
    return ACME_ERR_OOM;
  };
  for (int l = 0; l < r->nlevels; ++l) {
    if (hipMalloc(&r->levels[l], r->level_size[l] * sizeof(double)) != hipSuccess)
      return fail("sum tree");
    if (hipMemset(r->levels[l], 0, r->level_size[l] * sizeof(double)) != hipSuccess)
      return fail("sum tree memset");
  }
  if (hipMalloc(&r->raw_prio, cfg->capacity * sizeof(double)) != hipSuccess) return fail("prio");
  if (hipMalloc(&r->keys, cfg->capacity * sizeof(uint64_t)) != hipSuccess) return fail("keys");
  if (hipMalloc(&r->winner, cfg->capacity * sizeof(int32_t)) != hipSuccess) return fail("winner");
  if (hipMalloc(&r->upd_done, sizeof(uint32_t)) != hipSuccess ||
      hipMemset(r->upd_done, 0, sizeof(uint32_t)) != hipSuccess)
    return fail("update count");
  (void)hipMemset(r->raw_prio, 0, cfg->capacity * sizeof(double));
  // Keys of never-written slots must not match any real key: fill with all-ones.
  (void)hipMemset(r->keys, 0xFF, cfg->capacity * sizeof(uint64_t));
  fill_i32_kernel<<<(unsigned)ceil_div(cfg->capacity, 256), 256>>>(r->winner, cfg->capacity, -1);
  for (int f = 0; f < cfg->num_fields; ++f) {
    if (hipMalloc(&r->fields[f], cfg->capacity * cfg->field_bytes[f]) != hipSuccess)
      return fail("field storage");
  }
  if (hipDeviceSynchronize() != hipSuccess) return fail("init sync");
  *out = r;
  return ACME_OK;
}

int acme_replay_destroy(acme_replay* r) {
  if (!r) return ACME_OK;
  (void)hipDeviceSynchronize();
  for (int l = 0; l < 8; ++l)
    if (r->levels[l]) (void)hipFree(r->levels[l]);
  if (r->raw_prio) (void)hipFree(r->raw_prio);
  if (r->keys) (void)hipFree(r->keys);
  if (r->winner) (void)hipFree(r->winner);
  if (r->upd_done) (void)hipFree(r->upd_done);
  if (r->upd_slots) (void)hipFree(r->upd_slots);
  if (r->upd_valid) (void)hipFree(r->upd_valid);
  for (int f = 0; f < ACME_MAX_FIELDS; ++f)
    if (r->fields[f]) (void)hipFree(r->fields[f]);
  for (int c = 0; c < kStageChunks; ++c) {
    if (r->stage[c]) (void)hipHostFree(r->stage[c]);
    if (r->stage_dev[c]) (void)hipFree(r->stage_dev[c]);
    if (r->stage_done[c]) (void)hipEventDestroy(r->stage_done[c]);
    if (r->stage_up[c]) (void)hipEventDestroy(r->stage_up[c]);
  }
  for (int i = 0; i < r->nreaders; ++i) (void)hipEventDestroy(r->readers[i].ev);
  for (auto& p : r->pipes)
    if (p.ev) (void)hipEventDestroy(p.ev);
  if (r->insert_event) (void)hipEventDestroy(r->insert_event);
  if (r->side) (void)hipStreamDestroy(r->side);
  if (r->upload) (void)hipStreamDestroy(r->upload);
  delete r;
  return ACME_OK;
}

int64_t acme_replay_size(const acme_replay* r) {
  if (!r) return 0;
  return std::min(r->inserted, r->cfg.capacity);
}

int64_t acme_replay_capacity(const acme_replay* r) { return r ? r->cfg.capacity : 0; }

int acme_replay_debug_leaves(const acme_replay* r, const double** leaf_values,
                             const double** raw_priorities, const uint64_t** keys) {
  ACME_CHECK_ARG(r, "null replay");
  if (leaf_values) *leaf_values = r->levels[0];
  if (raw_priorities) *raw_priorities = r->raw_prio;
  if (keys) *keys = r->keys;
  return ACME_OK;
}

int acme_replay_storage(acme_replay* r, int32_t field, void** out) {
  ACME_CHECK_ARG(r && out, "null argument");
  ACME_CHECK_ARG(field >= 0 && field < r->cfg.num_fields, "field %d out of range", field);
  {  // the caller may write rows through the pointer (checkpoint restore)
    std::lock_guard<std::mutex> lock(r->mu);
    const int rc = flush_pipes(r, true);
    if (rc != ACME_OK) return rc;
  }
  *out = r->fields[field];
  return ACME_OK;
}

int64_t acme_replay_inserted(const acme_replay* r) { return r ? r->inserted : 0; }

int acme_replay_restore(acme_replay* r, int64_t inserted, void* stream) {
  ACME_CHECK_ARG(r, "null replay");
  ACME_CHECK_ARG(inserted >= 0, "negative insert count");
  std::lock_guard<std::mutex> lock(r->mu);
  hipStream_t st = as_stream(stream);
  int rc = flush_pipes(r, true);
  if (rc != ACME_OK) return rc;
  rc = order_after_inserts(r, st);
  if (rc != ACME_OK) return rc;
  const int64_t C = r->cfg.capacity, live = std::min(inserted, C);
  const int64_t n = r->level_size[0];
  restore_leaves_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(
      r->raw_prio, r->levels[0], live, n, r->cfg.sampler == ACME_SAMPLER_PRIORITIZED,
      r->cfg.priority_exponent);
  ACME_LAUNCH_CHECK();
  for (int l = 1; l < r->nlevels; ++l) {  // every node of every level
    const int64_t count = r->level_size[l - 1] / 64;
    level_update_kernel<<<(unsigned)ceil_div(count, 4), 256, 0, st>>>(
        r->levels[l - 1], r->levels[l], 0, count, nullptr, nullptr, 0);
    ACME_LAUNCH_CHECK();
  }
  std::lock_guard<std::mutex> olock(r->order_mu);
  r->inserted = inserted;
  return ACME_OK;
}

int64_t acme_replay_stage_capacity(acme_replay* r) {
  if (!r) return 0;
  std::lock_guard<std::mutex> lock(r->mu);
  if (ensure_insert_path(r) != ACME_OK) return 0;
  return r->stage_items;
}

int acme_replay_stage(acme_replay* r, int64_t n, void** field_ptrs) {
  ACME_CHECK_ARG(r && field_ptrs, "null argument");
  std::unique_lock<std::mutex> lock(r->mu);
  int rc = ensure_insert_path(r);
  if (rc != ACME_OK) return rc;
  ACME_CHECK_ARG(n >= 1 && n <= r->stage_items, "stage: n = %lld must be in [1, %lld]",
                 (long long)n, (long long)r->stage_items);
  const std::thread::id me = std::this_thread::get_id();
  ACME_CHECK_ARG(r->staged < 0 || r->staged_by != me,
                 "stage: this thread's previously staged chunk was not committed");
  // Another writer thread's chunk is outstanding: wait for its commit.
  r->stage_cv.wait(lock, [r] { return r->staged < 0; });
  int c;
  rc = acquire_chunk(r, &c);
  if (rc != ACME_OK) return rc;
  for (int f = 0; f < r->cfg.num_fields; ++f) field_ptrs[f] = r->stage[c] + r->stage_off[f];
  r->staged = c;
  r->staged_n = n;
  r->staged_by = me;
  return ACME_OK;
}

int acme_replay_commit(acme_replay* r, int64_t n, const double* priorities, uint64_t* out_keys,
                       void* stream) {
  ACME_CHECK_ARG(r, "null replay");
  std::lock_guard<std::mutex> lock(r->mu);
  ACME_CHECK_ARG(r->staged >= 0 && r->staged_by == std::this_thread::get_id(),
                 "commit without a chunk staged by this thread");
  ACME_CHECK_ARG(n >= 0 && n <= r->staged_n, "commit: n = %lld exceeds the %lld staged items",
                 (long long)n, (long long)r->staged_n);
  const int c = r->staged;
  r->staged = -1;
  r->stage_cv.notify_all();
  if (n == 0) return ACME_OK;  // the chunk's last copies (if any) are still tracked
  const int rc = commit_chunk(r, ring_chunk(r, c), n, priorities,
                              out_keys, as_stream(stream));
  if (rc == ACME_OK) r->stage_used[c] = true;
  return rc;
}

int acme_host_register(void* p, int64_t bytes) {
  ACME_CHECK_ARG(p && bytes > 0, "bad host range");
  ACME_HIP_TRY(hipHostRegister(p, (size_t)bytes, hipHostRegisterDefault));
  return ACME_OK;
}

int acme_host_unregister(void* p) {
  ACME_CHECK_ARG(p, "null host pointer");
  ACME_HIP_TRY(hipHostUnregister(p));
  return ACME_OK;
}

int acme_replay_sync_inserts(acme_replay* r) {
  ACME_CHECK_ARG(r, "null replay");
  if (r->side) ACME_HIP_TRY(hipStreamSynchronize(r->side));
  return ACME_OK;
}

int acme_replay_insert(acme_replay* r, const void* const* fields, int64_t n,
                       const double* priorities, int32_t src_on_device, uint64_t* out_keys,
                       void* stream) {
  ACME_CHECK_ARG(r && (n == 0 || fields), "null argument");
  ACME_CHECK_ARG(n >= 0, "negative item count");
  if (n == 0) return ACME_OK;
  for (int64_t i = 0; priorities && i < n; ++i)
    ACME_CHECK_ARG(priorities[i] >= 0.0, "priority %g at item %lld must be >= 0", priorities[i],
                   (long long)i);
  std::unique_lock<std::mutex> lock(r->mu);
  int rc = ensure_insert_path(r);
  if (rc != ACME_OK) return rc;
  ACME_CHECK_ARG(r->staged < 0 || r->staged_by != std::this_thread::get_id(),
                 "insert while this thread's staged chunk is uncommitted");
  r->stage_cv.wait(lock, [r] { return r->staged < 0; });
  hipStream_t st = as_stream(stream);
  const int64_t C = r->cfg.capacity;
  // Only the last C items of an over-capacity insert survive: the first `skip` consume
  // their keys (reported in out_keys) but never land.
  const int64_t skip = n > C ? n - C : 0;
  if (out_keys)
    for (int64_t i = 0; i < skip; ++i) out_keys[i] = (uint64_t)(r->inserted + i);
  int64_t pending_skip = skip;
  for (int64_t done = skip; done < n;) {
    const int64_t len = std::min(n - done, r->stage_items);
    int c;
    rc = acquire_chunk(r, &c);
    if (rc != ACME_OK) return rc;
    const void* dev[ACME_MAX_FIELDS] = {};
    for (int f = 0; f < r->cfg.num_fields; ++f) {
      const int64_t b = r->cfg.field_bytes[f];
      const uint8_t* src = static_cast<const uint8_t*>(fields[f]) + done * b;
      if (src_on_device) dev[f] = src;  // HBM rows: copied on the caller's stream
      else std::memcpy(r->stage[c] + r->stage_off[f], src, len * b);  // pack into pinned
    }
    rc = commit_chunk(r, ring_chunk(r, c), len,
                      priorities ? priorities + done : nullptr,
                      out_keys ? out_keys + done : nullptr, st,
                      src_on_device ? dev : nullptr, pending_skip);
    if (rc != ACME_OK) return rc;
    r->stage_used[c] = true;
    pending_skip = 0;
    done += len;
  }
  return ACME_OK;
}

int acme_replay_fill_synthetic(acme_replay* r, int64_t n, int32_t layout, int32_t num_actions,
                               uint64_t seed, void* stream) {
  ACME_CHECK_ARG(r, "null replay");
  ACME_CHECK_ARG(n >= 0, "negative count");
  ACME_CHECK_ARG(layout == 0 || layout == 1, "unknown synthetic layout %d", layout);
  ACME_CHECK_ARG(r->cfg.num_fields == 5, "synthetic transitions need 5 fields");
  ACME_CHECK_ARG((layout == 1 || r->cfg.field_bytes[1] == 4) && r->cfg.field_bytes[2] == 4 &&
                     r->cfg.field_bytes[3] == 4,
                 "field layout does not match a transition (o, a, r, d, o_t)");
  ACME_CHECK_ARG(layout == 1 || num_actions > 0, "num_actions must be > 0");
  if (n == 0) return ACME_OK;
  std::lock_guard<std::mutex> lock(r->mu);
  hipStream_t st = as_stream(stream);
  int rc0 = flush_pipes(r, true);
  if (rc0 != ACME_OK) return rc0;
  rc0 = order_after_inserts(r, st);
  if (rc0 != ACME_OK) return rc0;
  const int64_t C = r->cfg.capacity;
  const int64_t first_key = r->inserted;
  int64_t skip = n > C ? n - C : 0;
  const int64_t k0 = first_key + skip, cnt = n - skip;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(cnt * 64, 256), 8192);
  if (layout == 0) {
    ACME_CHECK_ARG(r->cfg.field_bytes[0] % 16 == 0 && r->cfg.field_bytes[4] == r->cfg.field_bytes[0],
                   "Atari observation rows must be equal multiples of 16 bytes");
    for (int f : {0, 4}) {
      fill_bytes_kernel<<<grid, 256, 0, st>>>(r->fields[f], r->cfg.field_bytes[f], C, k0, cnt,
                                              seed, (uint32_t)f);
      ACME_LAUNCH_CHECK();
    }
    // Discount: 0.99^4 (n = 5 with agent discount applied n-1 times by the adder).
    const float d4 = 0.99f * 0.99f * 0.99f * 0.99f;
    fill_scalars_kernel<<<(unsigned)ceil_div(cnt, 256), 256, 0, st>>>(
        reinterpret_cast<int32_t*>(r->fields[1]), reinterpret_cast<float*>(r->fields[2]),
        reinterpret_cast<float*>(r->fields[3]), 0, 0.01f, d4, num_actions, C, k0, cnt, seed,
        r->keys, r->raw_prio, r->levels[0]);
    ACME_LAUNCH_CHECK();
  } else {
    fill_f32_normal_kernel<<<grid, 256, 0, st>>>(reinterpret_cast<float*>(r->fields[0]),
                                                 r->cfg.field_bytes[0] / 4, C, k0, cnt, seed, 0,
                                                 0.f, 0.f, 0);
    ACME_LAUNCH_CHECK();
    fill_f32_normal_kernel<<<grid, 256, 0, st>>>(reinterpret_cast<float*>(r->fields[1]),
                                                 r->cfg.field_bytes[1] / 4, C, k0, cnt, seed, 1,
                                                 -1.f, 1.f, 1);
    ACME_LAUNCH_CHECK();
    fill_f32_normal_kernel<<<grid, 256, 0, st>>>(reinterpret_cast<float*>(r->fields[4]),
                                                 r->cfg.field_bytes[4] / 4, C, k0, cnt, seed, 4,
                                                 0.f, 0.f, 0);
    ACME_LAUNCH_CHECK();
    const float d4 = 0.99f * 0.99f * 0.99f * 0.99f;
    fill_scalars_kernel<<<(unsigned)ceil_div(cnt, 256), 256, 0, st>>>(
        nullptr, reinterpret_cast<float*>(r->fields[2]), reinterpret_cast<float*>(r->fields[3]),
        1, 0.001f, d4, 1, C, k0, cnt, seed, r->keys, r->raw_prio, r->levels[0]);
    ACME_LAUNCH_CHECK();
  }
  int rc = refresh_range(r, k0, cnt, st);
  if (rc != ACME_OK) return rc;
  std::lock_guard<std::mutex> olock(r->order_mu);
  r->inserted += n;
  return ACME_OK;
}

static int sample_impl(acme_replay* r, int64_t batch, uint64_t step_counter, double prob_scale,
                       int64_t* slots, uint64_t* keys, double* probabilities,
                       int64_t* table_size, double* priorities, void* stream);
static int sample_gather_impl(acme_replay* r, int64_t batch, uint64_t step_counter,
                              double prob_scale, int64_t* slots, uint64_t* keys,
                              double* probabilities, int64_t* table_size, double* priorities,
                              void* const* out_fields, void* stream,
                              uint16_t* frames_f16 = nullptr);

int acme_replay_sample(acme_replay* r, int64_t batch, uint64_t step_counter, int64_t* slots,
                       uint64_t* keys, double* probabilities, int64_t* table_size,
                       double* priorities, void* stream) {
  return sample_impl(r, batch, step_counter, 1.0, slots, keys, probabilities, table_size,
                     priorities, stream);
}

int acme_replay_total(acme_replay* r, double* out, void* stream) {
  ACME_CHECK_ARG(r && out, "null argument");
  hipStream_t st = as_stream(stream);
  int64_t size = 0;
  int rc = order_after_inserts(r, st, &size);
  if (rc != ACME_OK) return rc;
  total_kernel<<<1, 64, 0, st>>>(tree_view(r), r->cfg.sampler == ACME_SAMPLER_PRIORITIZED,
                                 size, out);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int acme_replay_sample_share(acme_replay* r, int64_t batch, uint64_t step_counter,
                             double prob_scale, int64_t* slots, uint64_t* keys,
                             double* probabilities, int64_t* table_size, double* priorities,
                             void* const* out_fields, void* stream) {
  ACME_CHECK_ARG(r, "null replay");
  ACME_CHECK_ARG(prob_scale > 0.0 && prob_scale <= 1.0, "prob_scale must be in (0, 1]");
  std::lock_guard<std::mutex> lock(r->mu);  // no insert commits between draw and gather
  if (!out_fields)
    return sample_impl(r, batch, step_counter, prob_scale, slots, keys, probabilities,
                       table_size, priorities, stream);
  return sample_gather_impl(r, batch, step_counter, prob_scale, slots, keys, probabilities,
                            table_size, priorities, out_fields, stream);
}

int acme_replay_sample_share_frames(acme_replay* r, int64_t batch, uint64_t step_counter,
                                    double prob_scale, int64_t* slots, uint64_t* keys,
                                    double* probabilities, int64_t* table_size,
                                    double* priorities, void* const* out_fields,
                                    uint16_t* frames_f16, void* stream) {
  ACME_CHECK_ARG(r && out_fields && frames_f16, "null argument");
  ACME_CHECK_ARG(prob_scale > 0.0 && prob_scale <= 1.0, "prob_scale must be in (0, 1]");
  std::lock_guard<std::mutex> lock(r->mu);
  return sample_gather_impl(r, batch, step_counter, prob_scale, slots, keys, probabilities,
                            table_size, priorities, out_fields, stream, frames_f16);
}

static int sample_impl(acme_replay* r, int64_t batch, uint64_t step_counter, double prob_scale,
                       int64_t* slots, uint64_t* keys, double* probabilities,
                       int64_t* table_size, double* priorities, void* stream) {
  ACME_CHECK_ARG(r && slots, "null argument");
  ACME_CHECK_ARG(batch > 0 && batch <= (int64_t(1) << 31), "batch must be in [1, 2^31]");
  hipStream_t st = as_stream(stream);
  int64_t size = 0;
  int rc = order_after_inserts(r, st, &size);
  if (rc != ACME_OK) return rc;
  if (size <= 0) {
    set_error("cannot sample from an empty table (rate limiter MinSize(1))");
    return ACME_ERR_EMPTY;
  }
  ACME_PROF("replay_sample", st, 0.0, (double)batch * (r->cfg.sampler == ACME_SAMPLER_PRIORITIZED ? 512.0 * r->nlevels + 40.0 : 48.0));
  if (r->cfg.sampler == ACME_SAMPLER_PRIORITIZED) {
    const TreeView tv = tree_view(r);
    sample_prioritized_kernel<<<(unsigned)ceil_div(batch, 4), 256, 0, st>>>(
        tv, r->raw_prio, r->keys, batch, size, r->cfg.seed, step_counter, prob_scale, slots,
        keys, probabilities, table_size, priorities);
  } else {
    sample_uniform_kernel<<<(unsigned)ceil_div(batch, 256), 256, 0, st>>>(
        r->raw_prio, r->keys, batch, size, r->cfg.seed, step_counter, prob_scale, slots, keys,
        probabilities, table_size, priorities);
  }
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

// The transition layout (two big fields of equal bytes, multiples of 16, 16-B aligned
// destinations; every other field below 1 KiB): its big fields and the small ones.
static bool pair_layout(const acme_replay* r, void* const* out_fields, int* f0, int* f1,
                        SmallFields* sm) {
  int big[ACME_MAX_FIELDS], nbig = 0;
  for (int f = 0; f < r->cfg.num_fields; ++f)
    if (r->cfg.field_bytes[f] >= 1024) big[nbig++] = f;
  if (nbig != 2) return false;
  const int64_t nb = r->cfg.field_bytes[big[0]];
  if (nb != r->cfg.field_bytes[big[1]] || nb % 16 != 0 || nb / 16 > 1024 * 16) return false;
  for (int i = 0; i < 2; ++i)
    if (reinterpret_cast<uintptr_t>(out_fields[big[i]]) % 16 != 0) return false;
  *f0 = big[0];
  *f1 = big[1];
  *sm = SmallFields{};
  for (int f = 0; f < r->cfg.num_fields; ++f)
    if (f != big[0] && f != big[1]) {
      sm->src[sm->n] = r->fields[f];
      sm->dst[sm->n] = static_cast<uint8_t*>(out_fields[f]);
      sm->words[sm->n] = (int32_t)(r->cfg.field_bytes[f] / 4);
      sm->n++;
    }
  return true;
}

// Every field under 1 KB and a whole number of 4-byte words: the small-row fused path.
static bool small_layout(const acme_replay* r, void* const* out_fields, SmallFields* sm) {
  *sm = SmallFields{};
  for (int f = 0; f < r->cfg.num_fields; ++f) {
    if (r->cfg.field_bytes[f] >= 1024 || r->cfg.field_bytes[f] % 4 != 0 ||
        reinterpret_cast<uintptr_t>(out_fields[f]) % 4 != 0)
      return false;
    sm->src[sm->n] = r->fields[f];
    sm->dst[sm->n] = static_cast<uint8_t*>(out_fields[f]);
    sm->words[sm->n] = (int32_t)(r->cfg.field_bytes[f] / 4);
    sm->n++;
  }
  return sm->n > 0;
}

// Sample + gather as a unit (the caller holds r->mu): one fused launch for the transition
// layout and for rows of small fields, else the sampling kernel then the gather.
static int sample_gather_impl(acme_replay* r, int64_t batch, uint64_t step_counter,
                              double prob_scale, int64_t* slots, uint64_t* keys,
                              double* probabilities, int64_t* table_size, double* priorities,
                              void* const* out_fields, void* stream,
                              uint16_t* frames_f16) {
  ACME_CHECK_ARG(slots && out_fields, "null argument");
  ACME_CHECK_ARG(batch > 0 && batch < (int64_t(1) << 31), "bad batch");
  int f0, f1;
  SmallFields sm;
  const bool pair = pair_layout(r, out_fields, &f0, &f1, &sm);
  ACME_CHECK_ARG(!frames_f16 || (pair && reinterpret_cast<uintptr_t>(frames_f16) % 16 == 0),
                 "a bf16 frame copy needs the transition layout (two equal big fields) and a "
                 "16-byte aligned buffer");
  if (frames_f16 || pair) {
    hipStream_t st = as_stream(stream);
    int64_t size = 0;
    int rc = order_after_inserts(r, st, &size);
    if (rc != ACME_OK) return rc;
    if (size <= 0) {
      set_error("cannot sample from an empty table (rate limiter MinSize(1))");
      return ACME_ERR_EMPTY;
    }
    double row_bytes = 0;
    for (int k = 0; k < r->cfg.num_fields; ++k) row_bytes += (double)r->cfg.field_bytes[k];
    const bool prio = r->cfg.sampler == ACME_SAMPLER_PRIORITIZED;
    ACME_PROF("replay_sample_gather", st, 0.0,
              (double)batch * (2.0 * row_bytes + 40.0 + (prio ? 512.0 * r->nlevels : 0.0) +
                               (frames_f16 ? 4.0 * (double)r->cfg.field_bytes[f0] : 0.0)));
    const TreeView tv = tree_view(r);
    const int32_t nvec = (int32_t)(r->cfg.field_bytes[f0] / 16);
    const unsigned gb = (unsigned)batch;
    const uint8_t *s0 = r->fields[f0], *s1 = r->fields[f1];
    uint8_t* d0 = static_cast<uint8_t*>(out_fields[f0]);
    uint8_t* d1 = static_cast<uint8_t*>(out_fields[f1]);
#define ACME_SGP(PRIO, T, MAXC)                                                                 \
  sample_gather_pair_kernel<PRIO, T, MAXC><<<gb, T, 0, st>>>(                                   \
      tv, r->raw_prio, r->keys, size, r->cfg.seed, step_counter, prob_scale, slots, keys,       \
      probabilities, table_size, priorities, s0, s1, d0, d1, nvec, sm, frames_f16)
    if (2 * nvec <= 256 * 14) {
      if (prio) ACME_SGP(true, 256, 14);
      else ACME_SGP(false, 256, 14);
    } else {
      if (prio) ACME_SGP(true, 1024, 32);
      else ACME_SGP(false, 1024, 32);
    }
#undef ACME_SGP
    ACME_LAUNCH_CHECK();
    return ACME_OK;
  }
  if (!pair && small_layout(r, out_fields, &sm)) {
    hipStream_t st = as_stream(stream);
    int64_t size = 0;
    int rc = order_after_inserts(r, st, &size);
    if (rc != ACME_OK) return rc;
    if (size <= 0) {
      set_error("cannot sample from an empty table (rate limiter MinSize(1))");
      return ACME_ERR_EMPTY;
    }
    double row_bytes = 0;
    for (int k = 0; k < r->cfg.num_fields; ++k) row_bytes += (double)r->cfg.field_bytes[k];
    const bool prio = r->cfg.sampler == ACME_SAMPLER_PRIORITIZED;
    ACME_PROF("replay_sample_gather", st, 0.0,
              (double)batch * (2.0 * row_bytes + 40.0 + (prio ? 512.0 * r->nlevels : 0.0)));
    const TreeView tv = tree_view(r);
    const unsigned gb = (unsigned)ceil_div(batch, 4);
    if (prio)
      sample_gather_small_kernel<true><<<gb, 256, 0, st>>>(
          tv, r->raw_prio, r->keys, batch, size, r->cfg.seed, step_counter, prob_scale, slots,
          keys, probabilities, table_size, priorities, sm);
    else
      sample_gather_small_kernel<false><<<gb, 256, 0, st>>>(
          tv, r->raw_prio, r->keys, batch, size, r->cfg.seed, step_counter, prob_scale, slots,
          keys, probabilities, table_size, priorities, sm);
    ACME_LAUNCH_CHECK();
    return ACME_OK;
  }
  int rc = sample_impl(r, batch, step_counter, prob_scale, slots, keys, probabilities,
                       table_size, priorities, stream);
  if (rc != ACME_OK) return rc;
  return acme_replay_gather(r, slots, batch, out_fields, stream);
}

int acme_replay_gather(acme_replay* r, const int64_t* slots, int64_t batch,
                       void* const* out_fields, void* stream) {
  ACME_CHECK_ARG(r && slots && out_fields, "null argument");
  ACME_CHECK_ARG(batch > 0 && batch < (int64_t(1) << 31), "bad batch");
  hipStream_t st = as_stream(stream);
  int rc = order_after_inserts(r, st);
  if (rc != ACME_OK) return rc;
  GatherArgs g = {};
  for (int f = 0; f < r->cfg.num_fields; ++f) {
    g.src[f] = r->fields[f];
    g.dst[f] = static_cast<uint8_t*>(out_fields[f]);
    g.bytes[f] = r->cfg.field_bytes[f];
  }
  double row_bytes = 0;
  for (int k = 0; k < r->cfg.num_fields; ++k) row_bytes += (double)r->cfg.field_bytes[k];
  ACME_PROF("replay_gather", st, 0.0, 2.0 * row_bytes * (double)batch + 8.0 * (double)batch);
  // Pieces path: every field a multiple of 4 B (always: acme_replay_create checks it) and
  // 16-B aligned rows and buffers for the big fields.
  bool pieces = true;
  PieceArgs pa = {};
  int64_t total = 0;
  for (int f = 0; f < r->cfg.num_fields && pieces; ++f) {
    const int64_t nb = r->cfg.field_bytes[f];
    if (nb < 1024) continue;
    pieces = nb % 16 == 0 && reinterpret_cast<uintptr_t>(g.dst[f]) % 16 == 0;
    pa.big[pa.nbig] = f;
    pa.ppr[pa.nbig] = (int32_t)ceil_div(nb, 1024);
    pa.first[pa.nbig] = (int32_t)total;
    total += (int64_t)pa.ppr[pa.nbig] * batch;
    pa.nbig++;
  }
  pieces = pieces && total < (int64_t(1) << 30) && pa.nbig > 0;
  // Transition layout: exactly two big fields of equal bytes, the rest small.
  if (pieces && pa.nbig == 2 && r->cfg.field_bytes[pa.big[0]] == r->cfg.field_bytes[pa.big[1]]) {
    const int f0 = pa.big[0], f1 = pa.big[1];
    const int32_t nvec = (int32_t)(r->cfg.field_bytes[f0] / 16);
    SmallFields sm = {};
    for (int f = 0; f < r->cfg.num_fields; ++f)
      if (f != f0 && f != f1) {
        sm.src[sm.n] = g.src[f];
        sm.dst[sm.n] = g.dst[f];
        sm.words[sm.n] = (int32_t)(r->cfg.field_bytes[f] / 4);
        sm.n++;
      }
    const unsigned gb = (unsigned)batch;
    bool done = true;
    // Measured (tools/gather_bench.py, 1M-slot Atari table, B = 512): 256 threads x 14
    // chunks 12.05 us (4.80 TB/s), 1024 x 4 12.17 us, 512 x 7 12.45 us; plain loads instead
    // of non-temporal 12.85 us; the contiguous copy of the same bytes 11.2 us.
    if (2 * nvec <= 256 * 14)
      gather_pair_kernel<256, 14, true><<<gb, 256, 0, st>>>(g.src[f0], g.src[f1], g.dst[f0],
                                                             g.dst[f1], nvec, sm, slots);
    else if (2 * nvec <= 1024 * 16)
      gather_pair_kernel<1024, 16, true><<<gb, 1024, 0, st>>>(g.src[f0], g.src[f1], g.dst[f0],
                                                               g.dst[f1], nvec, sm, slots);
    else
      done = false;
    if (done) {
      ACME_LAUNCH_CHECK();
      return ACME_OK;
    }
  }
  if (pieces) {
    pa.first[pa.nbig] = (int32_t)total;
    for (int f = 0; f < r->cfg.num_fields; ++f) {
      pa.src[f] = g.src[f];
      pa.dst[f] = g.dst[f];
      pa.bytes[f] = (int32_t)r->cfg.field_bytes[f];
      if (r->cfg.field_bytes[f] < 1024) pa.big[pa.nbig + pa.nsmall++] = f;
    }
    constexpr int K = 8;
    const int gcap = 2048;
    const int64_t waves = std::max(ceil_div(total, K), (int64_t)pa.nsmall * ceil_div(batch, 64));
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(waves, 4), gcap));
    gather_pieces_kernel<K><<<grid, 256, 0, st>>>(pa, slots, (int32_t)batch);
    ACME_LAUNCH_CHECK();
    return ACME_OK;
  }
  gather_fields_kernel<<<dim3((unsigned)batch, (unsigned)r->cfg.num_fields), 256, 0, st>>>(g, slots);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

int acme_replay_sample_gather(acme_replay* r, int64_t batch, uint64_t step_counter,
                              int64_t* slots, uint64_t* keys, double* probabilities,
                              int64_t* table_size, double* priorities, void* const* out_fields,
                              void* stream) {
  ACME_CHECK_ARG(r, "null replay");
  std::lock_guard<std::mutex> lock(r->mu);  // no insert commits between draw and gather
  return sample_gather_impl(r, batch, step_counter, 1.0, slots, keys, probabilities, table_size,
                            priorities, out_fields, stream);
}

int acme_replay_sample_gather_frames(acme_replay* r, int64_t batch, uint64_t step_counter,
                                     int64_t* slots, uint64_t* keys, double* probabilities,
                                     int64_t* table_size, double* priorities,
                                     void* const* out_fields, uint16_t* frames_f16,
                                     void* stream) {
  ACME_CHECK_ARG(r && frames_f16, "null argument");
  std::lock_guard<std::mutex> lock(r->mu);
  return sample_gather_impl(r, batch, step_counter, 1.0, slots, keys, probabilities, table_size,
                            priorities, out_fields, stream, frames_f16);
}

int acme_replay_pipe_open(acme_replay* r, int32_t* pipe) {
  ACME_CHECK_ARG(r && pipe, "null argument");
  std::lock_guard<std::mutex> lock(r->mu);
  for (int i = 0; i < kMaxPipes; ++i)
    if (!r->pipes[i].open) {
      acme_replay::Pipe& p = r->pipes[i];
      if (!p.ev) ACME_HIP_TRY(hipEventCreateWithFlags(&p.ev, hipEventDisableTiming));
      const hipEvent_t ev = p.ev;  // kept across close / open
      p = acme_replay::Pipe{};
      p.ev = ev;
      p.open = true;
      *pipe = i;
      return ACME_OK;
    }
  set_error("all %d pipes of this table are open", kMaxPipes);
  return ACME_ERR_INVALID;
}

int acme_replay_pipe_close(acme_replay* r, int32_t pipe) {
  ACME_CHECK_ARG(r, "null replay");
  ACME_CHECK_ARG(pipe >= 0 && pipe < kMaxPipes, "pipe %d out of range", pipe);
  std::lock_guard<std::mutex> lock(r->mu);
  r->pipes[pipe].open = false;
  r->pipes[pipe].pending = false;
  return ACME_OK;
}

int acme_replay_pipe_flush(acme_replay* r, int32_t pipe) {
  ACME_CHECK_ARG(r, "null replay");
  ACME_CHECK_ARG(pipe >= 0 && pipe < kMaxPipes, "pipe %d out of range", pipe);
  std::lock_guard<std::mutex> lock(r->mu);
  ACME_CHECK_ARG(r->pipes[pipe].open, "pipe %d is not open", pipe);
  return flush_pipe(r, r->pipes[pipe]);
}

int acme_replay_sample_gather_pipe(acme_replay* r, int32_t pipe, int64_t batch,
                                   uint64_t step_counter, int64_t* slots, uint64_t* keys,
                                   double* probabilities, int64_t* table_size,
                                   double* priorities, void* const* out_fields, void* stream) {
  ACME_CHECK_ARG(r && slots && out_fields, "null argument");
  ACME_CHECK_ARG(pipe >= 0 && pipe < kMaxPipes, "pipe %d out of range", pipe);
  ACME_CHECK_ARG(batch > 0 && batch < (int64_t(1) << 31), "bad batch");
  std::lock_guard<std::mutex> lock(r->mu);
  acme_replay::Pipe& p = r->pipes[pipe];
  ACME_CHECK_ARG(p.open, "pipe %d is not open", pipe);
  hipStream_t st = as_stream(stream);
  int f0, f1;
  SmallFields sm;
  const bool pair = pair_layout(r, out_fields, &f0, &f1, &sm);
  const int32_t nvec = pair ? (int32_t)(r->cfg.field_bytes[f0] / 16) : 0;
  // The pending copy rides with this draw when it is this stream's and writes none of the
  // buffers this draw writes; otherwise it is issued on its own first.
  bool ride = p.pending && pair && p.st == st && p.slots != slots;
  for (int f = 0; ride && f < r->cfg.num_fields; ++f) ride = p.out[f] != out_fields[f];
  if (p.pending && !ride) {
    const hipStream_t old = p.st;
    const int rc = flush_pipe(r, p);
    if (rc != ACME_OK) return rc;
    if (old != st) {  // the batch is complete where this stream's later events are recorded
      ACME_HIP_TRY(hipEventRecord(p.ev, old));
      ACME_HIP_TRY(hipStreamWaitEvent(st, p.ev, 0));
    }
  }
  if (!pair || 2 * nvec > 192 * kPipeChunks) {  // no pipelining for this layout
    return sample_gather_impl(r, batch, step_counter, 1.0, slots, keys, probabilities,
                              table_size, priorities, out_fields, stream);
  }
  int64_t size = 0;
  int rc = order_after_inserts(r, st, &size);
  if (rc != ACME_OK) return rc;
  if (size <= 0) {
    set_error("cannot sample from an empty table (rate limiter MinSize(1))");
    return ACME_ERR_EMPTY;
  }
  // The pending batch's outputs (same layout: the pipe only ever holds pair-layout batches).
  const int64_t pend = ride ? p.batch : 0;
  SmallFields psm = {};
  uint8_t *pd0 = nullptr, *pd1 = nullptr;
  if (ride) {
    void* po[ACME_MAX_FIELDS];
    for (int f = 0; f < r->cfg.num_fields; ++f) po[f] = p.out[f];
    int g0, g1;
    pair_layout(r, po, &g0, &g1, &psm);
    pd0 = static_cast<uint8_t*>(po[g0]);
    pd1 = static_cast<uint8_t*>(po[g1]);
  }
  double row_bytes = 0;
  for (int k = 0; k < r->cfg.num_fields; ++k) row_bytes += (double)r->cfg.field_bytes[k];
  const bool prio = r->cfg.sampler == ACME_SAMPLER_PRIORITIZED;
  ACME_PROF("replay_sample_gather", st, 0.0,
            (double)batch * (40.0 + (prio ? 512.0 * r->nlevels : 0.0)) +
                (double)pend * 2.0 * row_bytes);
  const TreeView tv = tree_view(r);
  const unsigned grid = (unsigned)std::max(batch, pend);
#define ACME_SGPIPE(PRIO)                                                                       \
  sample_gather_pipe_kernel<PRIO, kPipeChunks><<<grid, 256, 0, st>>>(                           \
      tv, r->raw_prio, r->keys, size, r->cfg.seed, step_counter, batch, slots, keys,            \
      probabilities, table_size, priorities, ride ? p.slots : nullptr, pend, r->fields[f0],     \
      r->fields[f1], pd0, pd1, nvec, psm)
  if (prio) ACME_SGPIPE(true);
  else ACME_SGPIPE(false);
#undef ACME_SGPIPE
  ACME_LAUNCH_CHECK();
  p.pending = true;
  p.st = st;
  p.batch = batch;
  p.slots = slots;
  for (int f = 0; f < ACME_MAX_FIELDS; ++f) p.out[f] = f < r->cfg.num_fields ? out_fields[f] : nullptr;
  return ACME_OK;
}

}  // extern "C"

int acme::replay_update_priorities_gated(acme_replay* r, const uint64_t* keys,
                                         const double* prios, int64_t n, const Gate& gate,
                                         hipStream_t st, const RescaleJob* job) {
  ACME_CHECK_ARG(r && (n == 0 || (keys && prios)), "null argument");
  ACME_CHECK_ARG(n >= 0 && n < (int64_t(1) << 31), "bad update count");
  Gate eff = gate;
  if (n == 0 || n > kFusedUpdateMax) {  // the job as its own launch
    if (job && job->s) {
      const int rc = launch_rescale_job(*job, st);
      if (rc != ACME_OK) return rc;
      if (job->rg.g && job->rg.mode == kRgStep) {  // its verdict, as Adam reads it
        eff = Gate{};
        eff.g = job->rg.g;
        eff.use_last = 1;
      }
    }
    if (n == 0) return ACME_OK;
  }
  std::lock_guard<std::mutex> lock(r->mu);
  int rc = order_after_inserts(r, st);
  if (rc != ACME_OK) return rc;
  // Scratch for resolved slots / validity (grown on demand; growth drains the device).
  if (n > r->upd_cap) {
    if (r->upd_slots) {
      ACME_HIP_TRY(hipDeviceSynchronize());
      (void)hipFree(r->upd_slots);
      (void)hipFree(r->upd_valid);
    }
    r->upd_cap = std::max<int64_t>(n, 4096);
    ACME_HIP_TRY(hipMalloc(&r->upd_slots, r->upd_cap * sizeof(int64_t)));
    ACME_HIP_TRY(hipMalloc(&r->upd_valid, r->upd_cap * sizeof(int32_t)));
  }
  int64_t* t_slots = r->upd_slots;
  int32_t* t_valid = r->upd_valid;
  const unsigned g = (unsigned)ceil_div(n, 256);
  const double alpha =
      r->cfg.sampler == ACME_SAMPLER_PRIORITIZED ? r->cfg.priority_exponent : 0.0;
  ACME_PROF("replay_update", st, 0.0, (double)n * (16.0 + 8.0 * 3 + 512.0 * (r->nlevels - 1)));
  if (n <= kFusedUpdateMax) {
    FusedUpdateArgs a;
    a.upd_keys = keys; a.prios = prios; a.n = (int)n; a.capacity = r->cfg.capacity;
    a.keys = r->keys; a.alpha = alpha; a.raw_prio = r->raw_prio; a.nlevels = r->nlevels;
    a.gate = gate;
    if (job) a.job = *job;
    for (int l = 0; l < 8; ++l) a.level[l] = r->levels[l];
    a.top_nodes = r->nlevels >= 2 ? r->level_size[r->nlevels - 2] / 64 : 0;
    a.top_computed = computed_top_nodes(r) > 0 ? 1 : 0;
    a.done = r->upd_done;
    a.stamps = g_update_stamps;
    const unsigned blocks = kFusedUpdateBlocks + (a.job.s ? 1 : 0);
    if (n <= 2 * 256) prio_update_fused_kernel<2><<<blocks, 256, 0, st>>>(a);
    else prio_update_fused_kernel<kFusedUpdateMax / 256><<<blocks, 256, 0, st>>>(a);
    ACME_LAUNCH_CHECK();
    return ACME_OK;
  }
  prio_resolve_kernel<<<g, 256, 0, st>>>(keys, n, r->keys, r->cfg.capacity, t_slots, t_valid,
                                         r->winner);
  ACME_LAUNCH_CHECK();
  prio_write_kernel<<<g, 256, 0, st>>>(prios, n, t_slots, t_valid, r->winner, alpha,
                                       r->raw_prio, r->levels[0], eff);
  ACME_LAUNCH_CHECK();
  for (int l = 1; l < r->nlevels; ++l) {
    level_update_kernel<<<(unsigned)ceil_div(n, 4), 256, 0, st>>>(
        r->levels[l - 1], r->levels[l], 0, n, t_slots, t_valid, 6 * l);
    ACME_LAUNCH_CHECK();
  }
  prio_reset_kernel<<<g, 256, 0, st>>>(t_slots, t_valid, n, r->winner);
  ACME_LAUNCH_CHECK();
  return ACME_OK;
}

extern "C" {

int acme_replay_update_priorities(acme_replay* r, const uint64_t* keys, const double* prios,
                                  int64_t n, void* stream) {
  return replay_update_priorities_gated(r, keys, prios, n, Gate{}, as_stream(stream));
}

int acme_replay_update_priorities_gated(acme_replay* r, const uint64_t* keys, const double* prios,
                                        int64_t n, const uint32_t* skip_word, void* stream) {
  // skip_word (a learner's acme_dqn_skip_word): the update is dropped when it is non-zero on
  // the device when the update runs.
  Gate q;
  if (skip_word) {
    q.g = reinterpret_cast<const StepGuard*>(reinterpret_cast<const char*>(skip_word) -
                                             offsetof(StepGuard, last));
    q.use_last = 1;
  }
  return replay_update_priorities_gated(r, keys, prios, n, q, as_stream(stream));
}

}  // extern "C"

// ---------------------------------------------------------------- n-step transition writer
// The native side of NStepTransitionAdder (acme/adders/reverb/transition.py:119-165) for a
// transition table (o_tm1, a, R, D, o_t): the adder hands over each environment step's raw
// fields and the writer keeps the last n steps (its own copies of their observations), forms
// every item the reference writes (head = oldest step of the window; shorter windows at the
// start of an episode and, on the last step, the drain of shrinking windows) straight into
// rows of its own pinned chunk and commits a full chunk like acme_replay_commit.  No Python
// work per field and one copy of each observation into the window plus one per row.
//
// The return and discount accumulate in f32 in the reference's order (the adder's numpy
// float32 scalars: total_discount *= g; ret += r_i * total_discount; total_discount *= d_i),
// each product and sum rounded on its own (no contraction).
struct acme_nstep_writer {
  acme_replay* r = nullptr;
  int n = 1;
  float g = 1.0f;
  int64_t obs_bytes = 0, act_bytes = 0;  // payload bytes of o and a (rows may be padded)
  int64_t rows = 0;                     // rows per chunk
  int64_t off[ACME_MAX_FIELDS + 3] = {};
  uint8_t* chunk[2] = {};
  uint8_t* mirror[2] = {};
  hipEvent_t done[2] = {}, up[2] = {};
  bool used[2] = {};
  int cur = 0;
  int64_t fill = 0;
  std::vector<double> prio;
  // Window: steps [lo, steps) of the current episode; observation k (before step k) in
  // obs slot k % (n + 1), step k's action / reward / discount in slot k % (n + 1).
  std::vector<uint8_t> obs, act;
  std::vector<float> rew, disc;
  int64_t lo = 0, steps = 0;
  bool started = false;
  std::mutex mu;
};

namespace {

int nstep_commit(acme_nstep_writer* w) {
  if (w->fill == 0) return ACME_OK;
  acme_replay* r = w->r;
  std::lock_guard<std::mutex> lock(r->mu);
  int rc = ensure_insert_path(r);
  if (rc != ACME_OK) return rc;
  const int c = w->cur;
  rc = commit_chunk(r, {w->chunk[c], w->off, w->done[c], w->mirror[c], w->up[c], w->rows}, w->fill,
                    w->prio.data(), nullptr, nullptr);
  if (rc != ACME_OK) return rc;
  w->used[c] = true;
  w->cur = c ^ 1;
  w->fill = 0;
  return ACME_OK;
}

// One item: head step `lo`, window [lo, hi), next observation hi.
int nstep_emit(acme_nstep_writer* w, int64_t lo, int64_t hi, double priority) {
#pragma clang fp contract(off)
  const int64_t m = w->n + 1;
  if (w->fill == 0 && w->used[w->cur]) ACME_HIP_TRY(hipEventSynchronize(w->done[w->cur]));
  float ret = w->rew[lo % m], dsc = w->disc[lo % m];
  for (int64_t k = lo + 1; k < hi; ++k) {
    dsc = dsc * w->g;
    ret = ret + w->rew[k % m] * dsc;
    dsc = dsc * w->disc[k % m];
  }
  const auto& fb = w->r->cfg.field_bytes;
  uint8_t* base = w->chunk[w->cur];
  const int64_t i = w->fill;
  std::memcpy(base + w->off[0] + i * fb[0], w->obs.data() + (lo % m) * w->obs_bytes, w->obs_bytes);
  std::memcpy(base + w->off[1] + i * fb[1], w->act.data() + (lo % m) * w->act_bytes, w->act_bytes);
  std::memcpy(base + w->off[2] + i * fb[2], &ret, 4);
  std::memcpy(base + w->off[3] + i * fb[3], &dsc, 4);
  std::memcpy(base + w->off[4] + i * fb[4], w->obs.data() + (hi % m) * w->obs_bytes, w->obs_bytes);
  w->prio[i] = priority;
  w->fill = i + 1;
  return w->fill == w->rows ? nstep_commit(w) : ACME_OK;
}

}  // namespace

extern "C" {

int acme_nstep_writer_create(acme_replay* r, int32_t n_step, float discount, int64_t obs_bytes,
                             int64_t action_bytes, int64_t rows_per_chunk,
                             acme_nstep_writer** out) {
  ACME_CHECK_ARG(r && out, "null argument");
  ACME_CHECK_ARG(n_step >= 1, "n_step must be >= 1, got %d", n_step);
  ACME_CHECK_ARG(rows_per_chunk >= 1, "rows_per_chunk must be >= 1");
  const auto& cfg = r->cfg;
  ACME_CHECK_ARG(cfg.num_fields == 5 && cfg.field_bytes[2] == 4 && cfg.field_bytes[3] == 4 &&
                     cfg.field_bytes[0] == cfg.field_bytes[4],
                 "table is not a transition table (o_tm1, a, f32 r, f32 d, o_t)");
  ACME_CHECK_ARG(obs_bytes >= 1 && obs_bytes <= cfg.field_bytes[0] && action_bytes >= 1 &&
                     action_bytes <= cfg.field_bytes[1],
                 "observation / action bytes do not fit the table's rows");
  auto* w = new acme_nstep_writer();
  w->r = r;
  w->n = n_step;
  w->g = discount;
  w->obs_bytes = obs_bytes;
  w->act_bytes = action_bytes;
  w->rows = std::min<int64_t>(rows_per_chunk, cfg.capacity);
  const int64_t bytes = stage_layout(cfg, w->rows, w->off);
  for (int c = 0; c < 2; ++c) {
    if (hipHostMalloc(reinterpret_cast<void**>(&w->chunk[c]), bytes, hipHostMallocDefault) !=
            hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&w->mirror[c]), bytes) != hipSuccess ||
        hipEventCreateWithFlags(&w->done[c], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&w->up[c], hipEventDisableTiming) != hipSuccess) {
      acme_nstep_writer_destroy(w);
      set_error("n-step writer: pinned chunk of %lld bytes", (long long)bytes);
      return ACME_ERR_OOM;
    }
    std::memset(w->chunk[c], 0, bytes);  // row padding stays zero
  }
  w->prio.assign(w->rows, 1.0);
  w->obs.assign((n_step + 1) * obs_bytes, 0);
  w->act.assign((n_step + 1) * action_bytes, 0);
  w->rew.assign(n_step + 1, 0.0f);
  w->disc.assign(n_step + 1, 0.0f);
  *out = w;
  return ACME_OK;
}

int acme_nstep_writer_destroy(acme_nstep_writer* w) {
  if (!w) return ACME_OK;
  for (int c = 0; c < 2; ++c) {
    if (w->done[c]) {
      if (w->used[c]) (void)hipEventSynchronize(w->done[c]);
      (void)hipEventDestroy(w->done[c]);
    }
    if (w->up[c]) (void)hipEventDestroy(w->up[c]);
    if (w->chunk[c]) (void)hipHostFree(w->chunk[c]);
    if (w->mirror[c]) (void)hipFree(w->mirror[c]);
  }
  delete w;
  return ACME_OK;
}

int acme_nstep_writer_start(acme_nstep_writer* w, const void* observation) {
  ACME_CHECK_ARG(w && observation, "null argument");
  std::lock_guard<std::mutex> lock(w->mu);
  w->lo = w->steps = 0;
  std::memcpy(w->obs.data(), observation, w->obs_bytes);
  w->started = true;
  return ACME_OK;
}

int acme_nstep_writer_add(acme_nstep_writer* w, const void* action, float reward,
                          float discount, const void* next_observation, int32_t last,
                          double priority) {
  ACME_CHECK_ARG(w && action && next_observation, "null argument");
  ACME_CHECK_ARG(priority >= 0.0, "priority %g must be >= 0", priority);
  std::lock_guard<std::mutex> lock(w->mu);
  ACME_CHECK_ARG(w->started, "add before start (adder.add_first)");
  const int64_t m = w->n + 1, s = w->steps;
  std::memcpy(w->act.data() + (s % m) * w->act_bytes, action, w->act_bytes);
  w->rew[s % m] = reward;
  w->disc[s % m] = discount;
  w->steps = s + 1;
  w->lo = std::max<int64_t>(w->lo, w->steps - w->n);
  std::memcpy(w->obs.data() + (w->steps % m) * w->obs_bytes, next_observation, w->obs_bytes);
  int rc = nstep_emit(w, w->lo, w->steps, priority);
  if (rc != ACME_OK) return rc;
  if (last) {  // the drain of transition.py:167-172
    for (int64_t k = w->lo + 1; k < w->steps; ++k) {
      rc = nstep_emit(w, k, w->steps, priority);
      if (rc != ACME_OK) return rc;
    }
    w->started = false;
  }
  return ACME_OK;
}

int acme_nstep_writer_flush(acme_nstep_writer* w) {
  ACME_CHECK_ARG(w, "null writer");
  std::lock_guard<std::mutex> lock(w->mu);
  return nstep_commit(w);
}

int acme_nstep_writer_reset(acme_nstep_writer* w) {
  ACME_CHECK_ARG(w, "null writer");
  std::lock_guard<std::mutex> lock(w->mu);
  w->started = false;
  w->lo = w->steps = 0;
  return nstep_commit(w);
}

int64_t acme_nstep_writer_pending(acme_nstep_writer* w) {
  if (!w) return 0;
  std::lock_guard<std::mutex> lock(w->mu);
  return w->fill;
}

}  // extern "C"
