// fp32 MFMA GEMM engine for the learner's dense layers (gfx950 / CDNA4).
//
// C[BM x BN tile] = sum_k A[m][k] * B[n][k], with A and B supplied by "problem" loaders
// that synthesise implicit-GEMM operands on the fly (im2col for convolution forward,
// transposed im2col for weight gradients, strided gather for input gradients), so no
// im2col matrix ever touches HBM.
//
// Arithmetic: v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulate; gfx950 has
// no xf32).  The reference learner is fp32, and parity is
// 1e-5 rtol, so the dense layers stay in f32.
//
// Tiling: 64*WM*WN threads; each wave owns a (BM/WM) x (BN/WN) output sub-tile made of
// 32x32 MFMA tiles.  BK (16 or 32) reduction elements per stage, two LDS stages (one
// barrier per stage), global->register prefetch of stage k+1 overlapping the MFMAs of
// stage k.
//
// LDS image: a lane (r = lane & 31, h = lane >> 5) fetches 4 consecutive k of its row
// with one ds_read_b128 and feeds them to four consecutive MFMAs (physical k =
// 8q + 4h + t at MFMA step t); A and B use the same k permutation, so the sum over k
// is unchanged.  Two row layouts, chosen per operand by how its loader delivers data:
//   * k-contiguous operands (loader returns 4 consecutive k, stored with ds_write_b128):
//     unpadded rows of BK floats with the 16-B chunks XOR-swizzled by the row,
//     chunk' = chunk ^ s(row), s = (row >> 2) & 3 (BK 16) or (row >> 1) & 7 (BK 32).
//     Conflict-free for both the b128 stores and the b128 fragment reads (checked
//     exhaustively against the LDS lane-group table of MI355X_MICROARCH.md).  The padded
//     layout it replaces had 2-way store conflicts (20-35% of LDS cycles, PMC).
//   * row-contiguous operands (loader returns 4 consecutive rows, stored with
//     ds_write_b32): rows of BK + 4 floats, conflict-free for b32 stores and b128 reads.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace acme {
namespace gemm {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;

// Operand global-memory orientation.
//   KCONTIG: the loader returns A[row][k .. k+3] (4 consecutive reduction elements).
//   RCONTIG: the loader returns A[row .. row+3][k] (4 consecutive rows).
enum OperandMode { KCONTIG = 0, RCONTIG = 1 };

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

template <int BK>
__device__ __forceinline__ int kswz(int row) {
  return BK == 16 ? ((row >> 2) & 3) : ((row >> 1) & 7);
}

// Per-thread slots and LDS image of an operand tile of R rows x BK.
template <int R, int NT, int MODE, int BK>
struct OperandPlan {
  static constexpr int CH = BK / 4;                 // 16-B chunks per row
  static constexpr int STRIDE = MODE == KCONTIG ? BK : BK + 4;
  static constexpr int FLOATS = R * STRIDE;         // one LDS stage
  static constexpr int VECS = R * BK / 4;           // float4 vectors per tile
  static constexpr int PER_THREAD = (VECS + NT - 1) / NT;
  static_assert(VECS % NT == 0 || VECS < NT, "tile vectors must divide evenly over the threads");
  // Thread tid owns vectors tid + i*NT; when the tile has fewer vectors than threads the
  // surplus threads own none.
  __device__ static __forceinline__ bool owns(int v) { return VECS >= NT || v < VECS; }
  // KCONTIG: vector v -> (row v / CH, kk 4*(v % CH)).  RCONTIG: v -> (row 4*(v / BK), kk v % BK).
  __device__ static __forceinline__ int row_of(int v) {
    return MODE == KCONTIG ? (v / CH) : ((v / BK) << 2);
  }
  __device__ static __forceinline__ int kk_of(int v) {
    return MODE == KCONTIG ? ((v % CH) << 2) : (v % BK);
  }
  __device__ static __forceinline__ void store(float* tile, int v, f32x4 x) {
    const int row = row_of(v);
    if (MODE == KCONTIG) {
      const int ch = (v % CH) ^ kswz<BK>(row);
      *reinterpret_cast<f32x4*>(&tile[row * STRIDE + 4 * ch]) = x;
    } else {
      const int kk = kk_of(v);
      tile[(row + 0) * STRIDE + kk] = x[0];
      tile[(row + 1) * STRIDE + kk] = x[1];
      tile[(row + 2) * STRIDE + kk] = x[2];
      tile[(row + 3) * STRIDE + kk] = x[3];
    }
  }
  // Fragment of 4 k values for row `row` (whose low 5 bits are the lane's r) and
  // logical chunk `c` (= 2q + h).
  __device__ static __forceinline__ f32x4 frag(const float* tile, int row, int c) {
    const int ch = MODE == KCONTIG ? (c ^ kswz<BK>(row)) : c;
    return *reinterpret_cast<const f32x4*>(&tile[row * STRIDE + 4 * ch]);
  }
};

// Optional column-sum hook: problems that define `static constexpr bool kColSum = true`
// get sum_k B[n][k] over their reduction range (bias gradients: B is the layer's dZ),
// accumulated from the LDS-resident B tiles by the blocks of the first M tile and
// delivered through p.store_colsum(n, value, split).
template <class P, class = void>
struct HasColSum {
  static constexpr bool value = false;
};
template <class P>
struct HasColSum<P, decltype(void(P::kColSum))> {
  static constexpr bool value = P::kColSum;
};

// Optional prefetched-epilogue hook: problems with `static constexpr bool kPreStore = true`
// supply p.pre(m, n), a value loaded for every output of the tile (clamped indices, no
// branch around the load), p.finish(v, pre) (arithmetic only) and p.put(m, n, value, split).
// The epilogue loads all of a lane's pre values, finishes every output, then stores: a load
// inside a per-element store (a bias, a ReLU mask) is otherwise waited for element by
// element, and behind the stores already issued (vmcnt counts both).
template <class P, class = void>
struct HasPreStore {
  static constexpr bool value = false;
};
template <class P>
struct HasPreStore<P, decltype(void(P::kPreStore))> {
  static constexpr bool value = P::kPreStore;
};

// Epilogue of the f32 / x6 engines: C/D map of the 32x32 MFMA, col = lane & 31,
// row = (v&3) + 8(v>>2) + 4h, for the wave tile at (mb, nb).
template <int MT, int NTL, class P>
__device__ __forceinline__ void store_tile(const P& p, const f32x16 (&acc)[MT][NTL], int mb,
                                           int nb, int h, int r, int split) {
  if constexpr (HasPreStore<P>::value) {
    float pre[MT][NTL][16];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NTL; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int m = mb + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
          const int n = nb + j * 32 + r;
          pre[i][j][v] = p.pre(m < p.M ? m : p.M - 1, n < p.N ? n : p.N - 1);
        }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NTL; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) pre[i][j][v] = p.finish(acc[i][j][v], pre[i][j][v]);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NTL; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int m = mb + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
          const int n = nb + j * 32 + r;
          if (m < p.M && n < p.N) p.put(m, n, pre[i][j][v], split);
        }
  } else {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NTL; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int m = mb + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
          const int n = nb + j * 32 + r;
          if (m < p.M && n < p.N) p.store(m, n, acc[i][j][v], split);
        }
  }
}

// Optional z-class hook: problems with `static constexpr bool kZClass = true` use
// blockIdx.z to select a sub-problem (p.for_z(z)) instead of a K split.
template <class P, class = void>
struct HasZClass {
  static constexpr bool value = false;
};
template <class P>
struct HasZClass<P, decltype(void(P::kZClass))> {
  static constexpr bool value = P::kZClass;
};
template <class P>
__device__ __forceinline__ P z_select(const P& p) {
  if constexpr (HasZClass<P>::value) return p.for_z(blockIdx.z);
  else return p;
}

// Several problems of one type in one launch (e.g. the online and target networks' same
// layer): blockIdx.z selects sub-problem z; the grid covers the largest M x N, and the tiles
// past a smaller problem's extent load zeros and store nothing.  Each sub-problem's outputs
// are computed exactly as by its own launch.
template <class Q, int NZ>
struct ZSet : Q {
  static constexpr bool kZClass = true;
  Q sub[NZ];
  __host__ __device__ ZSet for_z(int z) const {
    ZSet r = *this;
    static_cast<Q&>(r) = sub[z];
    return r;
  }
};

template <class Q, int NZ>
ZSet<Q, NZ> make_zset(const Q (&qs)[NZ]) {
  ZSet<Q, NZ> s;
  static_cast<Q&>(s) = qs[0];
  for (int i = 0; i < NZ; ++i) {
    s.sub[i] = qs[i];
    s.M = s.M > qs[i].M ? s.M : qs[i].M;
    s.N = s.N > qs[i].N ? s.N : qs[i].N;
  }
  return s;
}

// One operand as a single buffer for the direct engine's strided loads (gemm_direct.h):
// element (row, k) at byte offset row * row_bytes + k * k_bytes, `bytes` long.
struct StridedOp {
  const float* base;
  uint32_t bytes, row_bytes, k_bytes;
};

// Problem concept (see conv.h):
//   static constexpr int A_MODE, B_MODE;
//   int M, N, K;            rows of A (= C rows), rows of B (= C cols), reduction length
//   int k_chunk;            reduction elements per split (multiple of BK), K if no split
//   struct ARow; ARow a_row(int row) const;     f32x4 a_load(const ARow&, int k) const;
//   struct BRow; BRow b_row(int row) const;     f32x4 b_load(const BRow&, int k) const;
//   void store(int m, int n, float v, int split) const;
// The loaders must return zeros for rows >= M / N and k >= K.

// WK > 1 splits the reduction INSIDE the block: WK groups of WM x WN waves each take a
// contiguous share of the block's K range through their own LDS stages, and the partial
// accumulators are summed through LDS before the epilogue.  Small GEMMs (a few hundred
// rows, K <= 1024) use it to put 4x more waves on the same output tiles.
//
// LDS floats of one block: two stages per k-group, reused after the k loop for the k-group
// reduction: the accumulator partials, then the column-sum partials.
template <int BM, int BN, int WM, int WN, int BK, int WK, class P>
constexpr int gemm_smem_floats() {
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MT = TM / 32, NTL = TN / 32;
  constexpr int STAGE = OperandPlan<BM, 64 * WM * WN, P::A_MODE, BK>::FLOATS +
                        OperandPlan<BN, 64 * WM * WN, P::B_MODE, BK>::FLOATS;
  constexpr int STAGE_FLOATS = 2 * STAGE * WK;
  constexpr int RED_FLOATS = (WK - 1) * WM * WN * MT * NTL * 16 * 64;
  constexpr int RED_ALL = RED_FLOATS + (WK - 1) * BN;
  return STAGE_FLOATS > RED_ALL ? STAGE_FLOATS : RED_ALL;
}

// One output tile (`tile`, reduction split `split`) of problem p, LDS at `smem`
// (gemm_smem_floats<...>() floats).  Blocks whose tile lies past p's extent leave at once
// (block-uniform, before any barrier).
template <int BM, int BN, int WM, int WN, int BK, int WK, class P>
__device__ __forceinline__ void gemm_f32_block(const P& p, const int tile, const int split,
                                               float* __restrict__ smem) {
  constexpr int NTG = 64 * WM * WN;  // threads per k-group
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MT = TM / 32, NTL = TN / 32;
  static_assert(TM % 32 == 0 && TN % 32 == 0, "wave tile must be a multiple of 32x32");
  static_assert(BK == 16 || BK == 32, "BK must be 16 or 32");
  using PA = OperandPlan<BM, NTG, P::A_MODE, BK>;
  using PB = OperandPlan<BN, NTG, P::B_MODE, BK>;
  constexpr int STAGE = PA::FLOATS + PB::FLOATS;
  constexpr int STAGE_FLOATS = 2 * STAGE * WK;
  constexpr int RED_FLOATS = (WK - 1) * WM * WN * MT * NTL * 16 * 64;

  const int tid_all = threadIdx.x;
  const int grp = tid_all / NTG;
  const int tid = tid_all - grp * NTG;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int m0 = (tile / tiles_n) * BM;
  const int n0 = (tile % tiles_n) * BN;
  if (m0 >= p.M) return;
  int kbeg = split * p.k_chunk;
  int kend = kbeg + p.k_chunk;
  if (kend > p.K) kend = p.K;
  int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  int nk_all = nk;
  if constexpr (WK > 1) {
    const int per = (nk + WK - 1) / WK;  // stages per group
    nk_all = per;
    const int s0 = grp * per;
    const int s1 = s0 + per < nk ? s0 + per : nk;
    nk = s1 > s0 ? s1 - s0 : 0;
    kbeg += s0 * BK;
  }
  float* my = smem + grp * 2 * STAGE;
  typename P::ARow arow[PA::PER_THREAD];
  typename P::BRow brow[PB::PER_THREAD];
#pragma unroll
  for (int i = 0; i < PA::PER_THREAD; ++i)
    arow[i] = p.a_row(m0 + (PA::owns(tid + i * NTG) ? PA::row_of(tid + i * NTG) : 0));
#pragma unroll
  for (int i = 0; i < PB::PER_THREAD; ++i)
    brow[i] = p.b_row(n0 + (PB::owns(tid + i * NTG) ? PB::row_of(tid + i * NTG) : 0));

  f32x4 ra[PA::PER_THREAD], rb[PB::PER_THREAD];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < PA::PER_THREAD; ++i) {
      const int k = k0 + PA::kk_of(tid + i * NTG);
      ra[i] = (PA::owns(tid + i * NTG) && k < kend) ? p.a_load(arow[i], k) : zero4();
    }
#pragma unroll
    for (int i = 0; i < PB::PER_THREAD; ++i) {
      const int k = k0 + PB::kk_of(tid + i * NTG);
      rb[i] = (PB::owns(tid + i * NTG) && k < kend) ? p.b_load(brow[i], k) : zero4();
    }
  };
  auto stash = [&](int buf) {
    float* sa = my + buf * STAGE;
    float* sb = sa + PA::FLOATS;
#pragma unroll
    for (int i = 0; i < PA::PER_THREAD; ++i)
      if (PA::owns(tid + i * NTG)) PA::store(sa, tid + i * NTG, ra[i]);
#pragma unroll
    for (int i = 0; i < PB::PER_THREAD; ++i)
      if (PB::owns(tid + i * NTG)) PB::store(sb, tid + i * NTG, rb[i]);
  };

  f32x16 acc[MT][NTL];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  const int r = lane & 31, h = lane >> 5;
  constexpr bool kColSum = HasColSum<P>::value;
  const bool do_colsum = kColSum && m0 == 0 && tid < BN;
  float colsum = 0.f;
  if (nk > 0) {
    fetch(kbeg);
    stash(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk_all; ++kt) {
    const bool active = kt < nk;  // uniform per k-group
    const bool more = kt + 1 < nk;
    if (more) fetch(kbeg + (kt + 1) * BK);
    const float* sa = my + (kt & 1) * STAGE;
    const float* sb = sa + PA::FLOATS;
    if (active) {
      if constexpr (kColSum) {
        if (do_colsum) {
#pragma unroll
          for (int c = 0; c < BK / 4; ++c) {
            const f32x4 x = PB::frag(sb, tid, c);
            colsum += (x[0] + x[1]) + (x[2] + x[3]);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < BK / 8; ++q) {
        f32x4 af[MT], bf[NTL];
#pragma unroll
        for (int i = 0; i < MT; ++i) af[i] = PA::frag(sa, wm * TM + i * 32 + r, 2 * q + h);
#pragma unroll
        for (int j = 0; j < NTL; ++j) bf[j] = PB::frag(sb, wn * TN + j * 32 + r, 2 * q + h);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NTL; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][t], bf[j][t], acc[i][j], 0, 0, 0);
      }
    }
    if (more) stash((kt + 1) & 1);
    __syncthreads();
  }

  if constexpr (WK > 1) {
    // Sum the k-groups' accumulators into group 0 (fixed order: group 0 + 1 + 2 + ...).
    constexpr int PER_WAVE = MT * NTL * 16 * 64;
    float* cs_red = smem + RED_FLOATS;  // the stages are dead after the loop's last barrier
    if (grp > 0) {
      float* dst = smem + ((grp - 1) * WM * WN + wave) * PER_WAVE;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j)
#pragma unroll
          for (int v = 0; v < 16; ++v) dst[((i * NTL + j) * 16 + v) * 64 + lane] = acc[i][j][v];
      if constexpr (kColSum) {
        if (do_colsum) cs_red[(grp - 1) * BN + tid] = colsum;
      }
    }
    __syncthreads();
    if (grp > 0) return;
#pragma unroll
    for (int g = 1; g < WK; ++g) {
      const float* src = smem + ((g - 1) * WM * WN + wave) * PER_WAVE;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j)
#pragma unroll
          for (int v = 0; v < 16; ++v) acc[i][j][v] += src[((i * NTL + j) * 16 + v) * 64 + lane];
      if constexpr (kColSum) {
        if (do_colsum) colsum += cs_red[(g - 1) * BN + tid];
      }
    }
  }

  store_tile<MT, NTL>(p, acc, m0 + wm * TM, n0 + wn * TN, h, r, split);
  if constexpr (kColSum) {
    if (do_colsum && n0 + tid < p.N) p.store_colsum(n0 + tid, colsum, split);
  }
}


template <int BM, int BN, int WM, int WN, int BK, int WK, class P>
__global__ void __launch_bounds__(64 * WM * WN * WK) gemm_f32_kernel(const P p_in) {
  __shared__ __attribute__((aligned(16))) float smem[gemm_smem_floats<BM, BN, WM, WN, BK, WK, P>()];
  const P p = z_select(p_in);
  gemm_f32_block<BM, BN, WM, WN, BK, WK>(p, blockIdx.x, HasZClass<P>::value ? 0 : blockIdx.z, smem);
}

// Problems of different types in one launch: ZMulti<S0, S1, ...> holds one ZSet per type
// and its count n; blockIdx.z runs S0's sub-problems 0 .. n0-1, then S1's, and so on (the
// input and weight gradients of a layer, which read the same dZ and are independent).
// Each sub-problem's outputs are computed exactly as by its own launch.
template <class... S>
struct ZMulti;
template <>
struct ZMulti<> {};
template <class S0, class... R>
struct ZMulti<S0, R...> {
  S0 s;
  int n = 0;
  ZMulti<R...> rest;
};

template <int BM, int BN, int WM, int WN, int BK, int WK, class S0, class... R>
constexpr int zmulti_smem_floats() {
  constexpr int a = gemm_smem_floats<BM, BN, WM, WN, BK, WK, S0>();
  if constexpr (sizeof...(R) == 0) return a;
  else {
    constexpr int b = zmulti_smem_floats<BM, BN, WM, WN, BK, WK, R...>();
    return a > b ? a : b;
  }
}

template <int BM, int BN, int WM, int WN, int BK, int WK, class S0, class... R>
__device__ __forceinline__ void zmulti_run(const ZMulti<S0, R...>& q, int z, float* smem) {
  if (z < q.n) {
    const S0 p = q.s.for_z(z);
    gemm_f32_block<BM, BN, WM, WN, BK, WK>(p, blockIdx.x, 0, smem);
  } else if constexpr (sizeof...(R) > 0) {
    zmulti_run<BM, BN, WM, WN, BK, WK>(q.rest, z - q.n, smem);
  }
}

template <int BM, int BN, int WM, int WN, int BK, int WK, class... S>
__global__ void __launch_bounds__(64 * WM * WN * WK) gemm_f32_multi_kernel(const ZMulti<S...> q) {
  __shared__ __attribute__((aligned(16))) float smem[zmulti_smem_floats<BM, BN, WM, WN, BK, WK, S...>()];
  zmulti_run<BM, BN, WM, WN, BK, WK>(q, blockIdx.z, smem);
}

// The block size of every f32-engine launch is derived here from the kernel's own template
// parameters: a (BK, WK) build experiment in round 5 launched the multi kernel instantiated
// for WK = 4 (256 threads) with a hard-coded 512-thread block, so k-groups 4..7 indexed LDS
// and the reduction buffers of groups that do not exist ("unspecified launch failure",
// VERDICT r5 item 4).  The LDS of a block must also fit the CU's 160 KB.
template <int BM, int BN, int WM, int WN, int BK, int WK>
constexpr int gemm_threads() {
  static_assert(64 * WM * WN * WK <= 1024, "at most 1024 threads per block");
  return 64 * WM * WN * WK;
}

template <int BM, int BN, int WM, int WN, int BK = 16, int WK = 1, class P>
inline hipError_t launch_gemm(const P& p, int splits, hipStream_t st) {
  static_assert(gemm_smem_floats<BM, BN, WM, WN, BK, WK, P>() * 4 <= 160 * 1024,
                "block LDS exceeds 160 KB");
  const int tiles = ((p.N + BN - 1) / BN) * ((p.M + BM - 1) / BM);
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, BK, WK, P>), dim3(tiles, 1, splits),
                     dim3(gemm_threads<BM, BN, WM, WN, BK, WK>()), 0, st, p);
  return hipGetLastError();
}

// gemm_f32_multi_kernel over `count` sub-problems of `tiles` tiles each (grid z = count).
template <int BM, int BN, int WM, int WN, int BK, int WK, class... S>
inline hipError_t launch_gemm_multi(const ZMulti<S...>& q, int tiles, int count, hipStream_t st) {
  static_assert(zmulti_smem_floats<BM, BN, WM, WN, BK, WK, S...>() * 4 <= 160 * 1024,
                "block LDS exceeds 160 KB");
  hipLaunchKernelGGL((gemm_f32_multi_kernel<BM, BN, WM, WN, BK, WK, S...>),
                     dim3((unsigned)tiles, 1, (unsigned)count),
                     dim3(gemm_threads<BM, BN, WM, WN, BK, WK>()), 0, st, q);
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace acme
