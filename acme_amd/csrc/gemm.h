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

// Problem concept (see conv.h):
//   static constexpr int A_MODE, B_MODE;
//   int M, N, K;            rows of A (= C rows), rows of B (= C cols), reduction length
//   int k_chunk;            reduction elements per split (multiple of BK), K if no split
//   struct ARow; ARow a_row(int row) const;     f32x4 a_load(const ARow&, int k) const;
//   struct BRow; BRow b_row(int row) const;     f32x4 b_load(const BRow&, int k) const;
//   void store(int m, int n, float v, int split) const;
// The loaders must return zeros for rows >= M / N and k >= K.

template <int BM, int BN, int WM, int WN, int BK, class P>
__global__ void __launch_bounds__(64 * WM * WN) gemm_f32_kernel(const P p) {
  constexpr int NT = 64 * WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MT = TM / 32, NTL = TN / 32;
  static_assert(TM % 32 == 0 && TN % 32 == 0, "wave tile must be a multiple of 32x32");
  static_assert(BK == 16 || BK == 32, "BK must be 16 or 32");
  using PA = OperandPlan<BM, NT, P::A_MODE, BK>;
  using PB = OperandPlan<BN, NT, P::B_MODE, BK>;
  constexpr int STAGE = PA::FLOATS + PB::FLOATS;

  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int tile = blockIdx.x;
  const int m0 = (tile / tiles_n) * BM;
  const int n0 = (tile % tiles_n) * BN;
  const int split = blockIdx.z;
  const int kbeg = split * p.k_chunk;
  int kend = kbeg + p.k_chunk;
  if (kend > p.K) kend = p.K;
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  typename P::ARow arow[PA::PER_THREAD];
  typename P::BRow brow[PB::PER_THREAD];
#pragma unroll
  for (int i = 0; i < PA::PER_THREAD; ++i)
    arow[i] = p.a_row(m0 + (PA::owns(tid + i * NT) ? PA::row_of(tid + i * NT) : 0));
#pragma unroll
  for (int i = 0; i < PB::PER_THREAD; ++i)
    brow[i] = p.b_row(n0 + (PB::owns(tid + i * NT) ? PB::row_of(tid + i * NT) : 0));

  f32x4 ra[PA::PER_THREAD], rb[PB::PER_THREAD];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < PA::PER_THREAD; ++i) {
      const int k = k0 + PA::kk_of(tid + i * NT);
      ra[i] = (PA::owns(tid + i * NT) && k < kend) ? p.a_load(arow[i], k) : zero4();
    }
#pragma unroll
    for (int i = 0; i < PB::PER_THREAD; ++i) {
      const int k = k0 + PB::kk_of(tid + i * NT);
      rb[i] = (PB::owns(tid + i * NT) && k < kend) ? p.b_load(brow[i], k) : zero4();
    }
  };
  auto stash = [&](int buf) {
    float* sa = smem + buf * STAGE;
    float* sb = sa + PA::FLOATS;
#pragma unroll
    for (int i = 0; i < PA::PER_THREAD; ++i)
      if (PA::owns(tid + i * NT)) PA::store(sa, tid + i * NT, ra[i]);
#pragma unroll
    for (int i = 0; i < PB::PER_THREAD; ++i)
      if (PB::owns(tid + i * NT)) PB::store(sb, tid + i * NT, rb[i]);
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
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) fetch(kbeg + (kt + 1) * BK);
    const float* sa = smem + (kt & 1) * STAGE;
    const float* sb = sa + PA::FLOATS;
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
    if (more) stash((kt + 1) & 1);
    __syncthreads();
  }

  // Epilogue: C/D map of the 32x32 MFMA: col = lane & 31, row = (v&3) + 8(v>>2) + 4h.
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int m = m0 + wm * TM + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
        const int n = n0 + wn * TN + j * 32 + r;
        if (m < p.M && n < p.N) p.store(m, n, acc[i][j][v], split);
      }
  if constexpr (kColSum) {
    if (do_colsum && n0 + tid < p.N) p.store_colsum(n0 + tid, colsum, split);
  }
}

template <int BM, int BN, int WM, int WN, int BK = 16, class P>
inline hipError_t launch_gemm(const P& p, int splits, hipStream_t st) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, BK, P>), dim3(tiles, 1, splits),
                     dim3(64 * WM * WN), 0, st, p);
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace acme
