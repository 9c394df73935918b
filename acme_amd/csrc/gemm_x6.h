// Split-precision MFMA GEMM: f32 operands as three bf16 planes, six bf16 MFMAs per
// 16-deep k step, f32 accumulation (gfx950 / CDNA4).
//
// Each f32 operand value x is split exactly into x = h + m + l with h = bf16(x),
// m = bf16(x - h), l = bf16(x - h - m) (8 + 8 + 8 significant bits = f32's 24; both
// subtractions are exact in f32).  The product is
//     a b = ah bh + (ah bm + am bh) + (ah bl + al bh + am bm) + O(2^-24 a b)
// and the six terms run as v_mfma_f32_32x32x16_bf16 (exact bf16 x bf16 products, f32
// accumulate), smallest first.  The dropped terms (am bl, al bm, al bl) are below f32's
// unit roundoff, so the result has the error profile of an f32 MFMA GEMM (measured on the
// learner's layer shapes: median relative error 7.9e-7 vs 7.8e-7 for
// v_mfma_f32_32x32x2_f32, tests/test_gemm_gpu.py), at 6 x 32 = 192 MFMA cycles per 16 k
// instead of 8 x 64 = 512.  It is a faster way to compute the same f32 GEMM, not a
// reduced-precision one: ACME_MATMUL=f32 selects the f32-MFMA engine (gemm.h).
//
// Same problem concept as gemm.h (loaders return f32x4 of 4 consecutive k of a row
// (KCONTIG) or 4 consecutive rows at one k (RCONTIG)).  RCONTIG operands are loaded as
// 4 x 4 blocks (4 k per thread) and transposed in registers, so both modes store rows of
// 4 consecutive k.
//
// LDS image per stage and operand: 3 planes x R rows x BK bf16; 16-B chunks (8 k) of a
// row XOR-swizzled by row (chunk' = chunk ^ s(row)) so the ds_read_b128 fragment reads
// are conflict-free.  MFMA operand map (32x32x16 bf16): lane (r = l & 31, h = l >> 5)
// holds A[r][8h + j] and B[8h + j][r], j = 0..7, i.e. chunk 2s + h of k step s.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "gemm.h"

namespace acme {
namespace gemm {

using bf16x4 = __attribute__((ext_vector_type(4))) __bf16;
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;

// Process-wide matmul engine: x6 (default) or f32 (ACME_MATMUL=f32, or
// acme_set_matmul_engine(ACME_MATMUL_F32)).
bool use_x6();

template <int BK>
__device__ __forceinline__ int x6_swz(int row) {
  return BK == 16 ? ((row >> 3) & 1) : ((row >> 2) & 3);
}

__device__ __forceinline__ void split3(const f32x4 x, bf16x4& h, bf16x4& m, bf16x4& l) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const __bf16 hj = (__bf16)x[j];
    const float r = x[j] - (float)hj;
    const __bf16 mj = (__bf16)r;
    h[j] = hj;
    m[j] = mj;
    l[j] = (__bf16)(r - (float)mj);
  }
}

template <int R, int NT, int MODE, int BK>
struct PlanX6 {
  static constexpr int ROW_BYTES = 2 * BK;
  static constexpr int PLANE = R * ROW_BYTES;          // bytes of one plane
  static constexpr int BYTES = 3 * PLANE;              // one stage of this operand
  static constexpr int QPR = BK / 4;                   // 4-k groups per row
  // KCONTIG: unit = 4 k of one row.  RCONTIG: unit = 4 rows x 4 k.
  static constexpr int UNITS = MODE == KCONTIG ? R * QPR : (R / 4) * QPR;
  static constexpr int PER_THREAD = (UNITS + NT - 1) / NT;
  static_assert(UNITS % NT == 0 || UNITS < NT, "tile units must divide evenly over the threads");
  static constexpr int VECS = MODE == KCONTIG ? 1 : 4;  // f32x4 loads per unit
  __device__ static __forceinline__ bool owns(int u) { return UNITS >= NT || u < UNITS; }
  __device__ static __forceinline__ int row_of(int u) {
    return MODE == KCONTIG ? u / QPR : 4 * (u / QPR);
  }
  __device__ static __forceinline__ int kk_of(int u) { return 4 * (u % QPR); }
  // Store 4 consecutive k (one 8-B piece per plane) of row `row`, k-group q.
  __device__ static __forceinline__ void put(uint8_t* tile, int row, int q, const f32x4 x) {
    bf16x4 h, m, l;
    split3(x, h, m, l);
    const int c = (q >> 1) ^ x6_swz<BK>(row);
    const int off = row * ROW_BYTES + 16 * c + 8 * (q & 1);
    *reinterpret_cast<bf16x4*>(tile + off) = h;
    *reinterpret_cast<bf16x4*>(tile + PLANE + off) = m;
    *reinterpret_cast<bf16x4*>(tile + 2 * PLANE + off) = l;
  }
  __device__ static __forceinline__ bf16x8 frag(const uint8_t* tile, int plane, int row, int c) {
    return *reinterpret_cast<const bf16x8*>(tile + plane * PLANE + row * ROW_BYTES +
                                            16 * (c ^ x6_swz<BK>(row)));
  }
};

// Stores an RCONTIG 4 x 4 block (v[kv][r] = row r, k offset kv) as 4 rows of 4 k.
template <class PL>
__device__ __forceinline__ void put_block(uint8_t* tile, int u, const f32x4 (&v)[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
    PL::put(tile, PL::row_of(u) + r, u % PL::QPR, f32x4{v[0][r], v[1][r], v[2][r], v[3][r]});
}

template <int BM, int BN, int WM, int WN, int BK, class P>
__global__ void __launch_bounds__(64 * WM * WN) gemm_x6_kernel(const P p_in) {
  const P p = z_select(p_in);
  constexpr int NT = 64 * WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MT = TM / 32, NTL = TN / 32;
  static_assert(TM % 32 == 0 && TN % 32 == 0, "wave tile must be a multiple of 32x32");
  static_assert(BK == 16 || BK == 32, "BK must be 16 or 32");
  using PA = PlanX6<BM, NT, P::A_MODE, BK>;
  using PB = PlanX6<BN, NT, P::B_MODE, BK>;
  constexpr int STAGE = PA::BYTES + PB::BYTES;

  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int tile = blockIdx.x;
  const int m0 = (tile / tiles_n) * BM;
  const int n0 = (tile % tiles_n) * BN;
  const int split = HasZClass<P>::value ? 0 : blockIdx.z;
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

  f32x4 ra[PA::PER_THREAD][PA::VECS], rb[PB::PER_THREAD][PB::VECS];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < PA::PER_THREAD; ++i) {
      const int u = tid + i * NT;
      const int k = k0 + PA::kk_of(u);
#pragma unroll
      for (int v = 0; v < PA::VECS; ++v)
        ra[i][v] = (PA::owns(u) && k + v < kend) ? p.a_load(arow[i], k + v) : zero4();
    }
#pragma unroll
    for (int i = 0; i < PB::PER_THREAD; ++i) {
      const int u = tid + i * NT;
      const int k = k0 + PB::kk_of(u);
#pragma unroll
      for (int v = 0; v < PB::VECS; ++v)
        rb[i][v] = (PB::owns(u) && k + v < kend) ? p.b_load(brow[i], k + v) : zero4();
    }
  };
  // KCONTIG vectors already hold 4 k of one row; RCONTIG 4x4 blocks are transposed so
  // row r's 4 k are {rb[v][r]}.
  auto stash = [&](int buf) {
    uint8_t* sa = smem + buf * STAGE;
    uint8_t* sb = sa + PA::BYTES;
#pragma unroll
    for (int i = 0; i < PA::PER_THREAD; ++i) {
      const int u = tid + i * NT;
      if (!PA::owns(u)) continue;
      if constexpr (P::A_MODE == KCONTIG) {
        PA::put(sa, PA::row_of(u), u % PA::QPR, ra[i][0]);
      } else {
        put_block<PA>(sa, u, ra[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < PB::PER_THREAD; ++i) {
      const int u = tid + i * NT;
      if (!PB::owns(u)) continue;
      if constexpr (P::B_MODE == KCONTIG) {
        PB::put(sb, PB::row_of(u), u % PB::QPR, rb[i][0]);
      } else {
        put_block<PB>(sb, u, rb[i]);
      }
    }
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
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) fetch(kbeg + (kt + 1) * BK);
    const uint8_t* sa = smem + (kt & 1) * STAGE;
    const uint8_t* sb = sa + PA::BYTES;
    if constexpr (kColSum) {
      if (do_colsum) {
#pragma unroll
        for (int c = 0; c < BK / 8; ++c) {
          const bf16x8 x0 = PB::frag(sb, 0, tid, c), x1 = PB::frag(sb, 1, tid, c),
                       x2 = PB::frag(sb, 2, tid, c);
#pragma unroll
          for (int j = 0; j < 8; ++j) colsum += ((float)x0[j] + (float)x1[j]) + (float)x2[j];
        }
      }
    }
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int c = 2 * s + h;
      bf16x8 fa[MT][3], fb[NTL][3];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) fa[i][pl] = PA::frag(sa, pl, wm * TM + i * 32 + r, c);
#pragma unroll
      for (int j = 0; j < NTL; ++j)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) fb[j][pl] = PB::frag(sb, pl, wn * TN + j * 32 + r, c);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], fb[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][2], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][0], acc[i][j], 0, 0, 0);
        }
    }
    if (more) stash((kt + 1) & 1);
    __syncthreads();
  }

  store_tile<MT, NTL>(p, acc, m0 + wm * TM, n0 + wn * TN, h, r, split);
  if constexpr (kColSum) {
    if (do_colsum && n0 + tid < p.N) p.store_colsum(n0 + tid, colsum, split);
  }
}

template <int BM, int BN, int WM, int WN, int BK = 16, class P>
inline hipError_t launch_gemm_x6(const P& p, int splits, hipStream_t st) {
  // Two stages of three bf16 planes must fit the 64-KiB static LDS of a workgroup.
  constexpr int BKX = 2 * 3 * 2 * (BM + BN) * BK > 65536 ? 16 : BK;
  const int tiles = ((p.N + BN - 1) / BN) * ((p.M + BM - 1) / BM);
  hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, WM, WN, BKX, P>), dim3(tiles, 1, splits),
                     dim3(64 * WM * WN), 0, st, p);
  return hipGetLastError();
}

// Which problems the x6 engine takes.  Its stores want rows of 4 consecutive k; an
// RCONTIG operand (4 rows at one k) costs a 4 x 4 register transpose and row-strided LDS
// stores that land in one 8-bank window (rows 4 apart are 32 dwords apart), measured
// slower than the f32 engine for the weight-gradient GEMMs whose A operand is RCONTIG.
// So: A must be KCONTIG; an RCONTIG B is taken only when the problem opts in
// (kX6 = true: a narrow weight operand, e.g. convolution / dense forward).
template <class P, class = void>
struct X6OptIn {
  static constexpr bool value = false;
};
template <class P>
struct X6OptIn<P, decltype(void(P::kX6))> {
  static constexpr bool value = P::kX6;
};
template <class P>
constexpr bool x6_eligible() {
  return P::A_MODE == KCONTIG && (P::B_MODE == KCONTIG || X6OptIn<P>::value);
}

// TFLOP/s ceiling of the engine launch_matmul picks for P (profiler roofline): the x6
// engine runs six bf16 MFMA terms per f32 product (bf16 dense peak / 6), the f32 engine
// v_mfma_f32_32x32x2_f32.
template <int WK = 1, class P>
inline double matmul_peak_tflops() {
  if constexpr (WK == 1 && x6_eligible<P>()) {
    if (use_x6()) return 2500.0 / 6.0;
  }
  return 157.3;
}

// The engine a learner launch uses: x6 for eligible problems unless ACME_MATMUL=f32 / the
// C API chose f32.
template <int BM, int BN, int WM, int WN, int BK = 16, int WK = 1, class P>
inline hipError_t launch_matmul(const P& p, int splits, hipStream_t st) {
  if constexpr (WK == 1 && x6_eligible<P>()) {
    if (use_x6()) return launch_gemm_x6<BM, BN, WM, WN, BK>(p, splits, st);
  }
  return launch_gemm<BM, BN, WM, WN, BK, WK>(p, splits, st);
}

}  // namespace gemm
}  // namespace acme
