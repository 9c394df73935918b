// Direct-operand plane GEMM (gfx950): the block's waves are stacked along M (WN = 1), so
// every A element of the block's N panel (<= 128 columns) is used by exactly ONE wave.
// Written for the Nature-CNN convolutions (N = 32 or 64 channels: one panel); wider
// problems (the fused dense layer) tile N in 128-column panels and may split K
// (blockIdx.z, p.k_chunk per split, as gemm_p3_kernel).
//
// gemm_p3.h stages both operands through LDS.  With N <= 64 the A tile dominates the
// staging traffic: (BM + BN) * BK * 6 bytes of ds_write_b128 per stage against BM * BN * BK
// * 6 / 16384 MFMAs, about 384 B per MFMA at 128 x 64, so the LDS store path (~79 B/clk/CU,
// MI355X_MICROARCH.md §LDS) rivals the MFMA pipe.  Here each wave owns 32 * MT whole rows
// of C and all N columns; its A fragments are loaded straight from HBM / L2 into VGPRs in
// the MFMA operand layout (a KCONTIG unit is exactly one lane's 8 k of one row: lanes 0-31
// rows, lanes 32-63 the next 8 k), so A never touches LDS.  Only B (the small weight panel)
// is staged in LDS, shared by the block's NW waves.  Per stage of BK k:
//   A: MT * BK/16 * NPA buffer_load_b128 per lane (prefetched two stages ahead, into the
//      register set the stage just consumed);
//   B: the register-staged double buffer of gemm_p3_kernel (PlanP3 images, swizzled).
// One barrier per stage (for B).  Epilogue and problem concept as in gemm_p3.h (the
// problem's A_MODE must be KCONTIG).
#pragma once

#include "gemm_p3.h"

namespace acme {
namespace gemm {

template <int BN_, int MT, int NW, int BK, class P>
struct P3DCfg {
  static constexpr int BN = BN_;  // the problem's N rounded up to 32: 32 or 64
  static constexpr int BM = NW * 32 * MT;
  using Core = P3Core<BM, BN, NW, 1, BK, P>;
  static constexpr int STAGE_B = Core::PB::BYTES;
  static constexpr int LDS = 2 * STAGE_B > Core::EPI_BYTES ? 2 * STAGE_B : Core::EPI_BYTES;
};

template <int BN_, int MT, int NW, int BK, class P>
__global__ void __launch_bounds__(64 * NW) gemm_p3d_kernel(const P p_in, int n_major) {
  static_assert(P::A_MODE == KCONTIG, "direct A fragments need k-contiguous A units");
  using Cfg = P3DCfg<BN_, MT, NW, BK, P>;
  using C = typename Cfg::Core;
  using PB = typename C::PB;
  constexpr int BN = Cfg::BN, BM = Cfg::BM;
  constexpr int NT = 64 * NW, NPA = P::A_PLANES, NPB = P::B_PLANES, NTL = BN / 32;
  constexpr int KS = BK / 16;  // k16 steps per stage
  static_assert(BN % 32 == 0 && BN <= 128, "N panel of 32, 64, 96 or 128 columns");
  const BlockPlace bp = place_block<BM, BN>(p_in.M, p_in.N, n_major);
  const P p = z_select_at(p_in, bp.z);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int m0 = bp.m0, n0 = bp.n0;
  // blockIdx.z: the problem's class (kZClass) or its K split.
  const int split = HasZClass<P>::value ? 0 : bp.z;
  const int kbeg = split * p.k_chunk;
  const int kend = kbeg + p.k_chunk < p.K ? kbeg + p.k_chunk : p.K;
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  // This lane's A rows (one per 32-row block of the wave's tile) and k offset in a step.
  typename P::ARow arow[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) arow[i] = p.a_row(m0 + wave * 32 * MT + i * 32 + (lane & 31));
  const int kl = 8 * (lane >> 5);
  typename P::BRow brow[PB::PER_THREAD];
#pragma unroll
  for (int i = 0; i < PB::PER_THREAD; ++i)
    brow[i] = p.b_row(n0 + (PB::owns(tid + i * NT) ? PB::row_of(tid + i * NT) : 0));

  __amdgpu_buffer_rsrc_t srcA[NPA], srcB[NPB];
#pragma unroll
  for (int pl = 0; pl < NPA; ++pl) srcA[pl] = plane_rsrc(p.a_src, pl);
#pragma unroll
  for (int pl = 0; pl < NPB; ++pl) srcB[pl] = plane_rsrc(p.b_src, pl);

  bf16x8 fa[2][KS][MT][NPA];
  u32x4 rb[2][PB::PER_THREAD][NPB];
  auto fetch_a = [&](auto S, int k0) {
    constexpr int set = decltype(S)::value;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int kk = 16 * s + kl;
        const uint32_t off = k0 + kk < kend ? p.a_off(arow[i], k0, kk) : kOOB;
#pragma unroll
        for (int pl = 0; pl < NPA; ++pl) {
          if constexpr (HasAU8<P>::value)
            fa[set][s][i][pl] = __builtin_bit_cast(bf16x8, load_u8_unit(srcA[pl], off));
          else
            fa[set][s][i][pl] = __builtin_bit_cast(
                bf16x8, __builtin_amdgcn_raw_buffer_load_b128(srcA[pl], off, 0, 0));
        }
      }
  };
  auto fetch_b = [&](auto S, int k0) {
    constexpr int set = decltype(S)::value;
#pragma unroll
    for (int i = 0; i < PB::PER_THREAD; ++i) {
      const int u = tid + i * NT;
      const int kk = PB::kk_of(u);
      const uint32_t off = (PB::owns(u) && k0 + kk < kend) ? p.b_off(brow[i], k0, kk) : kOOB;
#pragma unroll
      for (int pl = 0; pl < NPB; ++pl)
        rb[set][i][pl] =
            __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(srcB[pl], off, 0, 0));
    }
  };
  auto stash_b = [&](auto S, int buf) {
    constexpr int set = decltype(S)::value;
    uint8_t* sb = smem + buf * Cfg::STAGE_B;
#pragma unroll
    for (int i = 0; i < PB::PER_THREAD; ++i) {
      const int u = tid + i * NT;
      if (!PB::owns(u)) continue;
      const int off = PB::offset(u);
#pragma unroll
      for (int pl = 0; pl < NPB; ++pl)
        *reinterpret_cast<u32x4*>(sb + pl * PB::PLANE + off) = rb[set][i][pl];
    }
  };

  f32x16 acc[MT][NTL];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  auto compute = [&](auto S, int buf) {
    constexpr int set = decltype(S)::value;
    const uint8_t* sb = smem + buf * Cfg::STAGE_B;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      bf16x8 fb[NTL][NPB];
#pragma unroll
      for (int j = 0; j < NTL; ++j)
#pragma unroll
        for (int pl = 0; pl < NPB; ++pl) fb[j][pl] = PB::frag(sb, pl, j * 32, s, lane);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j) {
          const bf16x8(&a)[NPA] = fa[set][s][i];
          // Smallest terms first, as gemm_p3.h.
          if constexpr (NPA == 3 && NPB == 3) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], fb[j][1], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], fb[j][0], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], fb[j][2], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], fb[j][0], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], fb[j][1], acc[i][j], 0, 0, 0);
          } else if constexpr (NPA == 3) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], fb[j][0], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], fb[j][0], acc[i][j], 0, 0, 0);
          } else if constexpr (NPB == 3) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], fb[j][2], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], fb[j][1], acc[i][j], 0, 0, 0);
          }
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], fb[j][0], acc[i][j], 0, 0, 0);
        }
    }
  };

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  // Prologue: stage 0 (A set 0, B in LDS buffer 0), stage 1 (A set 1, B registers set 1).
  fetch_b(S0{}, kbeg);
  fetch_a(S0{}, kbeg);
  fetch_b(S1{}, kbeg + BK);
  fetch_a(S1{}, kbeg + BK);
  stash_b(S0{}, 0);
  __syncthreads();
  // Iteration kt: LDS buffer kt & 1 and A set kt & 1 hold stage kt; B registers set
  // (kt + 1) & 1 hold stage kt + 1, stashed first (its buffer was last read in iteration
  // kt - 1, before the barrier); then B of stage kt + 2 is fetched into set kt & 1, stage kt
  // is computed, and A of stage kt + 2 is fetched into the set it just consumed.  Past the
  // end, fetches read zeros (offsets at or beyond kend are kOOB).
  auto iter = [&](auto S, int kt) {
    constexpr int set = decltype(S)::value;
    using Other = std::integral_constant<int, set ^ 1>;
    stash_b(Other{}, set ^ 1);
    fetch_b(S, kbeg + (kt + 2) * BK);
    compute(S, set);
    fetch_a(S, kbeg + (kt + 2) * BK);
    __syncthreads();
  };
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    iter(S0{}, kt);
    iter(S1{}, kt + 1);
  }
  if (kt < nk) iter(S0{}, kt);

  f32x16 cs[C::NCS];
  C::epilogue(p, smem, m0, n0, wave, wave, 0, lane, split, acc, cs, false);
}

// z: the number of classes of a kZClass problem, else of K splits (p.k_chunk each).
template <int BN, int MT, int NW, int BK, class P>
inline hipError_t launch_gemm_p3d(const P& p, int z, hipStream_t st) {
  using Cfg = P3DCfg<BN, MT, NW, BK, P>;
  static_assert(Cfg::LDS <= 160 * 1024, "LDS");
  static hipError_t attr = p3_set_lds(&gemm_p3d_kernel<BN, MT, NW, BK, P>, Cfg::LDS);
  if (attr != hipSuccess) return attr;
  const int tiles = ((p.N + Cfg::BN - 1) / Cfg::BN) * ((p.M + Cfg::BM - 1) / Cfg::BM);
  hipLaunchKernelGGL((gemm_p3d_kernel<BN, MT, NW, BK, P>), dim3(tiles, 1, z), dim3(64 * NW),
                     Cfg::LDS, st, p, p3_n_major(p));
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace acme
