// Image-resident stride-2 input gradient by sub-pixel classes (gfx950): conv2's dZ -> dX.
//
// conv_p3.h P3ConvDgradSubZ splits dX = conv2^T(dZ) into the S*S = 4 parity classes of the
// output pixel (each a stride-1 correlation with a 2x2 sub-kernel, K = 2*2*CO = 256) and
// gemm_p3.h runs the classes as blockIdx.z: every class gathers its dZ rows from HBM / L2
// again (PMC: 169 MB per launch against 81 MB of distinct bytes) and each block computes
// only 8 k-stages.  Here one block owns one frame: the frame's dZ image (OH x OW x CO, both
// planes, XOR-swizzled 16-B chunks as gemm_p3i.h) is loaded into LDS once, and the
// four classes are computed from it at once -- waves 2z and 2z + 1 own class z's rows (at
// most 128: 64 each, MT = 2) -- with the four classes' weight panels streamed together
// through the two-stage register-staged ring (one 16-B unit per thread per plane).  The
// epilogue is the problem's own (ReLU mask from the previous activation, plane stores).
#pragma once

#include "conv_p3.h"
#include "gemm_p3.h"

namespace acme {
namespace gemm {

template <class G, int FPB = 1>
struct P3SCfg {
  using P = conv::P3ConvDgradSubZ<G>;
  static constexpr int S = G::S, CLASSES = G::S * G::S;
  static constexpr int MT = 2, NW = 2 * CLASSES * FPB, NT = 64 * NW, BK = 32, KS = 2;
  static constexpr int BN = 32;                                // N = CI
  static constexpr int H = G::OH, W = G::OW, C = G::CO;        // the dZ image
  static constexpr int CPX = C / 8;
  static constexpr int FRAME = H * W * 2 * C;                  // one frame's image, one plane
  static constexpr int PLANE = FPB * FRAME + 16;               // + the zero unit
  static constexpr int NP = kPlanes;
  static constexpr int IMG = NP * PLANE;
  using PB = PlanP3<BN, 64 * 2 * CLASSES, KCONTIG, NP, BK>;    // one class's B stage
  static constexpr int STAGE_B = CLASSES * PB::BYTES;
  static constexpr int MAIN = IMG + 2 * STAGE_B;
  static constexpr int EPI = NW * 32 * (BN + 4) * 4;
  static constexpr int LDS = MAIN > EPI ? MAIN : EPI;
  using Core = P3Core<2 * 32 * MT, BN, 2, 1, BK, P>;           // a class's 2 waves x 64 rows
  static_assert(G::CI == BN && C == 64 && CPX == 8, "conv2 geometry (CI 32, CO 64)");
  static constexpr int BT = PB::UNITS * CLASSES;               // B loader threads
  static_assert(BT == 64 * 2 * CLASSES, "one B unit per loader thread per plane");
  static_assert(P::KR % BK == 0 && (P::KR / BK) % 2 == 0, "whole, even stage count");
  __device__ static __forceinline__ int swz(int q) { return (q >> 1) & (CPX - 1); }
};

template <class G, int FPB>
__global__ void __launch_bounds__(64 * 2 * G::S * G::S * FPB) gemm_p3s_kernel(
    const conv::P3ConvDgradSubZ<G> p_in, int frames) {
  using Cfg = P3SCfg<G, FPB>;
  using PB = typename Cfg::PB;
  using C = typename Cfg::Core;
  using P = conv::P3ConvDgradSubZ<G>;
  constexpr int NT = Cfg::NT, BK = Cfg::BK, KS = Cfg::KS, MT = Cfg::MT, PLANE = Cfg::PLANE;
  constexpr int W = Cfg::W, H = Cfg::H, CPX = Cfg::CPX, NP = Cfg::NP;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fi = wave / (2 * Cfg::CLASSES);  // this wave's frame in the block
  const int f = blockIdx.x * FPB + fi;
  const int z = (wave >> 1) % Cfg::CLASSES, half = wave & 1;  // its class, half of the rows
  const uint8_t* img = smem + fi * Cfg::FRAME;
  P pz = p_in.for_z(z);
  const int nhw = pz.nh * pz.nw;
  const int m0 = f * nhw;
  pz.M = m0 + nhw < pz.M ? m0 + nhw : pz.M;  // this frame's rows of the class only
  const int nk = P::KR / BK;

  // ---- B: loader thread tid loads unit tid % 128 of class tid / 128's panel (each plane).
  const bool bload = tid < Cfg::BT;
  const int bz = bload ? tid / PB::UNITS : 0, bu = tid - bz * PB::UNITS;
  const P pb = p_in.for_z(bz);
  const typename P::BRow brow = pb.b_row(PB::row_of(bu));
  __amdgpu_buffer_rsrc_t srcB[NP];
#pragma unroll
  for (int pl = 0; pl < NP; ++pl) srcB[pl] = plane_rsrc(p_in.b_src, pl);
  u32x4 rb[2][NP];
  auto fetch_b = [&](auto S_, int k0) {
    constexpr int set = decltype(S_)::value;
    const uint32_t off = bload && k0 < P::KR ? pb.b_off(brow, k0, PB::kk_of(bu)) : kOOB;
#pragma unroll
    for (int pl = 0; pl < NP; ++pl)
      rb[set][pl] =
          __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(srcB[pl], off, 0, 0));
  };
  auto stash_b = [&](auto S_, int buf) {
    constexpr int set = decltype(S_)::value;
    uint8_t* sb = smem + Cfg::IMG + buf * Cfg::STAGE_B + bz * PB::BYTES;
    if (!bload) return;
#pragma unroll
    for (int pl = 0; pl < NP; ++pl)
      *reinterpret_cast<u32x4*>(sb + pl * PB::PLANE + PB::offset(bu)) = rb[set][pl];
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  fetch_b(S0{}, 0);
  fetch_b(S1{}, BK);

  // ---- A: the block's dZ images, each 16-B unit of each plane once.
  {
    constexpr int UNITS = FPB * H * W * CPX;
    constexpr int PER = (UNITS + NT - 1) / NT;
    __amdgpu_buffer_rsrc_t srcA[NP];
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) srcA[pl] = plane_rsrc(p_in.a_src, pl);
    u32x4 v[PER][NP];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = tid + j * NT;
      const bool ok = u < UNITS && blockIdx.x * FPB + u / (H * W * CPX) < frames;
      const uint32_t off = ok ? (uint32_t)(((int64_t)blockIdx.x * UNITS + u) * 16) : kOOB;
#pragma unroll
      for (int pl = 0; pl < NP; ++pl)
        v[j][pl] =
            __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(srcA[pl], off, 0, 0));
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = tid + j * NT;
      if (u < UNITS) {
        const int fu = u / (H * W * CPX), uu = u - fu * (H * W * CPX);
        const int q = uu / CPX, c = uu - q * CPX;
        const int a = fu * Cfg::FRAME + q * (2 * Cfg::C) + 16 * (c ^ Cfg::swz(q));
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) *reinterpret_cast<u32x4*>(smem + pl * PLANE + a) = v[j][pl];
      }
    }
    if (tid < NP) *reinterpret_cast<u32x4*>(smem + tid * PLANE + PLANE - 16) = zero_u4();
  }
  stash_b(S0{}, 0);

  // ---- This lane's rows: dZ anchor (oh0, ow0) of output pixel (rh + S i, rw + S j).
  int oh0[MT], ow0[MT];
  bool rok[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int lr = half * 32 * MT + i * 32 + (lane & 31);
    rok[i] = lr < nhw && f < frames;
    const int ii = rok[i] ? lr / pz.nw : 0, jj = rok[i] ? lr - ii * pz.nw : 0;
    oh0[i] = (pz.rh + Cfg::S * ii + G::PT - pz.ph) / Cfg::S;
    ow0[i] = (pz.rw + Cfg::S * jj + G::PL - pz.pw) / Cfg::S;
  }
  __syncthreads();

  typename C::Acc acc;
  acc.zero();

  auto compute = [&](int k0, int buf) {
    const uint8_t* sb = smem + Cfg::IMG + buf * Cfg::STAGE_B + z * PB::BYTES;
    constexpr int T = P::JW * Cfg::C;
    const int jh = k0 / T, jw = (k0 - jh * T) / Cfg::C;  // wave-uniform
    const int cb = (k0 % Cfg::C) >> 3;
    int qb[MT], qs[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int oh = oh0[i] - jh, ow = ow0[i] - jw;
      const bool in = rok[i] && (unsigned)oh < (unsigned)H && (unsigned)ow < (unsigned)W;
      const int q = oh * W + ow;
      qb[i] = in ? q * (2 * Cfg::C) : -1;
      qs[i] = Cfg::swz(q);
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      f16x8 fb[NP];
#pragma unroll
      for (int pl = 0; pl < NP; ++pl) fb[pl] = PB::frag(sb, pl, 0, s, lane);
      const int c = cb + 2 * s + (lane >> 5);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const uint8_t* a = qb[i] >= 0 ? img + qb[i] + 16 * (c ^ qs[i]) : smem + PLANE - 16;
        f16x8 fa[NP];
#pragma unroll
        for (int pl = 0; pl < NP; ++pl)
          fa[pl] = *reinterpret_cast<const f16x8*>(a + pl * PLANE);
        acc.terms(i, 0, fa, fb);
      }
    }
  };
  auto iter = [&](auto S_, int kt) {
    constexpr int set = decltype(S_)::value;
    using Other = std::integral_constant<int, set ^ 1>;
    stash_b(Other{}, set ^ 1);
    fetch_b(S_, (kt + 2) * BK);
    compute(kt * BK, set);
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    iter(S0{}, kt);
    iter(S1{}, kt + 1);
  }

  // Row m = m0 + half * 64 + i * 32 + r of class z; LDS staging region of this wave.
  C::epilogue(pz, smem, m0, 0, wave, half, 0, lane, 0, acc, false);
}

template <class G, int FPB = 1>
inline hipError_t launch_gemm_p3s(const conv::P3ConvDgradSubZ<G>& p, int frames, hipStream_t st) {
  using Cfg = P3SCfg<G, FPB>;
  static_assert(Cfg::LDS <= 160 * 1024, "dZ images + two four-class B stages must fit the LDS");
  static hipError_t attr = p3_set_lds(&gemm_p3s_kernel<G, FPB>, Cfg::LDS);
  if (attr != hipSuccess) return attr;
  if (p.N > Cfg::BN || p.batch != frames || frames < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm_p3s_kernel<G, FPB>), dim3((frames + FPB - 1) / FPB), dim3(Cfg::NT),
                     Cfg::LDS, st, p, frames);
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace acme
