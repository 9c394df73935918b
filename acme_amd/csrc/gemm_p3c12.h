// Fused conv1 -> conv2 forward of the Nature torso, one frame per block (gfx950).
//
// conv1 writes its output x1 as two f16 planes (43 MB per launch on average) and conv2
// reads it back, im2col-duplicated, through L2 (129 MB).  Only the o_tm1 rows' x1 is ever
// needed again (conv2's weight gradient and input-gradient ReLU mask); the o_t rows of the
// online network and all target rows are consumed by conv2 alone.  Here a block computes
// conv1 for one frame from its image in LDS (gemm_p3i.h pixel pairs), its epilogue writes
// x1 straight into a second LDS image in conv2's layout (gemm_p3i.h ImgGeom: swizzled
// channel chunks, stride-2 column order) -- and to HBM only for frames below hbm_frames --
// then conv2 runs on that image.  Both weight panels stream through register-staged
// two-stage rings; conv2's first two stages are fetched at kernel start.  LDS: frame image
// 56 KB (later conv2's weight ring and both epilogue staging areas) + conv1 ring 8 KB +
// x1 image 57 KB = 121 KB, one block (8 waves) per CU.
#pragma once

#include "conv_p3.h"
#include "gemm_p3i.h"

namespace acme {
namespace gemm {

// conv1's epilogue sink: the frame's x1 image in LDS (both planes, x1's scale) and, when
// `hbm`, the x1 planes in HBM (the same values as P3ConvFwd<G1, 1>::store8).
template <class G1, class G2, bool U8 = false>
struct P3C1ToLds {
  using Base = conv::P3ConvFwd<G1, 1, U8>;
  using I2 = ImgGeom<G2, false>;
  static constexpr int A_MODE = Base::A_MODE, B_MODE = Base::B_MODE;
  static constexpr int A_PLANES = 1, B_PLANES = kPlanes;
  static constexpr bool kStore8 = true;
  static constexpr bool kAmax = true;
  int M, N, K, k_chunk;
  Base base;
  uint8_t* x1;  // LDS image, plane stride `plane` bytes
  int plane;
  int m0;       // the frame's first GEMM row
  bool hbm;
  __device__ PScale* amax_sc() const { return base.y.sc; }
  __device__ float store8(int m, int n, const conv::V8& acc, int) const {
    conv::V8 v;
    base.act8(n, acc, v);
    uint32_t h[4], l[4];
    const float mx = conv::split8(v, base.y.w(), h, l);
    const int pp = m - m0, oh = pp / G1::OW, ow = pp - oh * G1::OW;
    const int q = I2::pix(0, oh, ow);
    const int a = q * (2 * I2::C) + 16 * ((n / 8) ^ I2::swz(q));
    *reinterpret_cast<u32x4*>(x1 + a) = u32x4{h[0], h[1], h[2], h[3]};
    *reinterpret_cast<u32x4*>(x1 + plane + a) = u32x4{l[0], l[1], l[2], l[3]};
    if (hbm) {
      const int64_t e = (int64_t)m * G1::CO + n;
      *reinterpret_cast<uint4*>(base.y.p + e) = uint4{h[0], h[1], h[2], h[3]};
      *reinterpret_cast<uint4*>(base.y.p + base.y.stride + e) = uint4{l[0], l[1], l[2], l[3]};
    }
    return mx;
  }
};

template <class G1, class G2, bool U8 = false>
struct P3C12Cfg {
  using I1 = ImgGeomPairs<G1>;
  using I2 = ImgGeom<G2, false>;
  using P1 = conv::P3ConvFwd<G1, 1, U8>;
  using P2 = conv::P3ConvFwd<G2, kPlanes>;
  static constexpr int NP = kPlanes;
  using P1L = P3C1ToLds<G1, G2, U8>;
  static constexpr int NT = 512, BK = 32, KS = 2;
  using C1 = P3Core<512, 32, 8, 1, BK, P1L>;  // 8 waves x 64 rows >= 441
  using C2 = P3Core<128, 64, 4, 2, BK, P2>;   // 4 x 2 waves of 32 x 32 (121 rows)
  using PB1 = PlanP3<32, NT, RCONTIG, NP, BK>;
  using PB2 = PlanP3<64, NT, RCONTIG, NP, BK>;
  static constexpr int FRAME = I1::IMG + 16;  // region 0: frame image + zero unit
  static constexpr int RING1 = FRAME;
  static constexpr int X1 = RING1 + 2 * PB1::BYTES;
  static constexpr int PLANE2 = I2::IMG + 16;
  static constexpr int LDS = X1 + NP * PLANE2;
  static_assert(2 * PB2::BYTES <= I1::IMG && C1::EPI_BYTES <= I1::IMG && C2::EPI_BYTES <= I1::IMG,
                "conv2's ring and the epilogue staging reuse the frame image region");
  static_assert(G1::OPIX <= 512 && I2::OPIX <= 128 && P2::A_PLANES == NP, "geometry");
};

template <class G1, class G2, bool U8>
__global__ void __launch_bounds__(512) gemm_p3c12_kernel(const conv::P3ConvFwd<G1, 1, U8> p1,
                                                         const conv::P3ConvFwd<G2, kPlanes> p2,
                                                         int frames, int hbm_frames) {
  using Cfg = P3C12Cfg<G1, G2, U8>;
  using I1 = typename Cfg::I1;
  using I2 = typename Cfg::I2;
  using PB1 = typename Cfg::PB1;
  using PB2 = typename Cfg::PB2;
  using P1 = typename Cfg::P1;
  using P2 = typename Cfg::P2;
  constexpr int NT = Cfg::NT, BK = Cfg::BK, KS = Cfg::KS, NP = Cfg::NP;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int f = blockIdx.x;
  uint8_t* x1 = smem + Cfg::X1;
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;

  // ---- Weight rings (one unit per owning thread per plane).
  const bool own1 = PB1::owns(tid), own2 = PB2::owns(tid);
  const typename P1::BRow br1 = p1.b_row(own1 ? PB1::row_of(tid) : 0);
  const typename P2::BRow br2 = p2.b_row(own2 ? PB2::row_of(tid) : 0);
  __amdgpu_buffer_rsrc_t sb1[NP], sb2[NP];
#pragma unroll
  for (int pl = 0; pl < NP; ++pl) {
    sb1[pl] = plane_rsrc(p1.b_src, pl);
    sb2[pl] = plane_rsrc(p2.b_src, pl);
  }
  u32x4 r1[2][NP], r2[2][NP];
  auto fetch1 = [&](auto S, int k0) {
    constexpr int set = decltype(S)::value;
    const uint32_t off = own1 && k0 < p1.K ? p1.b_off(br1, k0, PB1::kk_of(tid)) : kOOB;
#pragma unroll
    for (int pl = 0; pl < NP; ++pl)
      r1[set][pl] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(sb1[pl], off, 0, 0));
  };
  auto fetch2 = [&](auto S, int k0) {
    constexpr int set = decltype(S)::value;
    const uint32_t off = own2 && k0 < p2.K ? p2.b_off(br2, k0, PB2::kk_of(tid)) : kOOB;
#pragma unroll
    for (int pl = 0; pl < NP; ++pl)
      r2[set][pl] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(sb2[pl], off, 0, 0));
  };
  auto stash1 = [&](auto S, int buf) {
    constexpr int set = decltype(S)::value;
    if (!own1) return;
    uint8_t* s = smem + Cfg::RING1 + buf * PB1::BYTES;
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) *reinterpret_cast<u32x4*>(s + pl * PB1::PLANE + PB1::offset(tid)) = r1[set][pl];
  };
  auto stash2 = [&](auto S, int buf) {
    constexpr int set = decltype(S)::value;
    if (!own2) return;
    uint8_t* s = smem + buf * PB2::BYTES;
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) *reinterpret_cast<u32x4*>(s + pl * PB2::PLANE + PB2::offset(tid)) = r2[set][pl];
  };
  fetch1(S0{}, 0);
  fetch1(S1{}, BK);
  fetch2(S0{}, 0);
  fetch2(S1{}, BK);

  // ---- The frame image (f16 copy, pixel-pair units), each unit once; zero units.
  if constexpr (AU8<P1>::value) {  // the uint8 frame itself, widened exactly (gemm_p3i.h)
    constexpr int U8U = I1::UNITS / 2;
    constexpr int PER = (U8U + NT - 1) / NT;
    const __amdgpu_buffer_rsrc_t sa = plane_rsrc(p1.a_src, 0);
    u32x4 v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = tid + j * NT;
      const uint32_t off = u < U8U ? (uint32_t)(((int64_t)f * U8U + u) * 16) : kOOB;
      v[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(sa, off, 0, 0));
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = tid + j * NT;
      if (u < U8U) {
        *reinterpret_cast<u32x4*>(smem + I1::fill(0, 2 * u)) = f16x8_of_bytes(v[j][0], v[j][1]);
        *reinterpret_cast<u32x4*>(smem + I1::fill(0, 2 * u + 1)) = f16x8_of_bytes(v[j][2], v[j][3]);
      }
    }
    if (tid == 0) *reinterpret_cast<u32x4*>(smem + Cfg::FRAME - 16) = zero_u4();
    if (tid < NP) *reinterpret_cast<u32x4*>(x1 + tid * Cfg::PLANE2 + Cfg::PLANE2 - 16) = zero_u4();
  } else {
    constexpr int PER = (I1::UNITS + NT - 1) / NT;
    const __amdgpu_buffer_rsrc_t sa = plane_rsrc(p1.a_src, 0);
    u32x4 v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = tid + j * NT;
      const uint32_t off = u < I1::UNITS ? (uint32_t)(((int64_t)f * I1::UNITS + u) * 16) : kOOB;
      v[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(sa, off, 0, 0));
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = tid + j * NT;
      if (u < I1::UNITS) *reinterpret_cast<u32x4*>(smem + I1::fill(0, u)) = v[j];
    }
    if (tid == 0) *reinterpret_cast<u32x4*>(smem + Cfg::FRAME - 16) = zero_u4();
    if (tid < NP) *reinterpret_cast<u32x4*>(x1 + tid * Cfg::PLANE2 + Cfg::PLANE2 - 16) = zero_u4();
  }
  stash1(S0{}, 0);
  __syncthreads();

  // ---- conv1: 8 waves x 64 rows.
  {
    typename I1::Lane ln[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int lr = wave * 64 + i * 32 + (lane & 31);
      ln[i] = I1::lane(0, lr, lr < G1::OPIX);
    }
    typename Cfg::C1::Acc acc;
    acc.zero();
    auto compute = [&](int k0, int buf) {
      const uint8_t* sb = smem + Cfg::RING1 + buf * PB1::BYTES;
      typename I1::Stage sg[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) sg[i] = I1::stage(ln[i], k0);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        f16x8 fb[NP];
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) fb[pl] = PB1::frag(sb, pl, 0, s, lane);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int u = I1::unit(sg[i], ln[i], k0, s, lane >> 5);
          const f16x8 fa[1] = {*reinterpret_cast<const f16x8*>(smem + (u >= 0 ? u : Cfg::FRAME - 16))};
          acc.terms(i, 0, fa, fb);
        }
      }
    };
    auto iter = [&](auto S, int kt) {
      constexpr int set = decltype(S)::value;
      using Other = std::integral_constant<int, set ^ 1>;
      stash1(Other{}, set ^ 1);
      fetch1(S, (kt + 2) * BK);
      compute(kt * BK, set);
      __syncthreads();
    };
    const int nk = p1.K / BK;
    for (int kt = 0; kt < nk; kt += 2) {
      iter(S0{}, kt);
      iter(S1{}, kt + 1);
    }
    typename Cfg::P1L q;
    q.M = (f + 1) * G1::OPIX < p1.M ? (f + 1) * G1::OPIX : p1.M;
    q.N = p1.N; q.K = p1.K; q.k_chunk = p1.k_chunk;
    q.base = p1; q.x1 = x1; q.plane = Cfg::PLANE2; q.m0 = f * G1::OPIX; q.hbm = f < hbm_frames;
    Cfg::C1::epilogue(q, smem, q.m0, 0, wave, wave, 0, lane, 0, acc, false);  // ends on a barrier
  }

  // ---- conv2 on the x1 image: 4 x 2 waves of 32 x 32.
  stash2(S0{}, 0);
  __syncthreads();
  {
    const int wm = wave >> 1, wn = wave & 1;
    const int lr = wm * 32 + (lane & 31);
    const typename I2::Lane ln = I2::lane(0, lr, lr < I2::OPIX);
    typename Cfg::C2::Acc acc;
    acc.zero();
    auto compute = [&](int k0, int buf) {
      const uint8_t* sb = smem + buf * PB2::BYTES;
      const typename I2::Stage sg = I2::stage(ln, k0);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        f16x8 fb[NP];
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) fb[pl] = PB2::frag(sb, pl, wn * 32, s, lane);
        const int u = I2::unit(sg, ln, k0, s, lane >> 5);
        const uint8_t* a = x1 + (u >= 0 ? u : Cfg::PLANE2 - 16);
        f16x8 fa[NP];
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) fa[pl] = *reinterpret_cast<const f16x8*>(a + pl * Cfg::PLANE2);
        acc.terms(0, 0, fa, fb);
      }
    };
    auto iter = [&](auto S, int kt) {
      constexpr int set = decltype(S)::value;
      using Other = std::integral_constant<int, set ^ 1>;
      stash2(Other{}, set ^ 1);
      fetch2(S, (kt + 2) * BK);
      compute(kt * BK, set);
      __syncthreads();
    };
    const int nk = p2.K / BK;
    for (int kt = 0; kt < nk; kt += 2) {
      iter(S0{}, kt);
      iter(S1{}, kt + 1);
    }
    P2 q = p2;
    q.M = (f + 1) * I2::OPIX < p2.M ? (f + 1) * I2::OPIX : p2.M;
    Cfg::C2::epilogue(q, smem, f * I2::OPIX, 0, wave, wm, wn, lane, 0, acc, false);
  }
}

// frames images; x1 planes are written to HBM for frames [0, hbm_frames) only.
template <class G1, class G2, bool U8>
inline hipError_t launch_gemm_p3c12(const conv::P3ConvFwd<G1, 1, U8>& p1,
                                    const conv::P3ConvFwd<G2, kPlanes>& p2, int frames, int hbm_frames,
                                    hipStream_t st) {
  using Cfg = P3C12Cfg<G1, G2, U8>;
  static_assert(Cfg::LDS <= 160 * 1024, "LDS");
  static hipError_t attr = p3_set_lds(&gemm_p3c12_kernel<G1, G2, U8>, Cfg::LDS);
  if (attr != hipSuccess) return attr;
  if (frames < 1 || p1.M != frames * G1::OPIX || p2.M != frames * G2::OPIX || p1.N > 32 ||
      p2.N > 64 || (p1.K / Cfg::BK) % 2 != 0 || (p2.K / Cfg::BK) % 2 != 0)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm_p3c12_kernel<G1, G2, U8>), dim3(frames), dim3(Cfg::NT), Cfg::LDS, st, p1, p2,
                     frames, hbm_frames);
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace acme
