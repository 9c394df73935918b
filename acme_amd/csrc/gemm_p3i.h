// Image-resident implicit-GEMM convolution on f16 operand planes (gfx950).
//
// gemm_p3.h reads a convolution's A operand as im2col rows: every input pixel is fetched
// KH*KW/S^2 times (4x for conv1 / conv2, 9x for conv3) and every fetch goes global -> VGPR
// -> LDS, so the A
// tile's LDS stores (ds_write_b128 ~79 B/clk/CU, MI355X_MICROARCH.md §LDS) or its TA
// issue bound the convolutions (15-34% of the plane-engine ceiling).  Here a block owns
// FPB whole frames: their input image, every plane, is loaded into LDS ONCE (each HBM
// byte once, each LDS byte stored once), and the MFMA A fragments are read from it
// directly, with the tap offset applied per lane (padding taps read a zero unit).  Only
// the weight panel B (K x BN) streams through a two-stage register-staged LDS ring.
//
// A geometry GI says where each 16-B unit (8 consecutive k of one GEMM row) lives:
//   UNITS            16-B HBM units per frame (frames contiguous in HBM);
//   IMG              LDS bytes of one frame's image (one plane);
//   fill(f, u)       LDS byte offset of HBM unit u of the block's frame f;
//   Lane lane(f, pp, ok)         per-lane state of output pixel pp of frame f;
//   Stage stage(lane, k0)        per 32-k stage (k0 a multiple of 32);
//   int unit(stage, lane, k0, s, h)  byte offset of the lane's unit in k16 step s (lane
//                                    half h), or -1 for padding (the zero unit).
#pragma once

#include "gemm_p3.h"

namespace acme {
namespace gemm {

// Channel-chunk images (conv2 / conv3 forward, stride-1 input gradient) over conv.h's Geom
// G.  Forward (DGRAD = false): the image is the layer input X [IH][IW][CI], GEMM rows are
// (frame, oh, ow), tap (kh, kw) reads (oh*S - PT + kh, ow*S - PL + kw).  Input gradient
// (DGRAD = true, stride 1): the image is dZ [OH][OW][CO], rows are (frame, ih, iw), tap
// (kh, kw) reads (ih + PT - kh, iw + PL - kw).  K is ordered (kh, kw, channel), as
// conv_p3.h; C is 32 or 64, so a 32-k stage stays within one tap.
// LDS layout, per plane: pixel q = (frame * H + ih) * W + col, col = iw (stride 1) or, for
// stride 2, the even columns then the odd ones (consecutive output columns, i.e. the
// consecutive rows of an MFMA fragment, read consecutive pixels); the 16-B channel chunk c
// of pixel q sits at chunk c ^ ((q >> SWZ) & (CPX - 1)), CPX chunks per pixel, so 16
// consecutive pixels' reads of one chunk fall in 16 distinct 4-bank groups.
template <class G, bool DGRAD>
struct ImgGeom {
  static constexpr int H = DGRAD ? G::OH : G::IH, W = DGRAD ? G::OW : G::IW;
  static constexpr int C = DGRAD ? G::CO : G::CI;
  static constexpr int OH = DGRAD ? G::IH : G::OH, OW = DGRAD ? G::IW : G::OW;
  static constexpr int S = DGRAD ? 1 : G::S;
  static constexpr int KW = G::KW;
  static constexpr int OPIX = OH * OW, IPIX = H * W;
  static constexpr int CPX = C / 8;         // 16-B chunks per pixel
  static constexpr int HALF = (W + 1) / 2;  // stride 2: even columns first
  static constexpr int SWZ = CPX == 8 ? 1 : 2;
  static constexpr int UNITS = IPIX * CPX, IMG = IPIX * 2 * C;
  static_assert(!DGRAD || G::S == 1, "strided input gradients are not image-resident");
  static_assert(C == 32 || C == 64, "a 32-k stage must stay within one tap");
  static_assert(S == 1 || S == 2, "stride 1 or 2");
  __device__ static __forceinline__ int dh(int kh) { return DGRAD ? G::PT - kh : kh - G::PT; }
  __device__ static __forceinline__ int dw(int kw) { return DGRAD ? G::PL - kw : kw - G::PL; }
  __device__ static __forceinline__ int pix(int fr, int ih, int iw) {
    return (fr * H + ih) * W + (S == 1 ? iw : (iw & 1) * HALF + (iw >> 1));
  }
  __device__ static __forceinline__ int swz(int q) { return (q >> SWZ) & (CPX - 1); }
  __device__ static __forceinline__ int fill(int f, int u) {
    const int px = u / CPX, c = u - px * CPX;
    const int ih = px / W, iw = px - ih * W;
    const int q = pix(f, ih, iw);
    return q * (2 * C) + 16 * (c ^ swz(q));
  }
  struct Lane {
    int f, ih, iw;
    bool ok;
  };
  __device__ static __forceinline__ Lane lane(int f, int pp, bool ok) {
    const int oh = pp / OW, ow = pp - oh * OW;
    return Lane{f, oh * S, ow * S, ok};
  }
  struct Stage {
    int base, x;  // pixel byte base (-1: padding), chunk swizzle
  };
  __device__ static __forceinline__ Stage stage(const Lane& l, int k0) {
    const int tap = k0 / C;  // wave-uniform
    const int kh = tap / KW, kw = tap - kh * KW;
    const int ih = l.ih + dh(kh), iw = l.iw + dw(kw);
    const bool in = l.ok && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
    const int q = pix(l.f, ih, iw);
    return Stage{in ? q * (2 * C) : -1, swz(q)};
  }
  __device__ static __forceinline__ int unit(const Stage& st, const Lane&, int k0, int s, int h) {
    const int c = ((k0 % C) >> 3) + 2 * s + h;
    return st.base >= 0 ? st.base + 16 * (c ^ st.x) : -1;
  }
};

// Pixel-pair images for a 4-channel input (conv1 over the frames, one plane): a unit is two
// horizontally adjacent pixels x 4 channels, which is exactly the 8 k of one MFMA lane
// (k = (kh, kw, c): kw even, kw + 1) -- 16 B of the f16 frame copy.  A 32-k stage is one
// kernel row kh (KW * CI = 32).  LDS layout: unit (ih, pw) (pw = iw / 2) at (frame * IH +
// ih) * PAIRS + col, col = the even pairs then the odd ones, so stride-S output columns
// read consecutive units (conflict-free ds_read_b128 lane groups).
template <class G>
struct ImgGeomPairs {
  static constexpr int UNIT = 16;  // LDS bytes per unit
  static constexpr int H = G::IH, W = G::IW;
  static constexpr int OW = G::OW, OPIX = G::OPIX;
  static constexpr int PAIRS = W / 2, HALF = (PAIRS + 1) / 2;
  static constexpr int UNITS = H * PAIRS, IMG = UNITS * UNIT;
  static_assert(G::CI == 4 && G::KW * G::CI == 32, "4 channels, one kernel row per stage");
  static_assert(W % 2 == 0 && G::S % 2 == 0 && G::PL % 2 == 0, "pairs never straddle the border");
  __device__ static __forceinline__ int col(int pw) { return (pw & 1) * HALF + (pw >> 1); }
  __device__ static __forceinline__ int fill(int f, int u) {
    const int ih = u / PAIRS, pw = u - ih * PAIRS;
    return ((f * H + ih) * PAIRS + col(pw)) * UNIT;
  }
  struct Lane {
    int f, ih, iw;
    bool ok;
  };
  __device__ static __forceinline__ Lane lane(int f, int pp, bool ok) {
    const int oh = pp / OW, ow = pp - oh * OW;
    return Lane{f, oh * G::S - G::PT, ow * G::S - G::PL, ok};
  }
  struct Stage {
    int base;  // image row byte base (-1: padding row)
  };
  __device__ static __forceinline__ Stage stage(const Lane& l, int k0) {
    const int ih = l.ih + k0 / 32;
    const bool in = l.ok && (unsigned)ih < (unsigned)H;
    return Stage{in ? (l.f * H + ih) * PAIRS * UNIT : -1};
  }
  __device__ static __forceinline__ int unit(const Stage& st, const Lane& l, int, int s, int h) {
    const int iw = l.iw + 4 * s + 2 * h;  // kw = (16 s + 8 h) / 4
    return st.base >= 0 && (unsigned)iw < (unsigned)W ? st.base + col(iw >> 1) * UNIT : -1;
  }
};


template <class GI, int FPB, int BN, int WM, int WN, int MT, class P>
struct P3ICfg {
  static constexpr int BK = 32, KS = 2;
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int TN = BN / WN, NTL = TN / 32;
  static constexpr int BM = WM * 32 * MT;
  static_assert(BM >= FPB * GI::OPIX, "the block's waves must cover its frames' rows");
  static_assert(TN % 32 == 0, "wave panel of whole 32-column MFMA tiles");
  using Core = P3Core<BM, BN, WM, WN, BK, P>;
  using PB = typename Core::PB;
  static constexpr int NPA = P::A_PLANES;
  static constexpr int PLANE = FPB * GI::IMG + 16;  // + the zero unit
  static constexpr int IMG = NPA * PLANE;
  static constexpr int STAGE_B = PB::BYTES;
  static constexpr int MAIN = IMG + 2 * STAGE_B;
  static constexpr int LDS = MAIN > Core::EPI_BYTES ? MAIN : Core::EPI_BYTES;
};

template <class GI, int FPB, int BN, int WM, int WN, int MT, class P>
__global__ void __launch_bounds__(64 * WM * WN) gemm_p3i_kernel(const P p_in, int frames) {
  using Cfg = P3ICfg<GI, FPB, BN, WM, WN, MT, P>;
  using C = typename Cfg::Core;
  using PB = typename Cfg::PB;
  constexpr int NT = Cfg::NT, NTL = Cfg::NTL, TN = Cfg::TN, BK = Cfg::BK, KS = Cfg::KS;
  constexpr int PLANE = Cfg::PLANE, NPA = Cfg::NPA;
  constexpr int NPB = kPlanes;
  static_assert(P::A_MODE == KCONTIG && (NPA == 1 || NPA == kPlanes) && P::B_PLANES == NPB,
                "k-contiguous A (one or two planes), two-plane B");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  // Phase stamps (timing experiment, as gemm_p3ws_kernel's): entry, after the image fill's
  // barrier, after the k loop, exit.
  uint64_t st_rt0 = 0, st_t0 = 0, st_t1 = 0, st_t2 = 0;
  bool stamp = false;
  if constexpr (HasStamps<P>::value) {
    stamp = p_in.stamps != nullptr && tid == 0;
    if (stamp) {
      st_rt0 = __builtin_amdgcn_s_memrealtime();
      st_t0 = __builtin_amdgcn_s_memtime();
    }
  }
  const int f0 = blockIdx.x * FPB;
  const int nf = frames - f0 < FPB ? frames - f0 : FPB;
  const int rows = nf * GI::OPIX;
  const int m0 = f0 * GI::OPIX;
  P p = p_in;
  p.M = m0 + rows < p_in.M ? m0 + rows : p_in.M;  // the epilogue writes this block's rows only
  const int nk = p.K / BK;

  // ---- B: the weight panel, register-staged double buffer.
  typename P::BRow brow[PB::PER_THREAD];
#pragma unroll
  for (int i = 0; i < PB::PER_THREAD; ++i)
    brow[i] = p.b_row(PB::owns(tid + i * NT) ? PB::row_of(tid + i * NT) : 0);
  __amdgpu_buffer_rsrc_t srcB[NPB];
#pragma unroll
  for (int pl = 0; pl < NPB; ++pl) srcB[pl] = plane_rsrc(p.b_src, pl);
  // Two register sets (round 5: a third, loads two iterations ahead, measured slower on the
  // step: 0.4949 -> 0.5011 ms).
  constexpr int RS = 2;
  u32x4 rb[RS][PB::PER_THREAD][NPB];
  auto fetch_b = [&](auto S, int k0) {
    constexpr int set = decltype(S)::value;
#pragma unroll
    for (int i = 0; i < PB::PER_THREAD; ++i) {
      const int u = tid + i * NT;
      const int kk = PB::kk_of(u);
      const uint32_t off = (PB::owns(u) && k0 + kk < p.K) ? p.b_off(brow[i], k0, kk) : kOOB;
#pragma unroll
      for (int pl = 0; pl < NPB; ++pl)
        rb[set][i][pl] =
            __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(srcB[pl], off, 0, 0));
    }
  };
  auto stash_b = [&](auto S, int buf) {
    constexpr int set = decltype(S)::value;
    uint8_t* sb = smem + Cfg::IMG + buf * Cfg::STAGE_B;
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

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  fetch_b(S0{}, 0);
  fetch_b(S1{}, BK);

  // ---- A: the block's frames, each unit of each plane loaded and stored once.
  constexpr int UB = 16;  // bytes per unit
  using UT = u32x4;
  if constexpr (AU8<P>::value) {
    // The uint8 frames themselves: a 16-B load holds two f16 units (units 2u, 2u + 1 of the
    // same image row), widened exactly; frames from a_src, or from a_src2 past a_split.
    static_assert(FPB == 1 && NPA == 1 && GI::UNITS % 2 == 0, "uint8 frames: one per block");
    constexpr int U8U = GI::UNITS / 2;
    constexpr int PER = (U8U + NT - 1) / NT;
    const bool second = f0 >= p.a_split;
    const __amdgpu_buffer_rsrc_t sa = plane_rsrc(second ? p.a_src2 : p.a_src, 0);
    const int fl = second ? f0 - p.a_split : f0;
    u32x4 v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = tid + j * NT;
      const uint32_t off = u < U8U ? (uint32_t)(((int64_t)fl * U8U + u) * 16) : kOOB;
      v[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(sa, off, 0, 0));
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = tid + j * NT;
      if (U8U % NT == 0 || u < U8U) {
        *reinterpret_cast<u32x4*>(smem + GI::fill(0, 2 * u)) = f16x8_of_bytes(v[j][0], v[j][1]);
        *reinterpret_cast<u32x4*>(smem + GI::fill(0, 2 * u + 1)) = f16x8_of_bytes(v[j][2], v[j][3]);
      }
    }
    if (tid == 0) *reinterpret_cast<u32x4*>(smem + PLANE - 16) = zero_u4();
  } else {
    constexpr int UNITS = FPB * GI::UNITS;
    constexpr int PER = (UNITS + NT - 1) / NT;
    __amdgpu_buffer_rsrc_t srcA[NPA];
#pragma unroll
    for (int pl = 0; pl < NPA; ++pl) srcA[pl] = plane_rsrc(p.a_src, pl);
    UT v[PER][NPA];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = tid + j * NT;
      const int f = u / GI::UNITS;
      const bool ok = u < UNITS && f < nf;
      // Units are HBM-linear over the block's frames: byte (f0 * UNITS + u) * UB.
      const uint32_t off = ok ? (uint32_t)(((int64_t)f0 * GI::UNITS + u) * UB) : kOOB;
#pragma unroll
      for (int pl = 0; pl < NPA; ++pl) {
        v[j][pl] = __builtin_bit_cast(UT, __builtin_amdgcn_raw_buffer_load_b128(srcA[pl], off, 0, 0));
      }
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = tid + j * NT;
      if (UNITS % NT == 0 || u < UNITS) {
        const int f = u / GI::UNITS;
        const int a = GI::fill(f, u - f * GI::UNITS);
#pragma unroll
        for (int pl = 0; pl < NPA; ++pl) *reinterpret_cast<UT*>(smem + pl * PLANE + a) = v[j][pl];
      }
    }
    if (tid < NPA) *reinterpret_cast<u32x4*>(smem + tid * PLANE + PLANE - 16) = zero_u4();
  }
  stash_b(S0{}, 0);

  // ---- This lane's GEMM rows (one per 32-row block of the wave's tile).
  typename GI::Lane ln[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int lr = wm * 32 * MT + i * 32 + (lane & 31);
    const int f = lr / GI::OPIX;
    ln[i] = GI::lane(f, lr - f * GI::OPIX, lr < rows);
  }
  __syncthreads();
  if constexpr (HasStamps<P>::value)
    if (stamp) st_t1 = __builtin_amdgcn_s_memtime();

  typename C::Acc acc;
  acc.zero();
  // The epilogue's constants, loaded now (their latency hides under the k loop).
  typename EpiPre<P>::type pre{};
  if constexpr (EpiPre<P>::has) pre = p.pre(wn * TN + C::epi_col(lane));

  auto compute = [&](int k0, int buf) {
    const uint8_t* sb = smem + Cfg::IMG + buf * Cfg::STAGE_B;
    typename GI::Stage sg[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) sg[i] = GI::stage(ln[i], k0);
    // Every fragment of the stage read first, then the MFMAs (fenced): one LDS latency per
    // stage instead of one per k16 step (the scheduler otherwise sinks each read to its first
    // use; round 5: step 0.4969 -> 0.4949 ms with the fences here and in iter below).
    f16x8 fb[KS][NTL][NPB], fa[KS][MT][NPA];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int j = 0; j < NTL; ++j)
#pragma unroll
        for (int pl = 0; pl < NPB; ++pl) fb[s][j][pl] = PB::frag(sb, pl, wn * TN + j * 32, s, lane);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int u = GI::unit(sg[i], ln[i], k0, s, lane >> 5);
        const int a = u >= 0 ? u : PLANE - 16;
#pragma unroll
        for (int pl = 0; pl < NPA; ++pl)
          fa[s][i][pl] = *reinterpret_cast<const f16x8*>(smem + pl * PLANE + a);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j) acc.terms(i, j, fa[s][i], fb[s][j]);
  };

  // Iteration kt: LDS buffer kt & 1 holds B of stage kt, register set (kt + 1) % RS holds
  // stage kt + 1 (stashed first into buffer (kt + 1) & 1: last read in iteration kt - 1,
  // before the barrier), then stage kt + RS is fetched into set kt % RS (zeros past the end).
  auto iter = [&](auto S, int kt) {
    constexpr int set = decltype(S)::value;
    using Next = std::integral_constant<int, (set + 1) % RS>;
    stash_b(Next{}, (kt + 1) & 1);
    fetch_b(S, (kt + RS) * BK);
    // The weight loads issue before the MFMAs (fenced), so they have the whole iteration
    // to land before the next iteration stores them (round 5: the scheduler had sunk them
    // to just before the barrier, and the next store waited out their latency).
    __builtin_amdgcn_sched_barrier(0);
    compute(kt * BK, kt & 1);
    __syncthreads();
  };
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    iter(S0{}, kt);
    iter(S1{}, kt + 1);
  }
  if (kt < nk) iter(S0{}, kt);

  if constexpr (HasStamps<P>::value)
    if (stamp) st_t2 = __builtin_amdgcn_s_memtime();
  C::epilogue(p, smem, m0, 0, wave, wm, wn, lane, 0, acc, false, &pre);
  if constexpr (HasStamps<P>::value) {
    if (stamp) {
      uint64_t* o = p_in.stamps + 8 * (int64_t)blockIdx.x;
      o[0] = st_rt0;
      o[1] = __builtin_amdgcn_s_memrealtime();
      o[2] = st_t0;
      o[3] = st_t1;
      o[4] = st_t2;
      o[5] = __builtin_amdgcn_s_memtime();
    }
  }
}

// frames: the number of images (p.M = frames * GI::OPIX rows).
template <class GI, int FPB, int BN, int WM, int WN, int MT, class P>
inline hipError_t launch_gemm_p3i(const P& p, int frames, hipStream_t st) {
  using Cfg = P3ICfg<GI, FPB, BN, WM, WN, MT, P>;
  static_assert(Cfg::LDS <= 160 * 1024, "image + two B stages must fit the 160-KiB LDS");
  static hipError_t attr = p3_set_lds(&gemm_p3i_kernel<GI, FPB, BN, WM, WN, MT, P>, Cfg::LDS);
  if (attr != hipSuccess) return attr;
  if (p.N > BN || p.M != frames * GI::OPIX || p.K % Cfg::BK != 0) return hipErrorInvalidValue;
  const int blocks = (frames + FPB - 1) / FPB;
  hipLaunchKernelGGL((gemm_p3i_kernel<GI, FPB, BN, WM, WN, MT, P>), dim3(blocks), dim3(Cfg::NT),
                     Cfg::LDS, st, p, frames);
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace acme
