// Image-resident implicit-GEMM convolution on exact bf16 planes (gfx950).
//
// gemm_p3.h reads a convolution's A operand as im2col rows: every input pixel is fetched
// KH*KW/S^2 times (4x for conv2, 9x for conv3) and every fetch goes global -> VGPR -> LDS,
// so the A tile's LDS stores (ds_write_b128 ~79 B/clk/CU, MI355X_MICROARCH.md §LDS) and its
// duplicated L2 reads bound conv2/conv3 (29-34% of the plane-engine ceiling).  Here a block
// owns FPB whole frames: their input image, all three planes, is loaded into LDS ONCE (each
// HBM byte once, each LDS byte stored once), and the MFMA A fragments are read from it
// directly, with the tap offset applied per lane (padding taps read a zero unit).  Only the
// weight panel B (K x BN) streams through the two-stage register-staged LDS ring of
// gemm_p3d.h.  Per 32-k stage a wave issues MT * 2 * 3 ds_read_b128 for A and its NTL B
// fragments per k16 step, against MT * NTL * 2 * 6 MFMAs.
//
// LDS image layout, per plane: pixel q = (frame * H + ih) * W + col, col = iw (stride 1)
// or, for stride 2, the even columns then the odd ones (consecutive output columns, i.e.
// the consecutive rows of an MFMA fragment, read consecutive pixels); the 16-B channel
// chunk c of pixel q sits at chunk c ^ ((q >> SWZ) & (CPX - 1)), CPX chunks per pixel, so
// 16 consecutive pixels' reads of one chunk fall in 16 distinct 4-bank groups (a
// conflict-free ds_read_b128 lane group).  A zero unit follows each plane's image.
#pragma once

#include "gemm_p3.h"

namespace acme {
namespace gemm {

// Image and tap geometry of a convolution GEMM over conv.h's Geom G.  Forward (DGRAD =
// false): the image is the layer input X [IH][IW][CI], GEMM rows are (frame, oh, ow), tap
// (kh, kw) reads (oh*S - PT + kh, ow*S - PL + kw).  Stride-1 input gradient (DGRAD = true):
// the image is dZ [OH][OW][CO], rows are (frame, ih, iw), tap (kh, kw) reads
// (ih + PT - kh, iw + PL - kw).  K is ordered (kh, kw, channel) in both, as conv_p3.h.
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
  static_assert(!DGRAD || G::S == 1, "strided input gradients are not image-resident");
  static_assert(C == 32 || C == 64, "a 32-k stage must stay within one tap");
  static_assert(S == 1 || S == 2, "stride 1 or 2");
  __device__ static __forceinline__ int dh(int kh) { return DGRAD ? G::PT - kh : kh - G::PT; }
  __device__ static __forceinline__ int dw(int kw) { return DGRAD ? G::PL - kw : kw - G::PL; }
  // LDS pixel index of (fr, ih, iw) among the block's frames.
  __device__ static __forceinline__ int pix(int fr, int ih, int iw) {
    return (fr * H + ih) * W + (S == 1 ? iw : (iw & 1) * HALF + (iw >> 1));
  }
  __device__ static __forceinline__ int swz(int q) { return (q >> SWZ) & (CPX - 1); }
  // Byte offset, within a plane, of chunk c of LDS pixel q.
  __device__ static __forceinline__ int addr(int q, int c) { return q * (2 * C) + 16 * (c ^ swz(q)); }
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
  static constexpr int PLANE = FPB * GI::IPIX * 2 * GI::C + 16;  // + the zero unit
  static constexpr int IMG = 3 * PLANE;
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
  constexpr int PLANE = Cfg::PLANE;
  static_assert(P::A_MODE == KCONTIG && P::A_PLANES == 3 && P::B_PLANES == 3,
                "three-plane operands, k-contiguous A");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int f0 = blockIdx.x * FPB;
  const int nf = frames - f0 < FPB ? frames - f0 : FPB;
  const int rows = nf * GI::OPIX;
  const int m0 = f0 * GI::OPIX;
  P p = p_in;
  p.M = m0 + rows < p_in.M ? m0 + rows : p_in.M;  // the epilogue writes this block's rows only
  const int nk = p.K / BK;

  // ---- B: the weight panel, register-staged double buffer (gemm_p3d.h).
  typename P::BRow brow[PB::PER_THREAD];
#pragma unroll
  for (int i = 0; i < PB::PER_THREAD; ++i)
    brow[i] = p.b_row(PB::owns(tid + i * NT) ? PB::row_of(tid + i * NT) : 0);
  __amdgpu_buffer_rsrc_t srcB[3];
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) srcB[pl] = plane_rsrc(p.b_src, pl);
  u32x4 rb[2][PB::PER_THREAD][3];
  auto fetch_b = [&](auto S, int k0) {
    constexpr int set = decltype(S)::value;
#pragma unroll
    for (int i = 0; i < PB::PER_THREAD; ++i) {
      const int u = tid + i * NT;
      const int kk = PB::kk_of(u);
      const uint32_t off = (PB::owns(u) && k0 + kk < p.K) ? p.b_off(brow[i], k0, kk) : kOOB;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
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
      for (int pl = 0; pl < 3; ++pl)
        *reinterpret_cast<u32x4*>(sb + pl * PB::PLANE + off) = rb[set][i][pl];
    }
  };

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  fetch_b(S0{}, 0);
  fetch_b(S1{}, BK);

  // ---- A: the block's frames, each 16-B unit of each plane loaded and stored once.
  {
    constexpr int UNITS = FPB * GI::IPIX * GI::CPX;
    constexpr int PER = (UNITS + NT - 1) / NT;
    __amdgpu_buffer_rsrc_t srcA[3];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) srcA[pl] = plane_rsrc(p.a_src, pl);
    u32x4 v[PER][3];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = tid + j * NT;
      const int f = u / (GI::IPIX * GI::CPX);
      const bool ok = u < UNITS && f < nf;
      // Units are HBM-linear over the block's frames: byte (f0 * IPIX * CPX + u) * 16.
      const uint32_t off = ok ? (uint32_t)(((int64_t)f0 * GI::IPIX * GI::CPX + u) * 16) : kOOB;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        v[j][pl] =
            __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(srcA[pl], off, 0, 0));
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int u = tid + j * NT;
      if (UNITS % NT == 0 || u < UNITS) {
        const int f = u / (GI::IPIX * GI::CPX);
        const int r = u - f * (GI::IPIX * GI::CPX);
        const int px = r / GI::CPX, c = r - px * GI::CPX;
        const int ih = px / GI::W, iw = px - ih * GI::W;
        const int a = GI::addr(GI::pix(f, ih, iw), c);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u32x4*>(smem + pl * PLANE + a) = v[j][pl];
      }
    }
    if (tid < 3) *reinterpret_cast<u32x4*>(smem + tid * PLANE + PLANE - 16) = zero_u4();
  }
  stash_b(S0{}, 0);

  // ---- This lane's GEMM rows (one per 32-row block of the wave's tile).
  int ihs[MT], iws[MT], frs[MT];
  bool rok[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int lr = wm * 32 * MT + i * 32 + (lane & 31);
    const int f = lr / GI::OPIX, pp = lr - f * GI::OPIX;
    const int oh = pp / GI::OW, ow = pp - oh * GI::OW;
    rok[i] = lr < rows;
    ihs[i] = oh * GI::S;
    iws[i] = ow * GI::S;
    frs[i] = f;
  }
  __syncthreads();

  f32x16 acc[MT][NTL];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTL; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  auto compute = [&](int k0, int buf) {
    const uint8_t* sb = smem + Cfg::IMG + buf * Cfg::STAGE_B;
    const int tap = k0 / GI::C;  // wave-uniform: a stage never crosses a tap
    const int kh = tap / GI::KW, kw = tap - kh * GI::KW;
    const int dh = GI::dh(kh), dw = GI::dw(kw);
    const int cb = (k0 - tap * GI::C) >> 3;
    int qb[MT], qs[MT];  // this stage's pixel byte base (-1: padding) and chunk swizzle
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int ih = ihs[i] + dh, iw = iws[i] + dw;
      const bool in = rok[i] && (unsigned)ih < (unsigned)GI::H && (unsigned)iw < (unsigned)GI::W;
      const int q = GI::pix(frs[i], ih, iw);
      qb[i] = in ? q * (2 * GI::C) : -1;
      qs[i] = GI::swz(q);
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      bf16x8 fb[NTL][3];
#pragma unroll
      for (int j = 0; j < NTL; ++j)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) fb[j][pl] = PB::frag(sb, pl, wn * TN + j * 32, s, lane);
      const int c = cb + 2 * s + (lane >> 5);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int a = qb[i] >= 0 ? qb[i] + 16 * (c ^ qs[i]) : PLANE - 16;
        bf16x8 fa[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          fa[pl] = *reinterpret_cast<const bf16x8*>(smem + pl * PLANE + a);
#pragma unroll
        for (int j = 0; j < NTL; ++j) {
          // Smallest terms first, as gemm_p3.h.
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[j][2], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[j][0], acc[i][j], 0, 0, 0);
        }
      }
    }
  };

  // Iteration kt: LDS buffer kt & 1 holds B of stage kt, register set (kt + 1) & 1 holds
  // stage kt + 1 (stashed first: its buffer was last read in iteration kt - 1, before the
  // barrier), then stage kt + 2 is fetched into set kt & 1 (zeros past the end).
  auto iter = [&](auto S, int kt) {
    constexpr int set = decltype(S)::value;
    using Other = std::integral_constant<int, set ^ 1>;
    stash_b(Other{}, set ^ 1);
    fetch_b(S, (kt + 2) * BK);
    compute(kt * BK, set);
    __syncthreads();
  };
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    iter(S0{}, kt);
    iter(S1{}, kt + 1);
  }
  if (kt < nk) iter(S0{}, kt);

  f32x16 cs[C::NCS];
  C::epilogue(p, smem, m0, 0, wave, wm, wn, lane, 0, acc, cs, false);
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
