// Image-resident stride-1 convolution weight gradient (conv3) on exact bf16 planes (gfx950).
//
// dW[tap][ci][co] = sum over frames and output pixels p of X[p + tap][ci] * dZ[p][co].  The
// im2col engine streams X's im2col^T and dZ through LDS per (tile, split) with 15 k-stages
// per block, so each block is mostly prologue / epilogue (24% of the ceiling).  Here a
// block owns FPB frames, one after another: the frame's X image and dZ image (all three
// planes each) are loaded into LDS once, and wave w = filter tap w owns dW[w] (64 x 64:
// 2 x 2 MFMA tiles), reading both operands with the gfx950 transpose read
// (ds_read_b64_tr_b16: 4 channels of one pixel per lane, transposed so a lane holds 8
// pixels of one channel) -- the X read for output pixel p goes to pixel p + tap (or a
// zero row).  Wave 0 also forms the bias gradient (column sums of dZ, one ones-fragment
// MFMA per plane).  Per frame: 8 k16 steps (121 pixels) x 24 MFMAs per wave.  The block's
// partial dW goes to its split-K slab row, reduced by the usual deterministic pass.
//
// Image layout ([pixel][channel], 128 B per pixel and plane): the 16-B channel chunk c of
// pixel q sits at chunk c ^ (4 * ((q >> 1) & 1)), so the four consecutive pixels of a
// transpose-read lane group hit four disjoint 16-bank ranges.
#pragma once

#include "conv_p3.h"
#include "gemm_p3.h"

namespace acme {
namespace gemm {

template <class G, int FPB>
struct P3WCfg {
  using P = conv::P3ConvWgrad<G, 3>;
  static constexpr int C = G::CI, CO = G::CO, TAPS = G::KH * G::KW;
  static constexpr int NW = TAPS, NT = 64 * NW;
  static constexpr int PIX = G::OPIX;                    // output pixels = dZ rows
  static constexpr int STEPS = (PIX + 15) / 16;          // k16 steps per frame
  static constexpr int IMG = G::IPIX * 2 * C;            // one plane of X
  static constexpr int DZ = PIX * 2 * CO;                // one plane of dZ
  static constexpr int XPL = IMG + 16, DPL = DZ + 16;    // + zero row (pixel-sized, 16 B used)
  static constexpr int X0 = 0, D0 = 3 * XPL;
  static constexpr int LDS_MAIN = D0 + 3 * DPL;
  using Core = P3Core<64 * TAPS, CO, TAPS, 1, 32, P>;  // wave w: rows [64 w, 64 w + 64)
  static constexpr int LDS = LDS_MAIN > Core::EPI_BYTES ? LDS_MAIN : Core::EPI_BYTES;
  static_assert(C == 64 && CO == 64 && G::S == 1, "conv3 geometry (64 -> 64, stride 1)");
  __device__ static __forceinline__ int chunk(int q, int c) { return c ^ (((q >> 1) & 1) << 2); }
};

template <class G, int FPB>
__global__ void __launch_bounds__(64 * G::KH * G::KW) gemm_p3w_kernel(
    const conv::P3ConvWgrad<G, 3> p, int frames) {
  using Cfg = P3WCfg<G, FPB>;
  using C = typename Cfg::Core;
  constexpr int NT = Cfg::NT;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kh = wave / G::KW, kw = wave - kh * G::KW;   // this wave's tap
  const int dh = kh - G::PT, dw = kw - G::PL;
  const bool colsum = wave == 0;
  const __amdgpu_buffer_rsrc_t sx[3] = {plane_rsrc(p.a_src, 0), plane_rsrc(p.a_src, 1),
                                        plane_rsrc(p.a_src, 2)};
  const __amdgpu_buffer_rsrc_t sd[3] = {plane_rsrc(p.b_src, 0), plane_rsrc(p.b_src, 1),
                                        plane_rsrc(p.b_src, 2)};
  if (tid < 3) {
    *reinterpret_cast<u32x4*>(smem + Cfg::X0 + tid * Cfg::XPL + Cfg::IMG) = zero_u4();
    *reinterpret_cast<u32x4*>(smem + Cfg::D0 + tid * Cfg::DPL + Cfg::DZ) = zero_u4();
  }
  const bf16x8 ones{(__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f,
                    (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f};
  f32x16 acc[2][2], cs[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) cs[j][e] = 0.f;

  for (int fi = 0; fi < FPB; ++fi) {
    const int f = blockIdx.x * FPB + fi;
    if (f >= frames) break;  // block-uniform
    // ---- the frame's X and dZ images (8 channels = one 16-B unit, each once per plane).
    {
      constexpr int XU = G::IPIX * 8, DU = Cfg::PIX * 8;  // units per plane
      constexpr int PX = (XU + NT - 1) / NT, PD = (DU + NT - 1) / NT;
      u32x4 vx[PX][3], vd[PD][3];
#pragma unroll
      for (int j = 0; j < PX; ++j) {
        const int u = tid + j * NT;
        const uint32_t off = u < XU ? (uint32_t)(((int64_t)f * XU + u) * 16) : kOOB;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          vx[j][pl] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(sx[pl], off, 0, 0));
      }
#pragma unroll
      for (int j = 0; j < PD; ++j) {
        const int u = tid + j * NT;
        const uint32_t off = u < DU ? (uint32_t)(((int64_t)f * DU + u) * 16) : kOOB;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          vd[j][pl] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(sd[pl], off, 0, 0));
      }
      if (fi > 0) __syncthreads();  // the previous frame's fragment reads are done
#pragma unroll
      for (int j = 0; j < PX; ++j) {
        const int u = tid + j * NT;
        if (u < XU) {
          const int q = u >> 3, c = u & 7;
          const int a = q * 128 + 16 * Cfg::chunk(q, c);
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            *reinterpret_cast<u32x4*>(smem + Cfg::X0 + pl * Cfg::XPL + a) = vx[j][pl];
        }
      }
#pragma unroll
      for (int j = 0; j < PD; ++j) {
        const int u = tid + j * NT;
        if (u < DU) {
          const int q = u >> 3, c = u & 7;
          const int a = q * 128 + 16 * Cfg::chunk(q, c);
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            *reinterpret_cast<u32x4*>(smem + Cfg::D0 + pl * Cfg::DPL + a) = vd[j][pl];
        }
      }
      __syncthreads();
    }
    // ---- 8 k16 steps over the frame's output pixels.  A lane's transpose reads touch
    // step pixels k0 = 8h + qq and k0 + 4 (as PlanP3's row-contiguous fragments) and
    // channels 16g + 4pp (+ 32 for the second row block): the pixel arithmetic is done
    // once per step, the chunk arithmetic once per lane.
    {
      const int h = lane >> 5, g = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;
      const int cbase = 2 * g + (pp >> 1), cbyte = 8 * (pp & 1);
      typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
      auto rd = [&](const uint8_t* img, const uint8_t* zero, int q, int i) -> i16x4 {
        const uint8_t* a =
            q < 0 ? zero : img + q * 128 + 16 * Cfg::chunk(q, 4 * i + cbase) + cbyte;
        return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)a);
      };
#pragma unroll 2
      for (int s = 0; s < Cfg::STEPS; ++s) {
        int qx[2], qd[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int pz = 16 * s + 8 * h + qq + 4 * t;
          const int oh = pz / G::OW, ow = pz - oh * G::OW;
          const int ih = oh + dh, iw = ow + dw;
          const bool in = pz < Cfg::PIX;
          qx[t] = in && (unsigned)ih < (unsigned)G::IH && (unsigned)iw < (unsigned)G::IW
                      ? ih * G::IW + iw : -1;
          qd[t] = in ? pz : -1;
        }
        bf16x8 fa[2][3], fb[2][3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          const uint8_t* xi = smem + Cfg::X0 + pl * Cfg::XPL;
          const uint8_t* di = smem + Cfg::D0 + pl * Cfg::DPL;
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const i16x4 xl = rd(xi, xi + Cfg::IMG, qx[0], i), xh = rd(xi, xi + Cfg::IMG, qx[1], i);
            const i16x4 dl = rd(di, di + Cfg::DZ, qd[0], i), dhh = rd(di, di + Cfg::DZ, qd[1], i);
            const __attribute__((ext_vector_type(8))) short vx{xl[0], xl[1], xl[2], xl[3],
                                                               xh[0], xh[1], xh[2], xh[3]};
            const __attribute__((ext_vector_type(8))) short vd{dl[0], dl[1], dl[2], dl[3],
                                                               dhh[0], dhh[1], dhh[2], dhh[3]};
            fa[i][pl] = __builtin_bit_cast(bf16x8, vx);
            fb[i][pl] = __builtin_bit_cast(bf16x8, vd);
          }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            // Smallest terms first, as gemm_p3.h.
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][1], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], fb[j][0], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][2], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][0], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][1], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][0], acc[i][j], 0, 0, 0);
          }
        if (colsum) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int pl = 2; pl >= 0; --pl)
              cs[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, fb[j][pl], cs[j], 0, 0, 0);
        }
      }
    }
  }
  __syncthreads();  // the LDS becomes the epilogue's staging area
  C::epilogue(p, smem, 0, 0, wave, wave, 0, lane, blockIdx.x, acc, cs, colsum);
}

// splits = ceil(frames / FPB) slab rows (p.slab holds that many [M + 1][N] partials).
template <class G, int FPB>
inline hipError_t launch_gemm_p3w(const conv::P3ConvWgrad<G, 3>& p, int frames, hipStream_t st) {
  using Cfg = P3WCfg<G, FPB>;
  static_assert(Cfg::LDS <= 160 * 1024, "X and dZ images must fit the LDS");
  static hipError_t attr = p3_set_lds(&gemm_p3w_kernel<G, FPB>, Cfg::LDS);
  if (attr != hipSuccess) return attr;
  if (frames < 1 || p.M != G::K || p.N != G::CO) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm_p3w_kernel<G, FPB>), dim3((frames + FPB - 1) / FPB), dim3(Cfg::NT),
                     Cfg::LDS, st, p, frames);
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace acme
