// Register-operand f32 GEMM for small layers (D4PG's LayerNormMLP widths: a few hundred
// rows, K <= 1024).  The staged engine (gemm.h) moves each k-group's operands through LDS
// in BK-wide stages, one global-load round trip per stage; at these sizes the step is that
// chain of round trips.  Here every lane loads its whole share of the reduction straight
// into registers in one burst and feeds the f32 MFMA from them: one round trip per block.
//
// One block = one 32 x 32 output tile, NW waves.  v_mfma_f32_32x32x2_f32 takes
// A[m = lane & 31][k = lane >> 5] and B[k = lane >> 5][n = lane & 31]; lane half h of wave w
// owns the k run [w * 2KL + h * KL, + KL) (then + NW * 2KL, ...), so MFMA t pairs the two
// halves' t-th elements — both operands of one product come from the same lane and index,
// which is all the instruction's k slot requires.  The waves' 32 x 32 partials are summed
// through LDS in wave order; wave w then finishes rows v = 2w, 2w + 1 of the C map (the
// epilogue is spread over the block instead of run by one wave).
//
// Problems follow gemm.h's concept with A_MODE = B_MODE = KCONTIG: a_load(ARow, k) /
// b_load(BRow, k) return elements k .. k+3 of one row (zeros past M / N; the caller
// guards k < K, so VEC loaders stay unconditional), store / pre-finish-put as in
// store_tile, colsum through store_colsum.
#pragma once

#include "gemm.h"

namespace acme {
namespace gemm {

constexpr int kDirectWaves = 8;

// Optional strided-operand hook: a problem with `static constexpr bool kStrided = true`
// describes each operand as one buffer, element (row, k) at byte offset
// row * row_bytes + k * k_bytes (VEC: k_bytes = 4, rows 16-byte aligned, loaded 4 k at a
// time), and the direct block reads whole chunks with buffer loads — one VGPR offset per
// lane, the k step in the scalar offset, no branch per load.  Offsets past `bytes` read zero
// (rows >= M of a row-major operand); rows past N of a column operand may read neighbouring
// elements, which reach only output columns that are never stored.  Elements past K read
// zero (their offsets are pushed past the buffer).
// (StridedOp: gemm.h.)
template <class P, class = void>
struct HasStrided {
  static constexpr bool value = false;
};
template <class P>
struct HasStrided<P, decltype(void(P::kStrided))> {
  static constexpr bool value = P::kStrided;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t strided_rsrc(const StridedOp& o) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(o.base), (short)0, o.bytes,
                                           0x00020000);
}

// KL / 4 vectors of elements k0 .. k0 + KL - 1 of `row`; elements at k >= K read zero (their
// offset is pushed past the buffer; VEC operands have K % 4 == 0).
template <int KL, bool VEC>
__device__ __forceinline__ void strided_run(const StridedOp& o, __amdgpu_buffer_rsrc_t rs, int row,
                                            int k0, int K, f32x4 (&out)[KL / 4]) {
  constexpr uint32_t kOut = 0x80000000u;
  const uint32_t off = (uint32_t)row * o.row_bytes + (uint32_t)k0 * o.k_bytes;
  if constexpr (VEC) {
#pragma unroll
    for (int i = 0; i < KL / 4; ++i)
      out[i] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, k0 + 4 * i < K ? off + 16 * i : kOut, 0, 0));
  } else {
#pragma unroll
    for (int i = 0; i < KL / 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        out[i][j] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rs, k0 + 4 * i + j < K ? off : kOut,
                                                        (4 * i + j) * o.k_bytes, 0));
  }
}

// LDS floats of a direct block: NW partial 32 x 32 tiles plus NW x 64 column-sum lanes.
template <int NW>
constexpr int direct_smem_floats() {
  return NW * 16 * 64 + NW * 64;
}

template <int KL, int NW, class P>
__device__ __forceinline__ void direct_block(const P& p, const int tile, float* __restrict__ smem) {
  static_assert(P::A_MODE == KCONTIG && P::B_MODE == KCONTIG, "direct GEMM: k-contiguous loaders");
  static_assert(KL % 4 == 0 && 16 % NW == 0, "direct GEMM shape");
  constexpr int VPW = 16 / NW;  // C-map rows finished per wave
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int tiles_n = (p.N + 31) / 32;
  const int m0 = (tile / tiles_n) * 32, n0 = (tile % tiles_n) * 32;
  if (m0 >= p.M) return;  // block-uniform, before any barrier

  // The epilogue's own loads (bias, activation masks) go out first: they are independent
  // of the product and retire under the operand burst.
  float pre[VPW];
  if constexpr (HasPreStore<P>::value) {
#pragma unroll
    for (int j = 0; j < VPW; ++j) {
      const int v = w * VPW + j;
      const int m = m0 + (v & 3) + 8 * (v >> 2) + 4 * h;
      const int n = n0 + r;
      pre[j] = p.pre(m < p.M ? m : p.M - 1, n < p.N ? n : p.N - 1);
    }
  }

  const typename P::ARow ar = p.a_row(m0 + r);
  const typename P::BRow br = p.b_row(n0 + r);
  f32x16 acc;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
  constexpr bool kColSum = HasColSum<P>::value;
  const bool do_colsum = kColSum && m0 == 0;
  float cs = 0.f;
  StridedOp oa{}, ob{};
  if constexpr (HasStrided<P>::value) {
    oa = p.a_op();
    ob = p.b_op();
  }
  const __amdgpu_buffer_rsrc_t ra = strided_rsrc(oa), rb = strided_rsrc(ob);
  for (int kb = w * 2 * KL; kb < p.K; kb += NW * 2 * KL) {
    const int k0 = kb + h * KL;
    f32x4 a[KL / 4], b[KL / 4];
    if constexpr (HasStrided<P>::value) {
      strided_run<KL, P::kAVec>(oa, ra, m0 + r, k0, p.K, a);
      strided_run<KL, P::kBVec>(ob, rb, n0 + r, k0, p.K, b);
    } else {
#pragma unroll
      for (int i = 0; i < KL / 4; ++i) {
        const bool in = k0 + 4 * i < p.K;
        a[i] = in ? p.a_load(ar, k0 + 4 * i) : zero4();
        b[i] = in ? p.b_load(br, k0 + 4 * i) : zero4();
      }
    }
    // Every load of the chunk is issued before the first product: left alone, the scheduler
    // interleaves them with the MFMAs to save registers and keeps only ~8 in flight.
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < KL / 4; ++i)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][t], b[i][t], acc, 0, 0, 0);
    if constexpr (kColSum) {
      if (do_colsum) {
#pragma unroll
        for (int i = 0; i < KL / 4; ++i) cs += (b[i][0] + b[i][1]) + (b[i][2] + b[i][3]);
      }
    }
  }

  // Partials in wave order: smem[(w * 16 + v) * 64 + lane]; column sums after them.
  float* cs_red = smem + NW * 16 * 64;
#pragma unroll
  for (int v = 0; v < 16; ++v) smem[(w * 16 + v) * 64 + lane] = acc[v];
  if constexpr (kColSum) cs_red[w * 64 + lane] = cs;
  __syncthreads();
  float out[VPW];
#pragma unroll
  for (int j = 0; j < VPW; ++j) {
    const int v = w * VPW + j;
    float s = smem[v * 64 + lane];
#pragma unroll
    for (int g = 1; g < NW; ++g) s += smem[(g * 16 + v) * 64 + lane];
    out[j] = s;
  }
#pragma unroll
  for (int j = 0; j < VPW; ++j) {
    const int v = w * VPW + j;
    const int m = m0 + (v & 3) + 8 * (v >> 2) + 4 * h;
    const int n = n0 + r;
    if constexpr (HasPreStore<P>::value) {
      const float y = p.finish(out[j], pre[j]);
      if (m < p.M && n < p.N) p.put(m, n, y, 0);
    } else {
      if (m < p.M && n < p.N) p.store(m, n, out[j], 0);
    }
  }
  if constexpr (kColSum) {
    // Column n0 + t: lanes t and t + 32 of every wave, summed in wave order.
    if (do_colsum && w == 0 && lane < 32 && n0 + lane < p.N) {
      float s = 0.f;
#pragma unroll
      for (int g = 0; g < NW; ++g) s += cs_red[g * 64 + lane] + cs_red[g * 64 + lane + 32];
      p.store_colsum(n0 + lane, s, 0);
    }
  }
}

template <int KL, int NW, class P>
__global__ void __launch_bounds__(64 * NW) gemm_direct_kernel(const P p_in) {
  __shared__ __attribute__((aligned(16))) float smem[direct_smem_floats<NW>()];
  const P p = z_select(p_in);
  direct_block<KL, NW>(p, blockIdx.x, smem);
}

// Optional non-GEMM member of a multi launch: a problem with `static constexpr bool kCustom =
// true` runs p.run_block(blockIdx.x, smem) (64 NW threads, direct_smem_floats<NW>() floats of
// LDS) instead of a GEMM tile; its M x N in 32 x 32 tiles sizes the launch's grid.
template <class P, class = void>
struct HasCustomBlock {
  static constexpr bool value = false;
};
template <class P>
struct HasCustomBlock<P, decltype(void(P::kCustom))> {
  static constexpr bool value = P::kCustom;
};

template <int KL, int NW, class S0, class... R>
__device__ __forceinline__ void direct_multi_run(const ZMulti<S0, R...>& q, int z, float* smem) {
  if (z < q.n) {
    const S0 p = q.s.for_z(z);
    if constexpr (HasCustomBlock<S0>::value) p.run_block(blockIdx.x, smem);
    else direct_block<KL, NW>(p, blockIdx.x, smem);
  } else if constexpr (sizeof...(R) > 0) {
    direct_multi_run<KL, NW>(q.rest, z - q.n, smem);
  }
}

template <int KL, int NW, class... S>
__global__ void __launch_bounds__(64 * NW) gemm_direct_multi_kernel(const ZMulti<S...> q) {
  __shared__ __attribute__((aligned(16))) float smem[direct_smem_floats<NW>()];
  direct_multi_run<KL, NW>(q, blockIdx.z, smem);
}

// k elements per lane per pass for reduction length K over NW waves: the smallest of
// 4, 8, 16, 32 that covers K in one pass, else 32 (more passes).
inline int direct_kl(int K, int NW = kDirectWaves) {
  for (int kl = 4; kl < 32; kl *= 2)
    if (NW * 2 * kl >= K) return kl;
  return 32;
}

// One launch over p's tiles (z sub-problems when P is a ZSet: grid z = nz).
template <class P>
inline hipError_t launch_direct(const P& p, int nz, int K, hipStream_t st) {
  constexpr int NW = kDirectWaves;
  const dim3 grid((unsigned)(((p.N + 31) / 32) * ((p.M + 31) / 32)), 1, (unsigned)nz);
  const dim3 block(64 * NW);
  switch (direct_kl(K)) {
    case 4: hipLaunchKernelGGL((gemm_direct_kernel<4, NW, P>), grid, block, 0, st, p); break;
    case 8: hipLaunchKernelGGL((gemm_direct_kernel<8, NW, P>), grid, block, 0, st, p); break;
    case 16: hipLaunchKernelGGL((gemm_direct_kernel<16, NW, P>), grid, block, 0, st, p); break;
    default: hipLaunchKernelGGL((gemm_direct_kernel<32, NW, P>), grid, block, 0, st, p); break;
  }
  return hipGetLastError();
}

template <class... S>
inline hipError_t launch_direct_multi(const ZMulti<S...>& q, int tiles, int count, int K,
                                      hipStream_t st) {
  constexpr int NW = kDirectWaves;
  const dim3 grid((unsigned)tiles, 1, (unsigned)count), block(64 * NW);
  switch (direct_kl(K)) {
    case 4: hipLaunchKernelGGL((gemm_direct_multi_kernel<4, NW, S...>), grid, block, 0, st, q); break;
    case 8: hipLaunchKernelGGL((gemm_direct_multi_kernel<8, NW, S...>), grid, block, 0, st, q); break;
    case 16: hipLaunchKernelGGL((gemm_direct_multi_kernel<16, NW, S...>), grid, block, 0, st, q); break;
    default: hipLaunchKernelGGL((gemm_direct_multi_kernel<32, NW, S...>), grid, block, 0, st, q); break;
  }
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace acme
