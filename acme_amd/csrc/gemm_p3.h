// Plane-operand GEMM engine (gfx950 / CDNA4): f32 GEMMs whose operands are ALREADY
// stored in HBM as exact-to-f32-rounding f16 planes, so the main loop is plain f16 MFMA work.
//
// An f32 tensor x is kept as two f16 arrays h, l of its scaled value y = x * w:
// h = f16(y), l = f16(y - h) (11 + 11 significant bits, each rounding to nearest, so
// |y - h - l| <= 2^-24 |y|: the representation error of an f32 rounding).  w is a power of
// two chosen per tensor (PScale) so that the tensor's largest element sits at 2^7..2^8,
// 2^8 below f16's overflow; every element within 2^-10 of the maximum then keeps the full
// 2^-24 relative precision and smaller ones an absolute error <= 2^-33 max|x| (f16
// subnormals), far below an f32 dot product's own rounding error.  Scaling by a power of
// two commutes with every rounding, so the results do not depend on w.
// The product a b is the three f16 MFMA terms hl, lh, hh (smallest first, f32
// accumulation; the dropped ll is <= 2^-22 |ab| before rounding and below the f32
// accumulation's own error), and the consumer multiplies its f32 result by
// 1 / (w_a w_b) (exact).  An operand that is exactly an f16 value (the uint8 Atari frames:
// integers 0..255) is ONE unscaled plane and its products take 2 MFMAs.  The planes are
// written once per element by the kernel that produces x (a GEMM epilogue, the Adam
// update, the head dZ kernel), which also records max|x| for the next step's scale.
//
// Operand modes (of the operand's HBM layout; gemm.h KCONTIG / RCONTIG):
//   KCONTIG: a load unit is 8 consecutive k of one row  -> LDS [row][k], fragment =
//            ds_read_b128 (16-B chunks XOR-swizzled by row, conflict-free).
//   RCONTIG: a load unit is 8 consecutive rows at one k  -> LDS [k][row], fragment =
//            2 x ds_read_b64_tr_b16 (the hardware transpose read); 32-row segments of a
//            k-row are XOR-swizzled by k so the four k-rows a 32-lane half reads fall
//            in four different 64-byte bank windows (conflict-free).
//
// Problem concept (conv_p3.h):
//   static constexpr int A_MODE, B_MODE, A_PLANES, B_PLANES;   (planes 1 or 2)
//   int M, N, K, k_chunk;
//   PlaneSrc a_src, b_src;   the operands' plane buffers (read through buffer descriptors)
//                            and their scale records (the result is multiplied by both r)
//   ARow a_row(int row) const;  uint32_t a_off(const ARow&, int k0, int kk) const;
//   BRow b_row(int row) const;  uint32_t b_off(const BRow&, int k0, int kk) const;
//     byte offset (within every plane) of the 16-byte unit at reduction index k0 + kk:
//     KCONTIG: k .. k+7 of `row`; RCONTIG: rows row .. row+7 at k; kOOB for a unit of
//     zeros (padding).  k0 is the stage's first k (a multiple of BK, wave-uniform, so the
//     loaders' k0 arithmetic stays scalar) and kk the unit's offset in the stage.
//   float store8(int m, int n, const float (&v)[8], int split) const;  8 consecutive
//     columns of one row (N a multiple of 8); returns max |value stored| of a plane output
//     (0 otherwise);
//   optional kAmax (+ PScale* amax_sc() const): the output's scale record, whose amax the
//   epilogue raises to the block's maximum;
//   optional kColSum (+ store_colsum): sum_k B[n][k], computed by one extra MFMA per B
//   plane against an all-ones A fragment in the blocks of the first row tile;
//   optional kZClass (+ for_z): blockIdx.z selects a sub-problem.
// Loads are raw buffer loads: an out-of-range offset returns zeros, so padding and the
// reduction tail cost no branches.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "gemm.h"
#include "gemm_x6.h"

namespace acme {
namespace gemm {

// XCD-aware block placement.  Blocks are dealt round-robin over the 8 XCDs (block b and
// b + 8 share one L2; MI355X_MICROARCH.md, Workgroup dispatch), so the flat block id is
// remapped (bijectively) to give each XCD one contiguous range of the logical order, in
// which consecutive tiles share an operand panel: K-splits outermost (a split's A and B
// slabs stay in one L2), then tiles with the LARGER operand's panel index slowest.
struct BlockPlace {
  int m0, n0, z;
};
template <int BM, int BN>
__device__ __forceinline__ BlockPlace place_block(int M, int N, int n_major) {
  const int tiles = gridDim.x;
  const int total = tiles * gridDim.z;
  const int orig = blockIdx.x + tiles * blockIdx.z;
  const int xcd = orig & 7, q = total >> 3, r = total & 7;
  const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int z = L / tiles, t = L - z * tiles;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  int mt, nt;
  if (n_major) {
    nt = t / tiles_m;
    mt = t - nt * tiles_m;
  } else {
    mt = t / tiles_n;
    nt = t - mt * tiles_n;
  }
  return BlockPlace{mt * BM, nt * BN, z};
}
template <class P>
__device__ __forceinline__ P z_select_at(const P& p, int z) {
  if constexpr (HasZClass<P>::value) return p.for_z(z);
  else return p;
}

using u32x4 = __attribute__((ext_vector_type(4))) uint32_t;
using i16x4 = __attribute__((ext_vector_type(4))) short;
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;

__device__ __forceinline__ u32x4 zero_u4() { return u32x4{0u, 0u, 0u, 0u}; }

// Byte offset of a unit of zeros: beyond every plane's descriptor range.
constexpr uint32_t kOOB = 0x80000000u;

// Planes of a full f32 operand (a one-plane operand is an exact f16 value, unscaled).
constexpr int kPlanes = 2;

// Scale record of a plane tensor (device memory; the learners own arrays of them).
//   w    producers store the planes of x * w (a power of two);
//   r    consumers multiply their f32 results by r: 1 / the w the stored planes carry;
//   wi   1 / w (a copy of the planes takes it as its r);
//   rl   the r of the planes stored now, after a rescale moved r to the next step's scale
//        (host-side joins of a transient tensor between steps: debug buffers);
//   flag the step guard word a producer raises when one of its writes overflowed f16
//        (|x| w >= 65520, or x not finite): the learner's gated kernels (Adam, the priority
//        write-back, the rescale) then skip the step's update (StepGuard, kernels.h);
//   slot max |x| written since the last rescale, spread over kAmaxSlots words on separate
//        128-B lines (f32 bits; atomicMax as an unsigned: one address took ~12 ns per wave's
//        atomic, 7,168 of them serialised added 87 us to conv1_fwd); the rescale reduces them.
constexpr int kAmaxSlots = 64;
struct PScale {
  float w, r, wi, rl;
  uint32_t* flag;
  uint32_t pad1[26];
  struct Slot {
    uint32_t v;
    uint32_t pad[31];
  } slot[kAmaxSlots];
};
static_assert(sizeof(PScale) == 128 * (1 + kAmaxSlots), "one 128-B line per amax slot");
__device__ __forceinline__ float read_scale(const PScale* s) { return s ? s->r : 1.f; }

// An operand's plane buffers: plane i at p + i * stride (elements), `bytes` readable
// bytes per plane (the descriptor range; < 2^31), and its scale record (null: unscaled).
struct PlaneSrc {
  const uint16_t* p;
  int64_t stride;
  int32_t bytes;
  const PScale* sc = nullptr;
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const PlaneSrc& s, int pl) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(s.p + pl * s.stride), (short)0,
                                           s.bytes, 0x00020000);
}
// The factor a consumer applies to its f32 accumulators: 1 / (w_a w_b).
__device__ __forceinline__ float result_scale(const PlaneSrc& a, const PlaneSrc& b) {
  return read_scale(a.sc) * read_scale(b.sc);
}

// Two-way split of a scaled f32 value y (f16 bit patterns): h = f16(y), l = f16(y - h)
// (y - h is exact in f32).  |y| >= 65520 overflows h (caught by the rescale's check).
__device__ __forceinline__ void split2_bits(float y, uint16_t& h, uint16_t& l) {
  const _Float16 hb = (_Float16)y;
  const _Float16 lb = (_Float16)(y - (float)hb);
  h = __builtin_bit_cast(uint16_t, hb);
  l = __builtin_bit_cast(uint16_t, lb);
}
__device__ __forceinline__ float f16_bits_to_f32(uint16_t b) {
  return (float)__builtin_bit_cast(_Float16, b);
}
// Exact f16 of a byte (integers 0..255 have 8 significant bits).
__device__ __forceinline__ uint32_t f16_of_byte(uint32_t x, int sh) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)(uint16_t)((x >> sh) & 0xffu));
}
// Two packed f16 of bytes sh and sh + 8 of x.
__device__ __forceinline__ uint32_t f16x2_of_bytes(uint32_t x, int sh) {
  return f16_of_byte(x, sh) | (f16_of_byte(x, sh + 8) << 16);
}

// Problems whose A operand is the uint8 Atari frames themselves (`static constexpr bool
// A_U8 = true`, byte offsets): a 16-B A unit (8 f16) is 8 frame bytes widened exactly, so
// the frames are read from HBM once as bytes instead of as an f16 copy (half the bytes).
// Problems with a `uint64_t* stamps` member (timing experiments, ACME_V_STAMPS=1): when it is
// set, the WS kernel's consumer wave 0 stamps its workgroup's phases (s_memrealtime at entry
// and exit, s_memtime at entry, after the prologue's first barrier, after the k loop and at
// exit) into stamps[8 * (flat block id) + 0..5].
template <class P, class = void>
struct HasStamps : std::false_type {};
template <class P>
struct HasStamps<P, std::void_t<decltype(std::declval<P>().stamps)>> : std::true_type {};

template <class P, class = void>
struct AU8 : std::false_type {};
template <class P>
struct AU8<P, std::void_t<decltype(P::A_U8)>> : std::integral_constant<bool, P::A_U8> {};
__device__ __forceinline__ u32x4 f16x8_of_bytes(uint32_t lo, uint32_t hi) {
  return u32x4{f16x2_of_bytes(lo, 0), f16x2_of_bytes(lo, 16), f16x2_of_bytes(hi, 0),
               f16x2_of_bytes(hi, 16)};
}
// One 16-B A unit at byte offset `off` of plane descriptor r (kOOB: zeros), as loaded: for
// uint8 frames the 8 bytes sit in the first two words and a_unit_f16 widens them when the
// unit is stored to LDS, so the widening waits for the load there and not at the fetch
// (which would end the fetch's look-ahead: round 5, conv1_wgrad 25.7 -> 32.5 us until this).
template <class P>
__device__ __forceinline__ u32x4 load_a_unit(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  if constexpr (AU8<P>::value) {
    const auto w = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    return u32x4{(uint32_t)w[0], (uint32_t)w[1], 0u, 0u};
  } else {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  }
}
template <class P>
__device__ __forceinline__ u32x4 a_unit_f16(const u32x4& v) {
  if constexpr (AU8<P>::value) return f16x8_of_bytes(v[0], v[1]);
  else return v;
}

// Maximum of two magnitudes (non-negative floats, or NaN) that keeps NaN: non-negative
// floats order as their bits, and a NaN (sign cleared by fabsf) above infinity.  A plane
// computed from overflowed planes is NaN, and its record must see that.
__device__ __forceinline__ float amax_max(float a, float b) {
  return __builtin_bit_cast(float, max(__builtin_bit_cast(uint32_t, a),
                                       __builtin_bit_cast(uint32_t, b)));
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = amax_max(v, __shfl_xor(v, o, 64));
  return v;
}
// Raises one of sc's amax slots (chosen by the wave's position in the grid) to the wave's
// maximum of v (v >= 0, or NaN) of planes written at sc->w, and raises the record's guard
// flag when that maximum overflowed them; every lane of the wave calls.
__device__ __forceinline__ void amax_commit(PScale* sc, float v) {
  v = wave_max(v);
  const int wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (sc && (threadIdx.x & 63) == 0 && v != 0.f) {
    atomicMax(&sc->slot[wid & (kAmaxSlots - 1)].v, __builtin_bit_cast(uint32_t, v));
    if (!(v * sc->w < 65520.f) && sc->flag) atomicOr(sc->flag, 1u);
  }
}

// As amax_commit, with the record's w and flag loaded beforehand (EpiPre below).
__device__ __forceinline__ void amax_commit_pre(PScale* sc, float v, float w, uint32_t* flag) {
  v = wave_max(v);
  const int wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (sc && (threadIdx.x & 63) == 0 && v != 0.f) {
    atomicMax(&sc->slot[wid & (kAmaxSlots - 1)].v, __builtin_bit_cast(uint32_t, v));
    if (!(v * w < 65520.f) && flag) atomicOr(flag, 1u);
  }
}

// Problems whose epilogue constants (bias, read scales, the output record's w and flag) a
// lane can load before the k loop (`Pre pre(int n)` for the lane's 8 columns n..n+7, then
// `store8p(m, n, v, split, pre)`): their latency then overlaps the k loop instead of
// stalling the epilogue's first store (round 5 stamps: conv1's epilogue took longer than
// its k loop).
template <class P, class = void>
struct EpiPre {
  struct type {};
  static constexpr bool has = false;
};
template <class P>
struct EpiPre<P, std::void_t<typename P::Pre>> {
  using type = typename P::Pre;
  static constexpr bool has = true;
};

// A plane tensor: plane i of element e at p[i * stride + e], written as x * sc->w.
struct Planes {
  uint16_t* p;
  int64_t stride;
  PScale* sc;
  __device__ __forceinline__ float w() const { return sc->w; }
  // Stores x; returns |x| (the caller's amax).
  __device__ __forceinline__ float put(int64_t e, float x) const {
    uint16_t h, l;
    split2_bits(x * w(), h, l);
    p[e] = h;
    p[stride + e] = l;
    return fabsf(x);
  }
};
struct CPlanes {
  const uint16_t* p;
  int64_t stride;
  const PScale* sc;
  // x > 0 of a value whose planes are stored (ReLU masks: h = f16(x w) has x's sign and
  // is zero only for x w below half of f16's smallest subnormal, i.e. x < 2^-33 max|x|).
  __device__ __forceinline__ bool positive(int64_t e) const {
    const uint16_t h = p[e];
    return h != 0 && (h & 0x8000) == 0;
  }
  // The stored value (between steps: at the scale the planes were written with).
  __device__ __forceinline__ float value(int64_t e) const {
    return (f16_bits_to_f32(p[e]) + f16_bits_to_f32(p[stride + e])) * (sc ? sc->rl : 1.f);
  }
};

// The MFMA terms of one 32x32x16 product of an NPA-plane A fragment and an NPB-plane B
// fragment, smallest first: (1,0), (0,1), (0,0).
#ifndef P3_FOUR_TERMS
#define P3_FOUR_TERMS 0  // 1: also the l*l term of two-plane products (exact products)
#endif
template <int NPA, int NPB>
__device__ __forceinline__ void p3_terms(const f16x8 (&fa)[NPA], const f16x8 (&fb)[NPB],
                                         f32x16& acc) {
  static_assert((NPA == 1 || NPA == 2) && (NPB == 1 || NPB == 2), "1 or 2 planes per operand");
  if constexpr (P3_FOUR_TERMS && NPA == 2 && NPB == 2)
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[1], fb[1], acc, 0, 0, 0);
  if constexpr (NPA == 2) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[1], fb[0], acc, 0, 0, 0);
  if constexpr (NPB == 2) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[0], fb[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[0], fb[0], acc, 0, 0, 0);
}
template <int NPA, int NPB>
constexpr int p3_nterms() {
  return 1 + (NPA == 2 ? 1 : 0) + (NPB == 2 ? 1 : 0) + (P3_FOUR_TERMS && NPA == 2 && NPB == 2 ? 1 : 0);
}

__device__ __forceinline__ f16x8 ones16() {
  const _Float16 o = (_Float16)1.f;
  return f16x8{o, o, o, o, o, o, o, o};
}

// Accumulators of a wave's tile (round 6).  v_mfma_f32_32x32x16_f16 does
// not accumulate without bias: the three terms of each product summed into one running
// accumulator carry an error whose mean is -0.05 (K = 256) to -0.13 (K = 4096) of its rms,
// against 0 for the f32 MFMA (tools/mfma_bias.hip, profiles/r06/accuracy/mfma_bias.log), and
// every dZ and activation tensor of the step inherited a mean of about -0.04 of its error
// rms.  A convolution's weight gradient sums such a tensor against non-negative activations
// over B x pixels rows, where a bias adds up linearly and unbiased errors as a square root:
// at B = 64 the conv weight gradients carried 2.5-7x the exact-f32 engine's error
// (profiles/r05/drift/grad_err_B64_step0.log).  The bits are lost where the small terms
// (l, h) and (h, l) -- 2^-11 of the (h, h) term -- meet a large accumulator: accumulated in
// their own tile (SPLIT) the bias falls 5x (K = 256) to 30x (K = 4096) and the rms error
// 1.6x, and the tiles are added (one f32 add per element) before the epilogue.  The column
// sums (bias gradients: ones x each B plane) split the same way (l plane apart).  Where the
// split applies: products of two two-plane operands (the uint8 frames are one exact plane:
// conv1's outputs carried a mean of -0.008 only) on wave tiles of at most four 32 x 32 MFMA
// tiles, except problems with `kNoSplitAcc` -- the dense forward (fc_fwd's 128 x 64 consumer
// tiles already hold 128 accumulators: a second set would not fit two waves per SIMD; its
// output feeds only the head) and the dense weight gradient (a batch-long reduction whose
// result is summed nowhere else; one block per CU instead of two with the second set).
#ifndef P3_SPLIT_ACC
#define P3_SPLIT_ACC 1  // 0: one accumulator per tile (the round-5 arithmetic; accuracy A/B)
#endif
template <class P, class = void>
struct P3NoSplit : std::false_type {};
template <class P>
struct P3NoSplit<P, std::void_t<decltype(P::kNoSplitAcc)>>
    : std::integral_constant<bool, P::kNoSplitAcc> {};
template <class P, int MT, int NTL>
constexpr bool p3_split_acc() {
  return P3_SPLIT_ACC != 0 && P::A_PLANES == 2 && P::B_PLANES == 2 && MT * NTL <= 4 &&
         !P3NoSplit<P>::value;
}
template <int MT, int NTL, int NCS, bool SPLIT>
struct P3Acc {
  static constexpr int SM = SPLIT ? MT : 1, SN = SPLIT ? NTL : 1, SC = SPLIT ? NCS : 1;
  f32x16 a[MT][NTL];  // the (h, h) terms (every term without SPLIT)
  f32x16 s[SM][SN];   // the small terms
  f32x16 c[NCS];      // column sums of B's h plane (every plane without SPLIT)
  f32x16 cl[SC];      // of its l plane
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NTL; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) a[i][j][v] = 0.f;
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < SN; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) s[i][j][v] = 0.f;
#pragma unroll
    for (int j = 0; j < NCS; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) c[j][v] = 0.f;
#pragma unroll
    for (int j = 0; j < SC; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) cl[j][v] = 0.f;
  }
  // The terms of tile (i, j): smallest first, (1,0), (0,1) [, (1,1)] into s (SPLIT) or a,
  // then (0,0) into a.
  template <int NPA, int NPB>
  __device__ __forceinline__ void terms(int i, int j, const f16x8 (&fa)[NPA],
                                        const f16x8 (&fb)[NPB]) {
    static_assert((NPA == 1 || NPA == 2) && (NPB == 1 || NPB == 2), "1 or 2 planes per operand");
    if constexpr (SPLIT) {
      f32x16& x = s[i][j];
      if constexpr (P3_FOUR_TERMS && NPA == 2 && NPB == 2)
        x = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[1], fb[1], x, 0, 0, 0);
      if constexpr (NPA == 2) x = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[1], fb[0], x, 0, 0, 0);
      if constexpr (NPB == 2) x = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[0], fb[1], x, 0, 0, 0);
      a[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[0], fb[0], a[i][j], 0, 0, 0);
    } else {
      p3_terms<NPA, NPB>(fa, fb, a[i][j]);
    }
  }
  // Column sums of B tile j: ones x each plane, the l plane first.
  template <int NPB>
  __device__ __forceinline__ void colsum(int j, const f16x8 (&fb)[NPB]) {
    if constexpr (NPB == 2) {
      f32x16& x = SPLIT ? cl[SPLIT ? j : 0] : c[j];
      x = __builtin_amdgcn_mfma_f32_32x32x16_f16(ones16(), fb[1], x, 0, 0, 0);
    }
    c[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ones16(), fb[0], c[j], 0, 0, 0);
  }
  // a += s, c += cl (before the epilogue).
  __device__ __forceinline__ void fold() {
    if constexpr (SPLIT) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j) a[i][j] += s[i][j];
#pragma unroll
      for (int j = 0; j < NCS; ++j) c[j] += cl[j];
    }
  }
};

// Problems with `static constexpr bool kAmax = true` write a plane output whose scale
// record amax_sc() collects max |x|.
template <class P, class = void>
struct HasAmax {
  static constexpr bool value = false;
};
template <class P>
struct HasAmax<P, decltype(void(P::kAmax))> {
  static constexpr bool value = P::kAmax;
};

// Optional vector epilogue: problems with `static constexpr bool kStore8 = true` receive
// 8 consecutive columns of one row, p.store8(m, n, v[8], split) with n % 8 == 0 (their N
// must be a multiple of 8).
template <class P, class = void>
struct HasStore8 {
  static constexpr bool value = false;
};
template <class P>
struct HasStore8<P, decltype(void(P::kStore8))> {
  static constexpr bool value = P::kStore8;
};

template <int BK>
__device__ __forceinline__ int p3_kswz(int row) {
  return BK == 16 ? ((row >> 3) & 1) : ((row >> 2) & 3);
}
template <int R>
__device__ __forceinline__ int p3_rswz(int k) {
  return R >= 128 ? (k & 3) : (R == 64 ? ((k >> 1) & 1) : 0);
}

template <int R, int NT, int MODE, int NPL, int BK>
struct PlanP3 {
  static_assert(R % 32 == 0, "operand tile rows must be a multiple of 32");
  static constexpr int PLANE = R * BK * 2;  // bytes of one plane per stage
  static constexpr int BYTES = NPL * PLANE;
  static constexpr int CPR = BK / 8;        // KCONTIG: 16-B chunks per row
  static constexpr int OPK = R / 8;         // RCONTIG: row octets per k
  static constexpr int UNITS = MODE == KCONTIG ? R * CPR : OPK * BK;
  static constexpr int PER_THREAD = (UNITS + NT - 1) / NT;
  static_assert(UNITS % NT == 0 || UNITS < NT, "tile units must divide evenly over the threads");
  __device__ static __forceinline__ bool owns(int u) { return UNITS >= NT || u < UNITS; }
  __device__ static __forceinline__ int row_of(int u) {
    return MODE == KCONTIG ? u / CPR : 8 * (u % OPK);
  }
  __device__ static __forceinline__ int kk_of(int u) {
    return MODE == KCONTIG ? 8 * (u % CPR) : u / OPK;
  }
  __device__ static __forceinline__ int offset(int u) {
    if constexpr (MODE == KCONTIG) {
      const int row = u / CPR;
      return row * (2 * BK) + 16 * ((u % CPR) ^ p3_kswz<BK>(row));
    } else {
      const int k = u / OPK, row = 8 * (u % OPK);
      return k * (2 * R) + 2 * (row ^ (p3_rswz<R>(k) << 5));
    }
  }
  // LDS-DMA view: the image is unit-linear (slot u at byte 16 u), so DMA block b (64
  // slots, one per lane) lands in 1 KiB at 1024 b, and the swizzle is applied by choosing
  // which logical unit each slot's lane fetches.
  static constexpr int BLOCKS = UNITS / 64;
  static_assert(UNITS % 64 == 0, "tile units must fill whole 64-lane DMA blocks");
  __device__ static __forceinline__ int slot_row(int u) {
    if constexpr (MODE == KCONTIG) return u / CPR;
    else return 8 * ((u % OPK) ^ (p3_rswz<R>(u / OPK) << 2));
  }
  __device__ static __forceinline__ int slot_kk(int u) {
    if constexpr (MODE == KCONTIG) return 8 * ((u % CPR) ^ p3_kswz<BK>(u / CPR));
    else return u / OPK;
  }
  // MFMA operand of rows rb .. rb+31 (rb a multiple of 32), k step s (16 k).
  __device__ static __forceinline__ f16x8 frag(const uint8_t* tile, int plane, int rb, int s,
                                               int lane) {
    const uint8_t* t = tile + plane * PLANE;
    if constexpr (MODE == KCONTIG) {
      const int row = rb + (lane & 31);
      const int c = 2 * s + (lane >> 5);
      return *reinterpret_cast<const f16x8*>(t + row * (2 * BK) + 16 * (c ^ p3_kswz<BK>(row)));
    } else {
      const int h = lane >> 5, g = (lane >> 4) & 1, q = (lane >> 2) & 3, pp = lane & 3;
      const int row = rb + 16 * g + 4 * pp;
      const int k0 = 16 * s + 8 * h + q;
      const int k1 = k0 + 4;
      typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
      const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_i16x4*)(t + k0 * (2 * R) + 2 * (row ^ (p3_rswz<R>(k0) << 5))));
      const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_i16x4*)(t + k1 * (2 * R) + 2 * (row ^ (p3_rswz<R>(k1) << 5))));
      const __attribute__((ext_vector_type(8))) short v{lo[0], lo[1], lo[2], lo[3],
                                                        hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(f16x8, v);
    }
  }
};

// Shared MFMA core of the plane kernels: one LDS stage's fragments and MFMAs, and the
// epilogue.
template <int BM, int BN, int WM, int WN, int BK, class P>
struct P3Core {
  static constexpr int NT = 64 * WM * WN;
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int MT = TM / 32, NTL = TN / 32;
  static constexpr int NPA = P::A_PLANES, NPB = P::B_PLANES;
  static_assert(TM % 32 == 0 && TN % 32 == 0, "wave tile must be a multiple of 32x32");
  static_assert(BK == 16 || BK == 32, "BK must be 16 or 32");
  static_assert((NPA == 1 || NPA == 2) && (NPB == 1 || NPB == 2), "1 or 2 planes per operand");
  using PA = PlanP3<BM, NT, P::A_MODE, NPA, BK>;
  using PB = PlanP3<BN, NT, P::B_MODE, NPB, BK>;
  static constexpr int STAGE = PA::BYTES + PB::BYTES;
  static constexpr bool kColSum = HasColSum<P>::value;
  static constexpr int NCS = kColSum ? NTL : 1;
  static constexpr int EPI_BYTES = HasStore8<P>::value ? WM * WN * 32 * (TN + 4) * 4 : 0;
  static constexpr bool SPLIT = p3_split_acc<P, MT, NTL>();
  using Acc = P3Acc<MT, NTL, NCS, SPLIT>;

  // The MFMAs of k16 steps S0 .. S1 - 1 of the stage at (sa, sb).
  template <int S0 = 0, int S1 = BK / 16>
  __device__ static __forceinline__ void mma(const uint8_t* sa, const uint8_t* sb, int wm, int wn,
                                             int lane, Acc& acc, bool do_colsum) {
#pragma unroll
    for (int s = S0; s < S1; ++s) {
      f16x8 fa[MT][NPA], fb[NTL][NPB];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int pl = 0; pl < NPA; ++pl)
          fa[i][pl] = PA::frag(sa, pl, wm * TM + i * 32, s, lane);
#pragma unroll
      for (int j = 0; j < NTL; ++j)
#pragma unroll
        for (int pl = 0; pl < NPB; ++pl)
          fb[j][pl] = PB::frag(sb, pl, wn * TN + j * 32, s, lane);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j) acc.terms(i, j, fa[i], fb[j]);
      if constexpr (kColSum) {
        if (do_colsum) {
#pragma unroll
          for (int j = 0; j < NTL; ++j) acc.colsum(j, fb[j]);
        }
      }
    }
  }

  // The two halves of mma() for one k16 step, for callers that software-pipeline the
  // fragment reads (same terms in the same order, so the same bits).
  using FragA = f16x8[MT][NPA];
  using FragB = f16x8[NTL][NPB];
  __device__ static __forceinline__ void read_frags(const uint8_t* sa, const uint8_t* sb, int wm,
                                                    int wn, int s, int lane, FragA& fa,
                                                    FragB& fb) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int pl = 0; pl < NPA; ++pl) fa[i][pl] = PA::frag(sa, pl, wm * TM + i * 32, s, lane);
#pragma unroll
    for (int j = 0; j < NTL; ++j)
#pragma unroll
      for (int pl = 0; pl < NPB; ++pl) fb[j][pl] = PB::frag(sb, pl, wn * TN + j * 32, s, lane);
  }
  __device__ static __forceinline__ void mfma_frags(const FragA& fa, const FragB& fb, Acc& acc,
                                                    bool do_colsum) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NTL; ++j) acc.terms(i, j, fa[i], fb[j]);
    if constexpr (kColSum) {
      if (do_colsum) {
#pragma unroll
        for (int j = 0; j < NTL; ++j) acc.colsum(j, fb[j]);
      }
    }
  }

  // Epilogue.  C/D map of the 32x32 MFMA: col = lane & 31, row = (v&3) + 8(v>>2) + 4h.
  // The LDS is free (every stage consumed) when this runs; it contains barriers, so all
  // waves of the block call it.
  // A lane's epilogue columns: n0 + wn TN + epi_col(lane) (the same in every chunk).
  __device__ static __forceinline__ int epi_col(int lane) {
    static_assert(64 % (TN / 8) == 0, "a lane's chunk columns repeat");
    return 8 * (lane % (TN / 8));
  }
  // The epilogue of an accumulator struct: its tiles folded first (a += s, c += cl).
  template <int M2, int N2, int C2, bool S2>
  __device__ static __forceinline__ void epilogue(const P& p, uint8_t* smem, int m0, int n0,
                                                  int wave, int wm, int wn, int lane, int split,
                                                  P3Acc<M2, N2, C2, S2>& acc, bool do_colsum,
                                                  const typename EpiPre<P>::type* pre = nullptr) {
    static_assert(M2 == MT && N2 == NTL && C2 == NCS, "the accumulators of this tile");
    acc.fold();
    epilogue(p, smem, m0, n0, wave, wm, wn, lane, split, acc.a, acc.c, do_colsum, pre);
  }
  __device__ static __forceinline__ void epilogue(const P& p, uint8_t* smem, int m0, int n0,
                                                  int wave, int wm, int wn, int lane, int split,
                                                  f32x16 (&acc)[MT][NTL], f32x16 (&cs)[NCS],
                                                  bool do_colsum,
                                                  const typename EpiPre<P>::type* pre = nullptr) {
    static_assert(HasStore8<P>::value, "plane problems store 8 columns at a time");
    const int r = lane & 31, h = lane >> 5;
    typename EpiPre<P>::type pl{};
    if constexpr (EpiPre<P>::has) pl = pre ? *pre : p.pre(n0 + wn * TN + epi_col(lane));
    // Row-major restage through LDS, one 32-row block of the wave's tile at a time, so
    // each lane finishes 8 consecutive columns of one row (one decode per 8 outputs,
    // 16-byte plane / 32-byte f32 stores).
    constexpr int PITCH = TN + 4;
    float* cw = reinterpret_cast<float*>(smem) + wave * 32 * PITCH;
    constexpr int CHUNKS = 32 * TN / 8;
    float amx = 0.f;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int j = 0; j < NTL; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v)
          cw[((v & 3) + 8 * (v >> 2) + 4 * h) * PITCH + j * 32 + r] = acc[i][j][v];
      __syncthreads();
#pragma unroll
      for (int c = lane; c < CHUNKS; c += 64) {
        const int row = c / (TN / 8), col = 8 * (c % (TN / 8));
        const int m = m0 + wm * TM + i * 32 + row;
        const int n = n0 + wn * TN + col;
        const f32x4 lo = *reinterpret_cast<const f32x4*>(cw + row * PITCH + col);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(cw + row * PITCH + col + 4);
        const float v8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        if constexpr (EpiPre<P>::has) {
          if (m < p.M && n < p.N) amx = amax_max(amx, p.store8p(m, n, v8, split, pl));
        } else {
          if (m < p.M && n < p.N) amx = amax_max(amx, p.store8(m, n, v8, split));
        }
      }
      __syncthreads();
    }
    if constexpr (HasAmax<P>::value) {
      if constexpr (EpiPre<P>::has) amax_commit_pre(p.amax_sc(), amx, pl.w, pl.flag);
      else amax_commit(p.amax_sc(), amx);
    }
    if constexpr (kColSum) {
      if (do_colsum && h == 0) {
#pragma unroll
        for (int j = 0; j < NTL; ++j) {
          const int n = n0 + wn * TN + j * 32 + r;
          if (n < p.N) p.store_colsum(n, cs[j][0], split);
        }
      }
    }
  }
};

// Register-staged kernel: global -> VGPR -> LDS, two LDS stages; with DEEP two register
// sets so a stage's loads are issued two stages before its compute.
template <int BM, int BN, int WM, int WN, int BK, bool DEEP, class P>
__global__ void __launch_bounds__(64 * WM * WN) gemm_p3_kernel(const P p_in, int n_major) {
  using C = P3Core<BM, BN, WM, WN, BK, P>;
  using PA = typename C::PA;
  using PB = typename C::PB;
  constexpr int NT = C::NT, NPA = C::NPA, NPB = C::NPB, STAGE = C::STAGE;
  const BlockPlace bp = place_block<BM, BN>(p_in.M, p_in.N, n_major);
  const P p = z_select_at(p_in, bp.z);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = bp.m0, n0 = bp.n0;
  const int split = HasZClass<P>::value ? 0 : bp.z;
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

  __amdgpu_buffer_rsrc_t srcA[NPA], srcB[NPB];
#pragma unroll
  for (int pl = 0; pl < NPA; ++pl) srcA[pl] = plane_rsrc(p.a_src, pl);
#pragma unroll
  for (int pl = 0; pl < NPB; ++pl) srcB[pl] = plane_rsrc(p.b_src, pl);

  constexpr int SETS = DEEP ? 2 : 1;
  u32x4 ra[SETS][PA::PER_THREAD][NPA], rb[SETS][PB::PER_THREAD][NPB];
  auto fetch = [&](auto S, int k0) {
    constexpr int set = decltype(S)::value;
#pragma unroll
    for (int i = 0; i < PA::PER_THREAD; ++i) {
      const int u = tid + i * NT;
      const int kk = PA::kk_of(u);
      const uint32_t off = (PA::owns(u) && k0 + kk < kend) ? p.a_off(arow[i], k0, kk) : kOOB;
#pragma unroll
      for (int pl = 0; pl < NPA; ++pl) {
        ra[set][i][pl] = load_a_unit<P>(srcA[pl], off);
      }
    }
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
  auto stash = [&](auto S, int buf) {
    constexpr int set = decltype(S)::value;
    uint8_t* sa = smem + buf * STAGE;
    uint8_t* sb = sa + PA::BYTES;
#pragma unroll
    for (int i = 0; i < PA::PER_THREAD; ++i) {
      const int u = tid + i * NT;
      if (!PA::owns(u)) continue;
      const int off = PA::offset(u);
#pragma unroll
      for (int pl = 0; pl < NPA; ++pl)
        *reinterpret_cast<u32x4*>(sa + pl * PA::PLANE + off) = a_unit_f16<P>(ra[set][i][pl]);
    }
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

  typename C::Acc acc;
  acc.zero();
  const bool do_colsum = C::kColSum && m0 == 0 && wm == 0;
  auto compute = [&](int buf) {
    const uint8_t* sa = smem + buf * STAGE;
    C::mma(sa, sa + PA::BYTES, wm, wn, lane, acc, do_colsum);
  };

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  if constexpr (DEEP) {
    if (nk > 0) {
      fetch(S0{}, kbeg);
      stash(S0{}, 0);
    }
    if (nk > 1) fetch(S1{}, kbeg + BK);
    __syncthreads();
    // Iteration kt: LDS buffer kt & 1 holds stage kt, register set (kt + 1) & 1 holds
    // stage kt + 1 (loaded during iteration kt - 1); stage kt + 2 is fetched into set
    // kt & 1.  Stage kt + 1 is stashed BEFORE the MFMAs of stage kt (its buffer was last
    // read in iteration kt - 1, before the barrier), so the LDS stores overlap the MFMAs and
    // the barrier waits only for the compute.
    auto iter = [&](auto S, int kt) {
      constexpr int set = decltype(S)::value;
      using Other = std::integral_constant<int, set ^ 1>;
      // Branch-free body (one basic block, so the scheduler can spread the LDS stores and
      // loads among the MFMAs): past the end, fetch reads zeros (offsets beyond kend are
      // kOOB) and stash fills a buffer that is never read.
      if constexpr (BK == 32) {
        // First k16 step's MFMAs, then the LDS stores of stage kt + 1 and the loads of stage
        // kt + 2, then the second step: the stores overlap MFMAs already queued (measured
        // +7% fc_fwd against the stores before the first step).
        const uint8_t* sa = smem + set * STAGE;
        C::template mma<0, 1>(sa, sa + PA::BYTES, wm, wn, lane, acc, do_colsum);
        stash(Other{}, set ^ 1);
        fetch(S, kbeg + (kt + 2) * BK);
        C::template mma<1, 2>(sa, sa + PA::BYTES, wm, wn, lane, acc, do_colsum);
      } else {
        stash(Other{}, set ^ 1);
        fetch(S, kbeg + (kt + 2) * BK);
        compute(set);
      }
      __syncthreads();
    };
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
      iter(S0{}, kt);
      iter(S1{}, kt + 1);
    }
    if (kt < nk) iter(S0{}, kt);
  } else {
    if (nk > 0) {
      fetch(S0{}, kbeg);
      stash(S0{}, 0);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk;
      if (more) fetch(S0{}, kbeg + (kt + 1) * BK);
      compute(kt & 1);
      if (more) stash(S0{}, (kt + 1) & 1);
      __syncthreads();
    }
  }
  C::epilogue(p, smem, m0, n0, wave, wm, wn, lane, split, acc, do_colsum);
}

// LDS-DMA kernel: every operand unit goes HBM -> LDS by buffer_load ... lds (no VGPR
// staging), through a ring of STAGES LDS buffers with STAGES - 1 stages in flight.  Each
// wave issues the same number of DMA instructions per stage (surplus lanes of a short
// operand fetch zeros into a scratch KiB), so one counted vmcnt per iteration retires the
// stage about to be read; one raw s_barrier per iteration publishes it and frees the
// buffer the next DMA overwrites.
template <int BM, int BN, int WM, int WN, int BK, int STAGES, class P>
__global__ void __launch_bounds__(64 * WM * WN) gemm_p3g_kernel(const P p_in, int n_major) {
  // Device pass only: hipcc does not emit this template's host launch stub when the host
  // pass instantiates the body (the LDS-DMA builtins), so the host sees an empty kernel.
#if defined(__HIP_DEVICE_COMPILE__)
  using C = P3Core<BM, BN, WM, WN, BK, P>;
  using PA = typename C::PA;
  using PB = typename C::PB;
  constexpr int NW = WM * WN, NPA = C::NPA, NPB = C::NPB, STAGE = C::STAGE;
  constexpr int PWA = (PA::BLOCKS + NW - 1) / NW, PWB = (PB::BLOCKS + NW - 1) / NW;
  static_assert(!AU8<P>::value, "LDS-DMA copies bytes as they are: no uint8 A operand");
  constexpr int D = PWA * NPA + PWB * NPB;  // DMA instructions per wave per stage
  static_assert(STAGES >= 2 && STAGES <= 4, "2..4 LDS stages");
  static_assert((STAGES - 2) * D <= 63, "vmcnt range");
  const BlockPlace bp = place_block<BM, BN>(p_in.M, p_in.N, n_major);
  const P p = z_select_at(p_in, bp.z);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* scratch = smem + STAGES * STAGE;  // 1 KiB sink of surplus DMA lanes

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = bp.m0, n0 = bp.n0;
  const int split = HasZClass<P>::value ? 0 : bp.z;
  const int kbeg = split * p.k_chunk;
  int kend = kbeg + p.k_chunk;
  if (kend > p.K) kend = p.K;
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  // The unit each lane fetches for each of its wave's DMA blocks.
  typename P::ARow arow[PWA];
  typename P::BRow brow[PWB];
  int akk[PWA], bkk[PWB];
#pragma unroll
  for (int j = 0; j < PWA; ++j) {
    const int b = wave + NW * j;
    const int u = 64 * (b < PA::BLOCKS ? b : 0) + lane;
    arow[j] = p.a_row(m0 + PA::slot_row(u));
    akk[j] = PA::slot_kk(u);
  }
#pragma unroll
  for (int j = 0; j < PWB; ++j) {
    const int b = wave + NW * j;
    const int u = 64 * (b < PB::BLOCKS ? b : 0) + lane;
    brow[j] = p.b_row(n0 + PB::slot_row(u));
    bkk[j] = PB::slot_kk(u);
  }
  __amdgpu_buffer_rsrc_t srcA[NPA], srcB[NPB];
#pragma unroll
  for (int pl = 0; pl < NPA; ++pl) srcA[pl] = plane_rsrc(p.a_src, pl);
#pragma unroll
  for (int pl = 0; pl < NPB; ++pl) srcB[pl] = plane_rsrc(p.b_src, pl);

  typedef __attribute__((address_space(3))) void lds_void;
  // DMA of stage `st` (k0 = kbeg + st * BK) into LDS buffer `buf`; stages past the end
  // fetch zeros (uniform instruction counts keep the vmcnt arithmetic exact).
  auto issue = [&](int st, int buf) {
    const int k0 = kbeg + st * BK;
    uint8_t* sa = smem + buf * STAGE;
    uint8_t* sb = sa + PA::BYTES;
#pragma unroll
    for (int j = 0; j < PWA; ++j) {
      const int b = wave + NW * j;
      const bool real = b < PA::BLOCKS;
      const uint32_t off = (real && k0 + akk[j] < kend) ? p.a_off(arow[j], k0, akk[j]) : kOOB;
#pragma unroll
      for (int pl = 0; pl < NPA; ++pl)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            srcA[pl], (lds_void*)(real ? sa + pl * PA::PLANE + 1024 * b : scratch), 16, off, 0, 0,
            0);
    }
#pragma unroll
    for (int j = 0; j < PWB; ++j) {
      const int b = wave + NW * j;
      const bool real = b < PB::BLOCKS;
      const uint32_t off = (real && k0 + bkk[j] < kend) ? p.b_off(brow[j], k0, bkk[j]) : kOOB;
#pragma unroll
      for (int pl = 0; pl < NPB; ++pl)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            srcB[pl], (lds_void*)(real ? sb + pl * PB::PLANE + 1024 * b : scratch), 16, off, 0, 0,
            0);
    }
  };

  typename C::Acc acc;
  acc.zero();
  const bool do_colsum = C::kColSum && m0 == 0 && wm == 0;

  // s_waitcnt immediates (gfx9 encoding): vmcnt(n) alone, and vmcnt(0) + lgkmcnt(0).
  constexpr int kWaitStage = (((STAGES - 2) * D) & 15) | ((((STAGES - 2) * D) >> 4) << 14) |
                             (0x7 << 4) | (0xF << 8);
#pragma unroll
  for (int st = 0; st < STAGES - 1; ++st) issue(st, st);
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    __builtin_amdgcn_s_waitcnt(kWaitStage);  // this wave's DMA of stage kt has landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();            // ... and every wave's; buffer kt-1 is free
    asm volatile("" ::: "memory");
    const int nb = buf == 0 ? STAGES - 1 : buf - 1;  // (kt + STAGES - 1) % STAGES
    issue(kt + STAGES - 1, nb);
    const uint8_t* sa = smem + buf * STAGE;
    C::mma(sa, sa + PA::BYTES, wm, wn, lane, acc, do_colsum);
    buf = buf == STAGES - 1 ? 0 : buf + 1;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  C::epilogue(p, smem, m0, n0, wave, wm, wn, lane, split, acc, do_colsum);
#endif
}

// Warp-specialised kernel: WM x WN consumer waves (fragment reads + MFMAs only, the same
// P3Core::mma as gemm_p3_kernel, so the same bits) and as many producer waves (global ->
// VGPR -> LDS only), two waves per SIMD, so one wave's staging instructions issue in the
// other's MFMA gaps instead of in its own instruction stream.  Ring of 3 LDS stages and two
// producer register sets: in iteration kt the consumers read stage kt (buffer kt % 3) while
// the producers store stage kt + 2 (loaded two iterations earlier) into buffer (kt + 2) % 3,
// last read in iteration kt - 1, and issue the loads of stage kt + 4; one barrier per
// iteration.  Stages past the end load zeros into buffers that are never read.
template <int BM, int BN, int WM, int WN, int BK, bool PIPE, class P>
__global__ void __launch_bounds__(128 * WM * WN) gemm_p3ws_kernel(const P p_in, int n_major) {
  constexpr int RING = 3;  // (two stages, two blocks per CU, measured slower on the step)
  using C = P3Core<BM, BN, WM, WN, BK, P>;
  using PA = typename C::PA;
  using PB = typename C::PB;
  constexpr int NT = C::NT, NPA = C::NPA, NPB = C::NPB, STAGE = C::STAGE;
  const BlockPlace bp = place_block<BM, BN>(p_in.M, p_in.N, n_major);
  const P p = z_select_at(p_in, bp.z);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x;
  const bool producer = __builtin_amdgcn_readfirstlane(tid) >= NT;
  const int lane = tid & 63;
  const int m0 = bp.m0, n0 = bp.n0;
  const int split = HasZClass<P>::value ? 0 : bp.z;
  const int kbeg = split * p.k_chunk;
  int kend = kbeg + p.k_chunk;
  if (kend > p.K) kend = p.K;
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;

  if (producer) {
    const int pt = tid - NT;
    typename P::ARow arow[PA::PER_THREAD];
    typename P::BRow brow[PB::PER_THREAD];
#pragma unroll
    for (int i = 0; i < PA::PER_THREAD; ++i)
      arow[i] = p.a_row(m0 + (PA::owns(pt + i * NT) ? PA::row_of(pt + i * NT) : 0));
#pragma unroll
    for (int i = 0; i < PB::PER_THREAD; ++i)
      brow[i] = p.b_row(n0 + (PB::owns(pt + i * NT) ? PB::row_of(pt + i * NT) : 0));
    __amdgpu_buffer_rsrc_t srcA[NPA], srcB[NPB];
#pragma unroll
    for (int pl = 0; pl < NPA; ++pl) srcA[pl] = plane_rsrc(p.a_src, pl);
#pragma unroll
    for (int pl = 0; pl < NPB; ++pl) srcB[pl] = plane_rsrc(p.b_src, pl);
    u32x4 ra[2][PA::PER_THREAD][NPA], rb[2][PB::PER_THREAD][NPB];
    auto fetch = [&](auto S, int st) {
      constexpr int set = decltype(S)::value;
      const int k0 = kbeg + st * BK;
#pragma unroll
      for (int i = 0; i < PA::PER_THREAD; ++i) {
        const int u = pt + i * NT;
        const int kk = PA::kk_of(u);
        const uint32_t off = (PA::owns(u) && k0 + kk < kend) ? p.a_off(arow[i], k0, kk) : kOOB;
#pragma unroll
        for (int pl = 0; pl < NPA; ++pl) ra[set][i][pl] = load_a_unit<P>(srcA[pl], off);
      }
#pragma unroll
      for (int i = 0; i < PB::PER_THREAD; ++i) {
        const int u = pt + i * NT;
        const int kk = PB::kk_of(u);
        const uint32_t off = (PB::owns(u) && k0 + kk < kend) ? p.b_off(brow[i], k0, kk) : kOOB;
#pragma unroll
        for (int pl = 0; pl < NPB; ++pl)
          rb[set][i][pl] =
              __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(srcB[pl], off, 0, 0));
      }
    };
    auto stash = [&](auto S, int buf) {
      constexpr int set = decltype(S)::value;
      uint8_t* sa = smem + buf * STAGE;
      uint8_t* sb = sa + PA::BYTES;
#pragma unroll
      for (int i = 0; i < PA::PER_THREAD; ++i) {
        const int u = pt + i * NT;
        if (!PA::owns(u)) continue;
#pragma unroll
        for (int pl = 0; pl < NPA; ++pl)
          *reinterpret_cast<u32x4*>(sa + pl * PA::PLANE + PA::offset(u)) =
              a_unit_f16<P>(ra[set][i][pl]);
      }
#pragma unroll
      for (int i = 0; i < PB::PER_THREAD; ++i) {
        const int u = pt + i * NT;
        if (!PB::owns(u)) continue;
#pragma unroll
        for (int pl = 0; pl < NPB; ++pl)
          *reinterpret_cast<u32x4*>(sb + pl * PB::PLANE + PB::offset(u)) = rb[set][i][pl];
      }
    };

    fetch(S0{}, 0);
    fetch(S1{}, 1);
    stash(S0{}, 0);
    fetch(S0{}, 2);
    stash(S1{}, 1);
    fetch(S1{}, 3);
    __syncthreads();
    // Iteration kt: stage kt + 2 sits in set kt % 2 (loaded in iteration kt - 2, or the
    // prologue); store it to buffer (kt + 2) % 3, then load stage kt + 4 into that set.
    // (Three sets, loads three iterations ahead, measured the same.)
    int wbuf = 2;
    auto iter = [&](auto S, int kt) {
      stash(S, wbuf);
      fetch(S, kt + 4);
      wbuf = wbuf == RING - 1 ? 0 : wbuf + 1;
      __syncthreads();
    };
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
      iter(S0{}, kt);
      iter(S1{}, kt + 1);
    }
    if (kt < nk) iter(S0{}, kt);
    // The consumers' epilogue barriers.
    if constexpr (HasStore8<P>::value) {
#pragma unroll
      for (int i = 0; i < C::MT; ++i) {
        __syncthreads();
        __syncthreads();
      }
    }
    return;
  }

  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  uint64_t st_rt0 = 0, st_t0 = 0, st_t1 = 0, st_t2 = 0;
  bool stamp = false;
  if constexpr (HasStamps<P>::value) {
    stamp = p.stamps != nullptr && tid == 0;
    if (stamp) {
      st_rt0 = __builtin_amdgcn_s_memrealtime();
      st_t0 = __builtin_amdgcn_s_memtime();
    }
  }
  typename C::Acc acc;
  acc.zero();
  const bool do_colsum = C::kColSum && m0 == 0 && wm == 0;
  __syncthreads();
  if constexpr (HasStamps<P>::value)
    if (stamp) st_t1 = __builtin_amdgcn_s_memtime();
  int rbuf = 0;
  if constexpr (PIPE && BK == 32) {
    // Fragment reads one k16 step ahead: step 1 of stage kt is read before step 0's
    // MFMAs, and step 0 of stage kt + 1 (published by the previous barrier) before step
    // 1's, so no MFMA waits on the LDS latency of its own reads.
    typename C::FragA fa0, fa1;
    typename C::FragB fb0, fb1;
    if (nk > 0) C::read_frags(smem, smem + PA::BYTES, wm, wn, 0, lane, fa0, fb0);
    for (int kt = 0; kt < nk; ++kt) {
      const uint8_t* sa = smem + rbuf * STAGE;
      rbuf = rbuf == RING - 1 ? 0 : rbuf + 1;
      const uint8_t* na = smem + rbuf * STAGE;
      // Scheduling fences: without them the compiler sinks each read to just before its
      // first MFMA, to save registers, and the wave waits out the LDS latency there several
      // times per stage (round 5: lgkmcnt(0) waits between the MFMAs; fenced, the step went
      // 0.5096 -> 0.5048 ms; reads threaded one per MFMA gap measured 0.5132).
      C::read_frags(sa, sa + PA::BYTES, wm, wn, 1, lane, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      C::mfma_frags(fa0, fb0, acc, do_colsum);
      __builtin_amdgcn_sched_barrier(0);
      C::read_frags(na, na + PA::BYTES, wm, wn, 0, lane, fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      C::mfma_frags(fa1, fb1, acc, do_colsum);
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
    }
  } else {
    for (int kt = 0; kt < nk; ++kt) {
      const uint8_t* sa = smem + rbuf * STAGE;
      C::mma(sa, sa + PA::BYTES, wm, wn, lane, acc, do_colsum);
      rbuf = rbuf == RING - 1 ? 0 : rbuf + 1;
      __syncthreads();
    }
  }
  if constexpr (HasStamps<P>::value)
    if (stamp) st_t2 = __builtin_amdgcn_s_memtime();
  C::epilogue(p, smem, m0, n0, wave, wm, wn, lane, split, acc, do_colsum);
  if constexpr (HasStamps<P>::value) {
    if (stamp) {
      const uint64_t t3 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
      uint64_t* o = p.stamps + 8 * ((int64_t)blockIdx.z * gridDim.x + blockIdx.x);
      o[0] = st_rt0;
      o[1] = rt1;
      o[2] = st_t0;
      o[3] = st_t1;
      o[4] = st_t2;
      o[5] = t3;
    }
  }
}

// Tile order: B's panels slowest when B is the larger operand (N * planes > M * planes).
template <class P>
inline int p3_n_major(const P& p) {
  return (int64_t)p.N * P::B_PLANES > (int64_t)p.M * P::A_PLANES ? 1 : 0;
}

// TFLOP/s ceiling of a plane GEMM in algorithmic (f32) FLOPs: the f16 dense MFMA peak
// (= bf16's, 2.5 PF) over the MFMA terms per product (3 for two planes x two planes, 2
// with a one-plane operand).
template <class P>
constexpr double p3_peak_tflops() {
  return 2500.0 / (double)p3_nterms<P::A_PLANES, P::B_PLANES>();
}

template <class Kern>
inline hipError_t p3_set_lds(Kern* k, int lds) {
  if (lds <= 65536) return hipSuccess;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                             hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}

template <int BM, int BN, int WM, int WN, int BK, bool DEEP = true, class P>
inline hipError_t launch_gemm_p3(const P& p, int splits, hipStream_t st) {
  using C = P3Core<BM, BN, WM, WN, BK, P>;
  constexpr int STAGES_BYTES = 2 * C::STAGE;
  constexpr int LDS = STAGES_BYTES > C::EPI_BYTES ? STAGES_BYTES : C::EPI_BYTES;
  static_assert(LDS <= 160 * 1024, "two stages must fit the 160-KiB LDS of a CU");
  static hipError_t attr = p3_set_lds(&gemm_p3_kernel<BM, BN, WM, WN, BK, DEEP, P>, LDS);
  if (attr != hipSuccess) return attr;
  const int tiles = ((p.N + BN - 1) / BN) * ((p.M + BM - 1) / BM);
  hipLaunchKernelGGL((gemm_p3_kernel<BM, BN, WM, WN, BK, DEEP, P>), dim3(tiles, 1, splits),
                     dim3(C::NT), LDS, st, p, p3_n_major(p));
  return hipGetLastError();
}

// Warp-specialised variant (gemm_p3ws_kernel): 2 x WM x WN waves, a ring of 3 stages.
template <int BM, int BN, int WM, int WN, int BK, bool PIPE = false, class P>
inline hipError_t launch_gemm_p3ws(const P& p, int splits, hipStream_t st) {
  using C = P3Core<BM, BN, WM, WN, BK, P>;
  constexpr int RING_BYTES = 3 * C::STAGE;
  constexpr int LDS = RING_BYTES > C::EPI_BYTES ? RING_BYTES : C::EPI_BYTES;
  static_assert(LDS <= 160 * 1024, "three stages must fit the 160-KiB LDS of a CU");
  static hipError_t attr = p3_set_lds(&gemm_p3ws_kernel<BM, BN, WM, WN, BK, PIPE, P>, LDS);
  if (attr != hipSuccess) return attr;
  const int tiles = ((p.N + BN - 1) / BN) * ((p.M + BM - 1) / BM);
  hipLaunchKernelGGL((gemm_p3ws_kernel<BM, BN, WM, WN, BK, PIPE, P>), dim3(tiles, 1, splits),
                     dim3(2 * C::NT), LDS, st, p, p3_n_major(p));
  return hipGetLastError();
}

// LDS-DMA variant (gemm_p3g_kernel) with STAGES buffers.
template <int BM, int BN, int WM, int WN, int BK, int STAGES, class P>
inline hipError_t launch_gemm_p3g(const P& p, int splits, hipStream_t st) {
  using C = P3Core<BM, BN, WM, WN, BK, P>;
  constexpr int RING = STAGES * C::STAGE + 1024;
  constexpr int LDS = RING > C::EPI_BYTES ? RING : C::EPI_BYTES;
  static_assert(LDS <= 160 * 1024, "the stage ring must fit the 160-KiB LDS of a CU");
  static hipError_t attr = p3_set_lds(&gemm_p3g_kernel<BM, BN, WM, WN, BK, STAGES, P>, LDS);
  if (attr != hipSuccess) return attr;
  const int tiles = ((p.N + BN - 1) / BN) * ((p.M + BM - 1) / BM);
  hipLaunchKernelGGL((gemm_p3g_kernel<BM, BN, WM, WN, BK, STAGES, P>), dim3(tiles, 1, splits),
                     dim3(C::NT), LDS, st, p, p3_n_major(p));
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace acme
