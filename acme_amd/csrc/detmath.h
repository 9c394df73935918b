// Deterministic scalar math shared by the replay kernels.
//
// Reverb samples with an unseeded absl::BitGen (SURVEY.md §7 "Reference sampling is
// nondeterministic"), so "bit-exact index sampling under a fixed seed" is defined
// against a published, seedable generator: Philox4x32-10 (Salmon et al., SC'11, the
// generator rocRAND/cuRAND also ship).  The oracle (oracle/replay_oracle.c) restates
// the same published algorithms independently in plain C.
//
// Leaf values of the prioritized sum tree are p^alpha (Reverb Prioritized(alpha),
// configured at acme/agents/tf/dqn/agent.py:97).  Library pow() implementations are
// not bitwise identical between the GPU (ocml) and glibc, and a single differing ulp
// changes a tree sum and therefore a sampled index.  We therefore compute
// p^alpha = exp(alpha * log(p)) with the fdlibm log/exp algorithms (Sun Microsystems,
// public domain, the algorithms of e_log.c / e_exp.c), written with the operations
// in a fixed order and with FP contraction disabled, so host and device produce the
// same bits.
#pragma once

#include <stdint.h>

#ifdef __HIPCC__
#define ACME_HD __host__ __device__ __forceinline__
#else
#define ACME_HD static inline
#endif

namespace acme {

// ---------------------------------------------------------------- Philox4x32-10
struct u32x4 {
  uint32_t x, y, z, w;
};

ACME_HD uint32_t mulhilo32(uint32_t a, uint32_t b, uint32_t* hi) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}

ACME_HD u32x4 philox4x32_10(u32x4 ctr, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, hi1;
    uint32_t lo0 = mulhilo32(M0, ctr.x, &hi0);
    uint32_t lo1 = mulhilo32(M1, ctr.z, &hi1);
    u32x4 n;
    n.x = hi1 ^ ctr.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ ctr.w ^ k1;
    n.w = lo0;
    ctr = n;
    k0 += W0;
    k1 += W1;
  }
  return ctr;
}

// 53-bit uniform double in [0, 1) from two 32-bit words (exactly representable).
ACME_HD double u01_53(uint32_t a, uint32_t b) {
  const uint64_t hi = (uint64_t)(a >> 5);  // 27 bits
  const uint64_t lo = (uint64_t)(b >> 6);  // 26 bits
  return (double)(hi * 67108864ull + lo) * (1.0 / 9007199254740992.0);
}

// Counter layout for replay sampling: (sample index, step lo, step hi, stream tag).
constexpr uint32_t kSampleTag = 0x534D504Cu;  // "SMPL"
constexpr uint32_t kFillTag = 0x46494C4Cu;    // "FILL"

ACME_HD double sample_uniform(uint64_t seed, uint64_t step, uint32_t j) {
  u32x4 c = {j, (uint32_t)step, (uint32_t)(step >> 32), kSampleTag};
  u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return u01_53(r.x, r.y);
}

// ---------------------------------------------------------------- fdlibm log/exp
ACME_HD uint64_t f64_bits(double x) {
  union {
    double d;
    uint64_t u;
  } v;
  v.d = x;
  return v.u;
}
ACME_HD double f64_from_bits(uint64_t u) {
  union {
    double d;
    uint64_t u;
  } v;
  v.u = u;
  return v.d;
}

// Natural log for finite x > 0 (fdlibm e_log.c algorithm).
ACME_HD double det_log(double x) {
#pragma clang fp contract(off)
  const double ln2_hi = 6.93147180369123816490e-01;
  const double ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  uint64_t u = f64_bits(x);
  int k = 0;
  if ((u >> 52) == 0) {  // subnormal: scale up by 2^54
    x = x * 18014398509481984.0;
    u = f64_bits(x);
    k = -54;
  }
  k += (int)((u >> 52) & 0x7ff) - 1023;
  uint64_t mant = u & 0x000fffffffffffffull;
  // Normalise the mantissa to [sqrt(2)/2, sqrt(2)).
  // 0x6a09e667f3bcd is the fraction of sqrt(2).
  double m;
  if (mant >= 0x6a09e667f3bcdull) {
    m = f64_from_bits(mant | 0x3fe0000000000000ull);  // [sqrt2/2, 1)
    k += 1;
  } else {
    m = f64_from_bits(mant | 0x3ff0000000000000ull);  // [1, sqrt2)
  }
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double dk = (double)k;
  const double z = s * s;
  const double w = z * z;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

// exp(x) for |x| < 700 (fdlibm e_exp.c algorithm, no overflow/underflow paths:
// callers only pass alpha*log(p) for priorities in a sane range; results below the
// smallest normal are flushed to 0 which is harmless for a sampling weight).
ACME_HD double det_exp(double x) {
#pragma clang fp contract(off)
  const double ln2HI = 6.93147180369123816490e-01;
  const double ln2LO = 1.90821492927058770002e-10;
  const double invln2 = 1.44269504088896338700e+00;
  const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08;
  if (x > 709.0) return f64_from_bits(0x7ff0000000000000ull);
  if (x < -708.0) return 0.0;
  const int k = (int)(invln2 * x + (x < 0.0 ? -0.5 : 0.5));
  const double dk = (double)k;
  const double hi = x - dk * ln2HI;
  const double lo = dk * ln2LO;
  const double r = hi - lo;
  const double t = r * r;
  const double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  const double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
  // y in [0.5, 2): scale by 2^k through the exponent field.
  const uint64_t yb = f64_bits(y);
  const int64_t e = (int64_t)((yb >> 52) & 0x7ff) + k;
  if (e <= 0) return 0.0;
  return f64_from_bits((yb & 0x800fffffffffffffull) | ((uint64_t)e << 52));
}

// Sum-tree leaf weight p^alpha; p == 0 maps to 0 (never sampled), alpha == 1 and
// p == 1 are exact.
ACME_HD double det_pow_priority(double p, double alpha) {
#pragma clang fp contract(off)
  if (!(p > 0.0)) return 0.0;
  if (alpha == 1.0) return p;
  if (alpha == 0.0) return 1.0;
  return det_exp(alpha * det_log(p));
}

}  // namespace acme
