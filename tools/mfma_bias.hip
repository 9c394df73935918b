// Error structure of the plane engine's accumulation (VERDICT r5 item 1 diagnosis): does
// v_mfma_f32_32x32x16_f16 accumulating the three plane terms round without bias, and does it
// keep f16 subnormal inputs?  Many 32x32 tiles C = A (32 x K) B (K x 32) are computed
//   mode 0  as the engine does: per k16 step the terms (l,h), (h,l), (h,h) into one running acc;
//   mode 1  each k16 step's three terms into a zeroed acc, added to the running sum by a VALU add;
//   mode 2  the exact-f32 engine's v_mfma_f32_32x32x2f32 on the f32 values;
// and compared (host, f64) against the exact value of the same arithmetic: the planes' exact
// three-term sum (modes 0, 1) or the f32 values' exact product (all modes).  Printed per mode:
// rms error / rms(C), mean(err) / rms(err) and corr(err, sign(C)) (bias), over all tiles.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_bias.hip -o tools/mfma_bias && tools/mfma_bias
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

// A planes: [tile][plane][32 rows][K]; B planes: [tile][plane][32 cols][K] (k contiguous).
// Lane l: A row (l & 31), B column (l & 31), k = 8 (l >> 5) .. +7 of each k16 step.
// Modes (the ones above, and candidate fixes):
//   3  order (h,h), (h,l), (l,h) into the running acc (largest first)
//   4  small terms (l,h) + (h,l) in their own acc, (h,h) in another; summed at the end
//   5  two accs by k16 parity: even steps as mode 0, odd steps with A negated into the other;
//      result even - odd (the truncation's direction cancels between them)
//   6  mode 5 for (h,h) only, the small terms in a third acc
//   7  in place: the acc and A negated from K/2 on (one flip), result negated back
template <int MODE>
__global__ void __launch_bounds__(64) tile_kernel(const _Float16* ap, const _Float16* bp,
                                                  const float* af, const float* bf, int K,
                                                  float* out) {
  const int t = blockIdx.x, l = threadIdx.x, r = l & 31, kh = 8 * (l >> 5);
  const _Float16* A = ap + (size_t)t * 2 * 32 * K;
  const _Float16* B = bp + (size_t)t * 2 * 32 * K;
  f32x16 acc, sum;
  for (int v = 0; v < 16; ++v) acc[v] = sum[v] = 0.f;
  if constexpr (MODE == 2) {
    const float* Af = af + (size_t)t * 32 * K;
    const float* Bf = bf + (size_t)t * 32 * K;
    // v_mfma_f32_32x32x2f32: lane l holds A row (l & 31), k = (l >> 5); B column (l & 31).
    for (int k = 0; k < K; k += 2) {
      const float a = Af[r * K + k + (l >> 5)], b = Bf[r * K + k + (l >> 5)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
  } else {
    f32x16 acc2, acc3;
    for (int v = 0; v < 16; ++v) acc2[v] = acc3[v] = 0.f;
    for (int k = 0; k < K; k += 16) {
      f16x8 ah, al, bh, bl;
      for (int j = 0; j < 8; ++j) {
        ah[j] = A[(0 * 32 + r) * K + k + kh + j];
        al[j] = A[(1 * 32 + r) * K + k + kh + j];
        bh[j] = B[(0 * 32 + r) * K + k + kh + j];
        bl[j] = B[(1 * 32 + r) * K + k + kh + j];
      }
      const bool odd = (k >> 4) & 1;
      if constexpr (MODE == 1)
        for (int v = 0; v < 16; ++v) acc[v] = 0.f;
      if constexpr (MODE == 0 || MODE == 1) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
      } else if constexpr (MODE == 3) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
      } else if constexpr (MODE == 4) {
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc2, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc2, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
      } else if constexpr (MODE == 5) {
        if (!odd) {
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
        } else {
          const f16x8 nh = -ah, nl = -al;
          acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(nl, bh, acc2, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(nh, bl, acc2, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(nh, bh, acc2, 0, 0, 0);
        }
      } else if constexpr (MODE == 6) {
        acc3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc3, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc3, 0, 0, 0);
        if (!odd) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
        else acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(-ah, bh, acc2, 0, 0, 0);
      } else if constexpr (MODE == 7) {
        const bool neg = k >= K / 2;
        if (k == K / 2) acc = -acc;
        const f16x8 xh = neg ? -ah : ah, xl = neg ? -al : al;
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, bh, acc, 0, 0, 0);
      }
      if constexpr (MODE == 1)
        for (int v = 0; v < 16; ++v) sum[v] += acc[v];
    }
    if constexpr (MODE == 1) acc = sum;
    if constexpr (MODE == 4) acc = acc + acc2;
    if constexpr (MODE == 5) acc = acc - acc2;
    if constexpr (MODE == 6) acc = (acc - acc2) + acc3;
    if constexpr (MODE == 7) acc = -acc;
  }
  // C layout of the 32x32 MFMAs: acc[v] is row 8 (v / 4) + 4 (l >> 5) + (v % 4), column l & 31.
  for (int v = 0; v < 16; ++v) {
    const int row = 8 * (v / 4) + 4 * (l >> 5) + (v % 4);
    out[(size_t)t * 1024 + row * 32 + r] = acc[v];
  }
}

__global__ void subnormal_kernel(float* out) {
  // One product 2^-20 (an f16 subnormal) x 1 in C[0][0], and 2^-14 (the smallest normal).
  const int l = threadIdx.x;
  f16x8 a, b, c;
  for (int j = 0; j < 8; ++j) a[j] = b[j] = c[j] = (_Float16)0.f;
  if (l == 0) {
    a[0] = (_Float16)ldexpf(1.f, -20);
    b[0] = (_Float16)1.f;
    c[0] = (_Float16)ldexpf(1.f, -14);
  }
  f32x16 acc, acc2;
  for (int v = 0; v < 16; ++v) acc[v] = acc2[v] = 0.f;
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(c, b, acc2, 0, 0, 0);
  if (l == 0) {
    out[0] = acc[0];
    out[1] = acc2[0];
  }
}

struct Stats {
  double se = 0, sc = 0, sm = 0, ss = 0;
  long n = 0;
  void add(double err, double c) {
    se += err * err;
    sc += c * c;
    sm += err;
    ss += err * (c > 0 ? 1 : c < 0 ? -1 : 0);
    ++n;
  }
  void print(const char* what) const {
    const double rms_e = std::sqrt(se / n);
    printf("  %-34s rms err / rms C %.3e   mean/rms %+.4f   corr(err, sign C) %+.4f\n", what,
           rms_e / std::sqrt(sc / n), sm / n / rms_e, ss / n / rms_e);
  }
};

static void run(const char* name, int K, bool a_pos, int tiles) {
  std::mt19937_64 g(1234 + K + a_pos);
  std::normal_distribution<float> nd(0.f, 1.f);
  const size_t ne = (size_t)tiles * 32 * K;
  std::vector<float> af(ne), bf(ne);
  for (size_t i = 0; i < ne; ++i) {
    af[i] = nd(g);
    if (a_pos) af[i] = af[i] > 0 ? af[i] : 0.f;  // ReLU activations
    bf[i] = nd(g) * 1e-3f;                         // gradients
  }
  // Per-tensor power-of-two scales: max |x| w in [128, 256), as the engine's rescale sets.
  auto scale = [](const std::vector<float>& x) {
    float m = 0;
    for (float v : x) m = std::max(m, std::fabs(v));
    int e;
    std::frexp(m, &e);  // m in [2^(e-1), 2^e)
    return std::ldexp(1.f, 8 - e);
  };
  const float wa = scale(af), wb = scale(bf);
  std::vector<_Float16> ap(2 * ne), bp(2 * ne);
  std::vector<double> ah(ne), al(ne), bh(ne), bl(ne);
  for (int t = 0; t < tiles; ++t)
    for (int r = 0; r < 32; ++r)
      for (int k = 0; k < K; ++k) {
        const size_t i = ((size_t)t * 32 + r) * K + k;
        const float ya = af[i] * wa, yb = bf[i] * wb;
        const _Float16 h1 = (_Float16)ya, l1 = (_Float16)(ya - (float)h1);
        const _Float16 h2 = (_Float16)yb, l2 = (_Float16)(yb - (float)h2);
        const size_t o0 = ((size_t)t * 2 * 32 + r) * K + k, o1 = o0 + 32 * (size_t)K;
        ap[o0] = h1;
        ap[o1] = l1;
        bp[o0] = h2;
        bp[o1] = l2;
        ah[i] = (double)(float)h1;
        al[i] = (double)(float)l1;
        bh[i] = (double)(float)h2;
        bl[i] = (double)(float)l2;
      }
  _Float16 *dap, *dbp;
  float *daf, *dbf, *dout;
  CK(hipMalloc(&dap, 2 * ne * sizeof(_Float16)));
  CK(hipMalloc(&dbp, 2 * ne * sizeof(_Float16)));
  CK(hipMalloc(&daf, ne * sizeof(float)));
  CK(hipMalloc(&dbf, ne * sizeof(float)));
  CK(hipMalloc(&dout, (size_t)tiles * 1024 * sizeof(float)));
  CK(hipMemcpy(dap, ap.data(), 2 * ne * sizeof(_Float16), hipMemcpyHostToDevice));
  CK(hipMemcpy(dbp, bp.data(), 2 * ne * sizeof(_Float16), hipMemcpyHostToDevice));
  CK(hipMemcpy(daf, af.data(), ne * sizeof(float), hipMemcpyHostToDevice));
  CK(hipMemcpy(dbf, bf.data(), ne * sizeof(float), hipMemcpyHostToDevice));
  // Exact references (f64): the planes' three-term sum (in the scaled domain) and the f32 product.
  std::vector<double> ex3((size_t)tiles * 1024), exf((size_t)tiles * 1024);
  for (int t = 0; t < tiles; ++t)
    for (int r = 0; r < 32; ++r)
      for (int c = 0; c < 32; ++c) {
        double s3 = 0, sf = 0;
        const size_t ia = ((size_t)t * 32 + r) * K, ib = ((size_t)t * 32 + c) * K;
        for (int k = 0; k < K; ++k) {
          s3 += ah[ia + k] * bh[ib + k] + ah[ia + k] * bl[ib + k] + al[ia + k] * bh[ib + k];
          sf += (double)af[ia + k] * (double)bf[ib + k];
        }
        ex3[(size_t)t * 1024 + r * 32 + c] = s3;
        exf[(size_t)t * 1024 + r * 32 + c] = sf;
      }
  printf("%s (K %d, %d tiles)\n", name, K, tiles);
  std::vector<float> got((size_t)tiles * 1024);
  const double inv = 1.0 / ((double)wa * wb);
  for (int mode = 0; mode < 8; ++mode) {
    if (mode == 0) tile_kernel<0><<<tiles, 64>>>(dap, dbp, daf, dbf, K, dout);
    if (mode == 1) tile_kernel<1><<<tiles, 64>>>(dap, dbp, daf, dbf, K, dout);
    if (mode == 2) tile_kernel<2><<<tiles, 64>>>(dap, dbp, daf, dbf, K, dout);
    if (mode == 3) tile_kernel<3><<<tiles, 64>>>(dap, dbp, daf, dbf, K, dout);
    if (mode == 4) tile_kernel<4><<<tiles, 64>>>(dap, dbp, daf, dbf, K, dout);
    if (mode == 5) tile_kernel<5><<<tiles, 64>>>(dap, dbp, daf, dbf, K, dout);
    if (mode == 6) tile_kernel<6><<<tiles, 64>>>(dap, dbp, daf, dbf, K, dout);
    if (mode == 7) tile_kernel<7><<<tiles, 64>>>(dap, dbp, daf, dbf, K, dout);
    CK(hipGetLastError());
    CK(hipMemcpy(got.data(), dout, got.size() * sizeof(float), hipMemcpyDeviceToHost));
    Stats acc3, tot;
    for (size_t i = 0; i < got.size(); ++i) {
      if (mode != 2) {
        acc3.add((double)got[i] - ex3[i], ex3[i]);
        tot.add((double)got[i] * inv - exf[i], exf[i]);
      } else {
        tot.add((double)got[i] - exf[i], exf[i]);
      }
    }
    const char* mn[] = {"engine (running acc)", "fresh acc per k16 + VALU add", "f32 MFMA",
                        "largest term first", "small terms in own acc",
                        "two accs by k16 parity, odd negated", "hh by parity + small acc",
                        "one in-place flip at K/2"};
    printf(" mode %d: %s\n", mode, mn[mode]);
    if (mode != 2) acc3.print("accumulation vs exact 3-term sum");
    tot.print("total vs exact f32 product");
  }
  CK(hipFree(dap));
  CK(hipFree(dbp));
  CK(hipFree(daf));
  CK(hipFree(dbf));
  CK(hipFree(dout));
}

// One MFMA: C[0][0] = acc0 + sum_k a[k] b[k] (k < n <= 16), other entries zero.
__global__ void probe_kernel(const _Float16* a, const _Float16* b, float acc0, int n, float* out) {
  const int l = threadIdx.x;
  f16x8 fa, fb;
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * (l >> 5) + j;
    const bool row0 = (l & 31) == 0;
    fa[j] = row0 && k < n ? a[k] : (_Float16)0.f;
    fb[j] = row0 && k < n ? b[k] : (_Float16)0.f;
  }
  f32x16 acc;
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
  acc[0] = acc0;
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa, fb, acc, 0, 0, 0);
  if (l == 0) out[0] = acc[0];
}

static void probe(const char* what, float acc0, std::vector<double> prods) {
  // Each product p as a[k] b[k] with exact f16 factors: p = m 2^e -> a = m' , b = 2^e'.
  const int n = (int)prods.size();
  _Float16 ha[16], hb[16];
  double exact = acc0;
  for (int k = 0; k < 16; ++k) {
    ha[k] = hb[k] = (_Float16)0.f;
    if (k >= n) continue;
    int e;
    const double m = std::frexp(prods[k], &e);  // p = m 2^e, |m| in [0.5, 1)
    // a = m 2^ea, b = 2^eb with ea + eb = e, both in f16's normal range.
    const int ea = e / 2, eb = e - ea;
    ha[k] = (_Float16)std::ldexp(m, ea);
    hb[k] = (_Float16)std::ldexp(1.0, eb);
    exact += (double)(float)ha[k] * (double)(float)hb[k];
  }
  _Float16 *da, *db;
  float* dout;
  float got = 0;
  CK(hipMalloc(&da, sizeof(ha)));
  CK(hipMalloc(&db, sizeof(hb)));
  CK(hipMalloc(&dout, 4));
  CK(hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice));
  CK(hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice));
  probe_kernel<<<1, 64>>>(da, db, acc0, n, dout);
  CK(hipMemcpy(&got, dout, 4, hipMemcpyDeviceToHost));
  CK(hipFree(da));
  CK(hipFree(db));
  CK(hipFree(dout));
  const float lo = (float)exact <= exact ? (float)exact : std::nextafter((float)exact, -INFINITY);
  const float hi = (float)exact >= exact ? (float)exact : std::nextafter((float)exact, INFINITY);
  const float rn = (float)exact;
  const char* cls = got == rn && lo == hi ? "exact" : got == rn ? "RN" : got == lo ? "down" :
                    got == hi ? "up" : "other";
  printf("  %-40s exact %.12e got %.12e  [%s]%s\n", what, exact, (double)got, cls,
         got != rn ? " != RN" : "");
}

int main() {
  const double u = std::ldexp(1.0, -23);
  printf("rounding probes (one v_mfma_f32_32x32x16_f16, u = ulp(1)):\n");
  probe("0 + {1, 0.25u}", 0.f, {1.0, 0.25 * u});
  probe("0 + {1, 0.75u}", 0.f, {1.0, 0.75 * u});
  probe("0 + {1, -0.375u}", 0.f, {1.0, -0.375 * u});
  probe("0 + {-1, 0.25u}", 0.f, {-1.0, 0.25 * u});
  probe("0 + {-1, -0.25u}", 0.f, {-1.0, -0.25 * u});
  probe("0 + {-1, -0.75u}", 0.f, {-1.0, -0.75 * u});
  probe("1 + {0.25u}", 1.f, {0.25 * u});
  probe("1 + {0.75u}", 1.f, {0.75 * u});
  probe("-1 + {-0.25u}", -1.f, {-0.25 * u});
  probe("-1 + {-0.75u}", -1.f, {-0.75 * u});
  probe("1 + {-0.375u}", 1.f, {-0.375 * u});
  probe("0 + {1, 8 x 0.25u} (= 1 + 2u)", 0.f, {1.0, .25 * u, .25 * u, .25 * u, .25 * u, .25 * u, .25 * u, .25 * u, .25 * u});
  probe("1 + {8 x 0.25u} (= 1 + 2u)", 1.f, {.25 * u, .25 * u, .25 * u, .25 * u, .25 * u, .25 * u, .25 * u, .25 * u});
  probe("1 + {8 x 0.125u} (= 1 + u)", 1.f, {.125 * u, .125 * u, .125 * u, .125 * u, .125 * u, .125 * u, .125 * u, .125 * u});
  probe("1 + {8 x -0.125u} (= 1 - u)", 1.f, {-.125 * u, -.125 * u, -.125 * u, -.125 * u, -.125 * u, -.125 * u, -.125 * u, -.125 * u});
  probe("1 + {0.5u, 0.25u, 0.125u, 0.0625u}", 1.f, {.5 * u, .25 * u, .125 * u, .0625 * u});
  probe("0 + {1, 2^-30}", 0.f, {1.0, std::ldexp(1.0, -30)});
  probe("0 + {1, -2^-30}", 0.f, {1.0, -std::ldexp(1.0, -30)});
  probe("0 + {2^-20, 2^-20 x 3}", 0.f, {std::ldexp(1.0, -20), 3 * std::ldexp(1.0, -20)});
  float* d;
  CK(hipMalloc(&d, 2 * sizeof(float)));
  subnormal_kernel<<<1, 64>>>(d);
  float h[2];
  CK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  printf("subnormal f16 input 2^-20 x 1 -> %.6e (kept: %.6e); 2^-14 x 1 -> %.6e\n", h[0],
         ldexp(1.0, -20), h[1]);
  CK(hipFree(d));
  run("signed A, signed B", 256, false, 512);
  run("ReLU A, signed B", 256, true, 512);
  run("ReLU A, signed B", 4096, true, 64);
  return 0;
}
