// How v_mfma_f32_32x32x16_f16 rounds its f32 accumulation (diagnostic for the plane
// engine's error structure, tools/grad_err_diag.py).  Each case puts one nonzero product
// (or a few) into column 0 of row 0 and an accumulator value, and prints the result next to
// the round-to-nearest-even and round-toward-zero answers.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_round.hip -o tools/mfma_round && tools/mfma_round
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Lane l holds A row (l & 31), k = 8 (l >> 5) .. +7 and B column (l & 31), same k.
__global__ void mfma_case(const _Float16* a, const _Float16* b, float acc0, int nterms, float* out) {
  const int l = threadIdx.x;
  f16x8 fa, fb;
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * (l >> 5) + j;
    const bool row0 = (l & 31) == 0;
    fa[j] = row0 && k < nterms ? a[k] : (_Float16)0.f;
    fb[j] = row0 && k < nterms ? b[k] : (_Float16)0.f;
  }
  f32x16 acc;
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
  acc[0] = acc0;  // lane 0's acc[0] is C[0][0]
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa, fb, acc, 0, 0, 0);
  if (l == 0) out[0] = acc[0];
}

static float run(float acc0, const float* av, const float* bv, int n) {
  _Float16 ha[16], hb[16];
  for (int i = 0; i < 16; ++i) {
    ha[i] = (_Float16)(i < n ? av[i] : 0.f);
    hb[i] = (_Float16)(i < n ? bv[i] : 0.f);
  }
  _Float16 *da, *db;
  float* dout;
  float out = 0.f;
  (void)hipMalloc(&da, sizeof(ha));
  (void)hipMalloc(&db, sizeof(hb));
  (void)hipMalloc(&dout, sizeof(float));
  (void)hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice);
  (void)hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
  mfma_case<<<1, 64>>>(da, db, acc0, n, dout);
  (void)hipMemcpy(&out, dout, sizeof(float), hipMemcpyDeviceToHost);
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dout);
  return out;
}

int main() {
  const float ulp = ldexpf(1.f, -23);
  struct Case {
    const char* what;
    float acc;
    float a[4], b[4];
    int n;
    double exact;
  } cs[] = {
      {"1 + 0.75 ulp", 1.f, {0.75f}, {ldexpf(1.f, -23)}, 1, 1.0 + 0.75 * ulp},
      {"-1 - 0.75 ulp", -1.f, {-0.75f}, {ldexpf(1.f, -23)}, 1, -1.0 - 0.75 * ulp},
      {"1 + 0.25 ulp", 1.f, {0.25f}, {ldexpf(1.f, -23)}, 1, 1.0 + 0.25 * ulp},
      {"1 - 0.25 ulp(1-)", 1.f, {-0.25f}, {ldexpf(1.f, -23)}, 1, 1.0 - 0.25 * ulp},
      {"1 + 0.5 ulp (tie, even)", 1.f, {0.5f}, {ldexpf(1.f, -23)}, 1, 1.0 + 0.5 * ulp},
      {"0 + 3 terms 1, 2^-24, 2^-24", 0.f, {1.f, 1.f, 1.f}, {1.f, ldexpf(1.f, -24), ldexpf(1.f, -24)}, 3,
       1.0 + 2 * ldexp(1.0, -24)},
      {"0 + 1 - 2^-25 ... (4 terms)", 0.f, {1.f, -1.f, 1.f, 1.f}, {1.f, ldexpf(1.f, -14), ldexpf(1.f, -12), ldexpf(1.f, -13)}, 4,
       1.0 - ldexp(1.0, -14) + ldexp(1.0, -12) + ldexp(1.0, -13)},
  };
  for (auto& c : cs) {
    const float got = run(c.acc, c.a, c.b, c.n);
    const float rn = (float)c.exact;
    const float rz = std::nextafter(rn, 0.f);
    const float rz2 = std::fabs((double)rn) > std::fabs(c.exact) ? rz : rn;  // toward zero
    printf("%-32s got %.10e  RN %.10e  RZ %.10e  -> %s\n", c.what, got, rn, rz2,
           got == rn && got == rz2 ? "exact" : got == rn ? "RN" : got == rz2 ? "RZ" : "other");
  }
  return 0;
}
