// f64 complex FFT building blocks shared by the spectral front end (features.hip) and the Praat autocorrelation
// (f0.hip): radix-2/4/5/8 butterflies and one Stockham autosort stage, in place in LDS.
#pragma once
#include "common.h"

namespace svc {

__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ double2 mul_mi(double2 a) { return make_double2(a.y, -a.x); }  // -i a

// forward R-point DFTs in registers (V[q] = sum_r v[r] e^{-2 pi i r q / R})
template <int R>
__device__ __forceinline__ void bfly(double2* v);
template <>
__device__ __forceinline__ void bfly<2>(double2* v) {
  const double2 a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}
template <>
__device__ __forceinline__ void bfly<4>(double2* v) {
  const double2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]), t2 = cadd(v[1], v[3]), t3 = mul_mi(csub(v[1], v[3]));
  v[0] = cadd(t0, t2);
  v[2] = csub(t0, t2);
  v[1] = cadd(t1, t3);
  v[3] = csub(t1, t3);
}
template <>
__device__ __forceinline__ void bfly<8>(double2* v) {
  double2 e[4] = {v[0], v[2], v[4], v[6]}, o[4] = {v[1], v[3], v[5], v[7]};
  bfly<4>(e);
  bfly<4>(o);
  constexpr double h = 0.70710678118654752440;  // W_8 = (h, -h)
  const double2 w1 = make_double2(h, -h), w3 = make_double2(-h, -h);
  o[1] = cmul(o[1], w1);
  o[2] = mul_mi(o[2]);
  o[3] = cmul(o[3], w3);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = cadd(e[q], o[q]);
    v[q + 4] = csub(e[q], o[q]);
  }
}
template <>
__device__ __forceinline__ void bfly<5>(double2* v) {
  constexpr double c1 = 0.30901699437494742410, c2 = -0.80901699437494742410;  // cos(2 pi / 5), cos(4 pi / 5)
  constexpr double s1 = 0.95105651629515357212, s2 = 0.58778525229247312917;   // sin(2 pi / 5), sin(4 pi / 5)
  const double2 a1 = cadd(v[1], v[4]), a2 = cadd(v[2], v[3]), b1 = csub(v[1], v[4]), b2 = csub(v[2], v[3]);
  const double2 x0 = v[0];
  const double2 t1 = make_double2(x0.x + c1 * a1.x + c2 * a2.x, x0.y + c1 * a1.y + c2 * a2.y);
  const double2 t2 = make_double2(x0.x + c2 * a1.x + c1 * a2.x, x0.y + c2 * a1.y + c1 * a2.y);
  const double2 u1 = make_double2(s1 * b1.x + s2 * b2.x, s1 * b1.y + s2 * b2.y);
  const double2 u2 = make_double2(s2 * b1.x - s1 * b2.x, s2 * b1.y - s1 * b2.y);
  v[0] = cadd(x0, cadd(a1, a2));
  v[1] = cadd(t1, mul_mi(u1));
  v[4] = csub(t1, mul_mi(u1));
  v[2] = cadd(t2, mul_mi(u2));
  v[3] = csub(t2, mul_mi(u2));
}

// One Stockham stage of an N-point complex FFT (N = n/2) over the frame's z, radix R, NS = product of the earlier
// radices: butterfly b reads z[b + r N/R], multiplies by W_{NS R}^{r (b mod NS)} (= W_n^{2 N r (b mod NS) / (NS R)},
// the table tw holds W_n^m), and writes z[(b / NS) NS R + (b mod NS) + q NS]. All reads of the workgroup precede all
// writes (barrier), so the stage runs in place. tw(m) returns W_n^m (a table read, or a quarter-table lookup).
template <int N, int R, int NS, int TPF, typename TW>
__device__ __forceinline__ void fft_stage(double2* z, TW tw, int t) {
  constexpr int NB = N / R, PER = (NB + TPF - 1) / TPF, TS = 2 * N / (NS * R);
  static_assert(N % (NS * R) == 0, "radix plan");
  double2 v[PER][R];
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const int b = t + p * TPF;
    if (b < NB) {
      const int k = b % NS;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double2 x = z[b + r * NB];
        v[p][r] = (NS == 1 || r == 0) ? x : cmul(x, tw(r * k * TS));
      }
      bfly<R>(v[p]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const int b = t + p * TPF;
    if (b < NB) {
      const int k = b % NS, d = (b / NS) * NS * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) z[d + r * NS] = v[p][r];
    }
  }
  __syncthreads();
}


}  // namespace svc
