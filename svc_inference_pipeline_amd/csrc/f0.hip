// Praat autocorrelation pitch (parselmouth Sound.to_pitch_ac, utils/f0.py:120-161) on gfx950.
//
// Restates Praat's Sound_to_Pitch (AC, Hanning window, 3 periods) + Pitch_pathFinder, the same
// algorithm as oracle/praat_ac.py, in float64:
//   1. per utterance: sum, max and min of the samples (16 partial blocks); the global peak |x - mean| is
//      max(xmax - mean, mean - xmin) (f64 subtraction of a constant is monotonic: bit-equal to the max of |x - mean|)
//   2. per frame (one workgroup, f0_frame_kernel): local mean over one longest period each side, windowed frame,
//      local peak; the autocorrelation as Praat and the oracle compute it, by FFT (nfft = the power of two >= 1.5 nw:
//      the frame's real nfft-point spectrum from an nfft/2-point complex Stockham FFT, |X|^2, and the inverse real
//      transform as one more nfft/2-point complex FFT of the packed even / odd spectrum); r[lag] = ac[lag] / (ac[0] *
//      wR[lag]); the local maxima above half the voicing threshold, compacted in lag order (wave ballots), their
//      parabolic frequency and sinc(30) strength; the candidate list (Praat's sequential replacement rule). Each voiced
//      candidate is appended to a work list, and the frame's r row (the lags a refinement can reach) goes to HBM.
//   2b. per candidate (f0_brent_kernel, the work list at full occupancy): the Brent maximisation of the
//      sinc(70)-interpolated r around the candidate's peak. The sinc sums run on 8-lane groups (four lanes per side,
//      each a contiguous run of terms with Praat's angle-rotation recurrence started by sincospi).
//      (Refined inside the frame workgroup instead, one wave did a frame's ~5 candidates while the other three
//      waited: 1.23 ms of the frame kernel's 1.90 per 32 x 10 s batch; as its own pass 0.40 ms, r05c / r05g.)
//   3. per utterance: Viterbi path over candidates (voiced/unvoiced and octave-jump costs), then the
//      chosen frequencies are written zero-padded to the mel length (utils/f0.py:156-157).
// The Hann window, its normalised autocorrelation wR and the FFT's quarter twiddle table are host-built per parameter
// set and kept by the context (f0_tables).
//
// Provenance: the reference calls Praat through parselmouth; Praat (GPL v2 or later, P. Boersma & D. Weenink) is not in
// this image. sinc_interp / brent_neg_sinc below restate Praat's published NUM_interpolate_sinc and NUMminimize_brent
// (keeping Praat's variable names: midleft, halfsina, cosaa, daa ...) and the pitch path restates Sound_to_Pitch /
// Pitch_pathFinder (Boersma 1993), so that the F0 is comparable with what the reference computes; oracle/praat_ac.py
// restates the same algorithm in Python. Parity with Praat itself is unpinned (tests/test_f0.py).
#include <math.h>

#include <algorithm>
#include <vector>

#include "common.h"
#include "fft.h"

namespace svc {

constexpr int F0_MAXC = 16;  // >= max candidates (15 for the parselmouth defaults)
constexpr int F0_NT = 256;   // threads per frame workgroup
constexpr int F0_G = 8;      // lanes per sinc group (4 per side)
constexpr int F0_GP = 16;    // partial blocks of the per-utterance sum / max / min

struct F0Params {
  int nsp, hnsp, nw, hnw, maxlag, nf, bmax, maxc;
  int nfft;  // autocorrelation FFT length (power of two >= 1.5 nw)
  double dx, t1, x1, ts, floor_hz, ceiling, voicing, silence, octave_cost, octave_jump, vuv_cost;
};

static F0Params f0_params(int64_t n, double fs, double ts, double floor_hz, double ceiling) {
  F0Params P{};
  P.dx = 1.0 / fs;
  P.maxc = 15;
  if (P.maxc < ceiling / floor_hz) P.maxc = (int)floor(ceiling / floor_hz);
  P.nsp = (int)floor(1.0 / P.dx / floor_hz);
  P.hnsp = P.nsp / 2 + 1;
  if (ceiling > 0.5 / P.dx) ceiling = 0.5 / P.dx;
  const double dtw = 3.0 / floor_hz;
  int nw = (int)floor(dtw / P.dx);
  P.hnw = nw / 2 - 1;
  P.nw = 2 * P.hnw;
  P.maxlag = std::min((int)floor(P.nw / 3.0) + 2, P.nw);
  const double duration = (double)n * P.dx;
  P.nf = (int)floor((duration - dtw) / ts) + 1;
  P.x1 = 0.5 * P.dx;
  const double mid = P.x1 - 0.5 * P.dx + 0.5 * duration;
  P.t1 = mid - 0.5 * P.nf * ts + 0.5 * ts;
  P.ts = ts;
  P.bmax = (int)floor(P.nw * 0.5);
  P.floor_hz = floor_hz;
  P.ceiling = ceiling;
  P.nfft = 1;
  while (P.nfft < P.nw * 1.5) P.nfft *= 2;
  return P;
}

// ---------------------------------------------------------------------------- NUM helpers (y(i) = Praat's y[i + 1])
template <typename Y>
__device__ double sinc_interp(Y y, int n, double x, int depth) {
  const int midleft = (int)floor(x), midright = midleft + 1;
  if (x > n) return y(n - 1);
  if (x < 1) return y(0);
  if (x == (double)midleft) return y(midleft - 1);
  if (depth > midright - 1) depth = midright - 1;
  if (depth > n - midleft) depth = n - midleft;
  if (depth <= 0) return y((int)floor(x + 0.5) - 1);
  if (depth == 1) return y(midleft - 1) + (x - midleft) * (y(midright - 1) - y(midleft - 1));
  if (depth == 2) {
    double yl = y(midleft - 1), yr = y(midright - 1);
    double dyl = 0.5 * (yr - y(midleft - 2)), dyr = 0.5 * (y(midright) - yl);
    double fil = x - midleft, fir = midright - x;
    return yl * fir + yr * fil - fil * fir * (0.5 * (dyr - dyl) + (fil - 0.5) * (dyl + dyr - 2 * (yr - yl)));
  }
  const int left = midright - depth, right = midleft + depth;
  double result = 0.0;
  double a = M_PI * (x - midleft);
  double halfsina = 0.5 * sin(a);
  double aa = a / (x - left + 1.0), daa = M_PI / (x - left + 1.0);
  double cosaa = cos(aa), sinaa = sin(aa), cosdaa = cos(daa), sindaa = sin(daa);
  for (int ix = midleft; ix >= left; --ix) {
    double d = halfsina / a * (1.0 + cosaa);
    result += y(ix - 1) * d;
    a += M_PI;
    double h = cosaa * cosdaa - sinaa * sindaa;
    sinaa = cosaa * sindaa + sinaa * cosdaa;
    cosaa = h;
    halfsina = -halfsina;
  }
  a = M_PI * (midright - x);
  halfsina = 0.5 * sin(a);
  aa = a / (right - x + 1.0);
  daa = M_PI / (right - x + 1.0);
  cosaa = cos(aa);
  sinaa = sin(aa);
  cosdaa = cos(daa);
  sindaa = sin(daa);
  for (int ix = midright; ix <= right; ++ix) {
    double d = halfsina / a * (1.0 + cosaa);
    result += y(ix - 1) * d;
    a += M_PI;
    double h = cosaa * cosdaa - sinaa * sindaa;
    sinaa = cosaa * sindaa + sinaa * cosdaa;
    cosaa = h;
    halfsina = -halfsina;
  }
  return result;
}

// NUMminimize_brent on f(x) = -sinc(y, x, depth) over [a, b]; returns (x, f(x)). SINC: a group-wide sinc sum
// (sinc_group: uniform control flow within the group).
template <typename SINC, typename Y>
__device__ __forceinline__ double2 brent_neg_sinc(SINC sinc, Y y, int n, int depth, double a, double b, double tol) {
  const double golden = 1.0 - 0.6180339887498949;
  const double sqrt_eps = 1.4901161193847656e-08;  // sqrt(DBL_EPSILON)
  double v = a + golden * (b - a);
  double fv = -sinc(y, n, v, depth);
  double x = v, w = v, fx = fv, fw = fv;
  for (int it = 0; it < 60; ++it) {
    const double range = b - a, middle = (a + b) / 2;
    const double tol_act = sqrt_eps * fabs(x) + tol / 3;
    if (fabs(x - middle) + range / 2 <= 2 * tol_act) break;
    double new_step = golden * (x < middle ? b - x : a - x);
    if (fabs(x - w) >= tol_act) {
      double t = (x - w) * (fx - fv);
      double q = (x - v) * (fx - fw);
      double p = (x - v) * q - (x - w) * t;
      q = 2 * (q - t);
      if (q > 0) p = -p; else q = -q;
      if (fabs(p) < fabs(new_step * q) && p > q * (a - x + 2 * tol_act) && p < q * (b - x - 2 * tol_act))
        new_step = p / q;
    }
    if (fabs(new_step) < tol_act) new_step = new_step > 0 ? tol_act : -tol_act;
    const double t = x + new_step;
    const double ft = -sinc(y, n, t, depth);
    if (ft <= fx) {
      if (t < x) b = x; else a = x;
      v = w; w = x; x = t;
      fv = fw; fw = fx; fx = ft;
    } else {
      if (t < x) a = t; else b = t;
      if (ft <= fw || w == x) {
        v = w; w = t;
        fv = fw; fw = ft;
      } else if (ft <= fv || v == x || v == w) {
        v = t;
        fv = ft;
      }
    }
  }
  return make_double2(x, fx);
}

// Ragged batches: per-utterance sound length and the frame grid it implies (f0_params of that length), set by the
// host; NULL = every utterance has the batch length (the uniform P). Rows keep the batch stride (n_max samples,
// nf_max frames, T_max output frames).
struct F0Utt {
  int64_t n;  // samples
  double t1;  // first frame time
  int nf;     // frames
  int pad;    // left zero padding of the mel-length output (utils/f0.py:156-157)
  int T;      // mel frames of this utterance
};

// ---------------------------------------------------------------------------- kernels
// per-utterance partial sum / max / min over F0_GP contiguous blocks: part[(b * F0_GP + g) * 3 + {0, 1, 2}]
__global__ __launch_bounds__(256) void f0_global_kernel(const float* __restrict__ wav, int64_t stride,
                                                        const F0Utt* __restrict__ utt, double* __restrict__ part,
                                                        int* __restrict__ work_count) {
  const int g = blockIdx.x, b = blockIdx.y;
  if (g == 0 && b == 0 && threadIdx.x == 0) *work_count = 0;  // the Brent work list of this call (stream-ordered)
  const float* x = wav + (int64_t)b * stride;
  const int64_t n = utt ? utt[b].n : stride;
  const int64_t per = (n + F0_GP - 1) / F0_GP, i0 = (int64_t)g * per, i1 = std::min(n, i0 + per);
  double s = 0.0;
  float mx = -INFINITY, mn = INFINITY;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
    const float v = x[i];
    s += (double)v;
    mx = fmaxf(mx, v);
    mn = fminf(mn, v);
  }
  __shared__ double rs[4];
  __shared__ float rx[4], rn[4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    mx = fmaxf(mx, __shfl_xor(mx, o));
    mn = fminf(mn, __shfl_xor(mn, o));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    rs[w] = s;
    rx[w] = mx;
    rn[w] = mn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double* p = part + ((int64_t)b * F0_GP + g) * 3;
    p[0] = (rs[0] + rs[1]) + (rs[2] + rs[3]);
    p[1] = (double)fmaxf(fmaxf(rx[0], rx[1]), fmaxf(rx[2], rx[3]));
    p[2] = (double)fminf(fminf(rn[0], rn[1]), fminf(rn[2], rn[3]));
  }
}

__device__ double block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
  return t;
}

__device__ double block_max(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = red[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) t = fmax(t, red[w]);
  return t;
}

// 1 / a to within an ulp: v_rcp_f64 and two Newton steps (the sinc terms' a = pi (h + q) are normal positive numbers)
__device__ __forceinline__ double rcp_nr(double a) {
  double r = __builtin_amdgcn_rcp(a);
  double e = fma(-a, r, 1.0);
  r = fma(r, e, r);
  e = fma(-a, r, 1.0);
  return fma(r, e, r);
}

// NUM_interpolate_sinc on a G-lane group (x and depth group-uniform, depth <= DEPTH; every lane of the group returns
// the same value): lanes [0, G/2) take the left terms ix = midleft - q, lanes [G/2, G) the right terms ix = midright +
// q, each lane a contiguous run of at most K = DEPTH / (G/2) terms. With h = x - midleft (left) or midright - x (right),
// term q is
//   y[ix] * (-1)^q * (sin(pi h) / 2) / a_q * (1 + cos(aa_q)),   a_q = pi (h + q),   aa_q = a_q / (h + depth)
// as Praat's recurrence forms it (a += pi; aa rotated by daa = pi / (h + depth)); a lane starts its run's angle with
// sincospi and continues with the same rotation, and loads its run's y values before the first term. The group's
// partial sums meet in an xor butterfly, so every lane adds the same pairs and ends with the same bits. Equal to
// sinc_interp up to rounding (~1e-15 relative).
template <int G, int DEPTH, typename Y>
__device__ double sinc_group(Y y, int n, double x, int depth, int gl) {
  const int midleft = (int)floor(x), midright = midleft + 1;
  if (x > n) return y(n - 1);
  if (x < 1) return y(0);
  if (x == (double)midleft) return y(midleft - 1);
  if (depth > midright - 1) depth = midright - 1;
  if (depth > n - midleft) depth = n - midleft;
  if (depth <= 2) return sinc_interp(y, n, x, depth);
  constexpr int H = G / 2, K = (DEPTH + H - 1) / H;
  const bool rs = gl >= H;
  const int c = rs ? gl - H : gl;
  const double h = rs ? (double)midright - x : x - (double)midleft;
  const int k = (depth + H - 1) / H;
  const int q0 = c * k, q1 = min(q0 + k, depth);
  const int i0 = rs ? midright - 1 : midleft - 1, step = rs ? 1 : -1;
  double yv[K];
#pragma unroll
  for (int j = 0; j < K; ++j) yv[j] = q0 + j < q1 ? y(i0 + step * (q0 + j)) : 0.0;
  double part = 0.0;
  if (q0 < q1) {
    const double inv = 1.0 / (h + (double)depth);
    double sd, cd, sn, cs;
    sincospi(inv, &sd, &cd);
    sincospi((h + (double)q0) * inv, &sn, &cs);
    const double hs0 = 0.5 * sinpi(h);
    double hs = (q0 & 1) ? -hs0 : hs0;
    double a = M_PI * (h + (double)q0);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (q0 + j < q1) {
        part = fma(yv[j], hs * rcp_nr(a) * (1.0 + cs), part);
        const double t = cs * cd - sn * sd;
        sn = cs * sd + sn * cd;
        cs = t;
        hs = -hs;
        a += M_PI;
      }
    }
  }
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) part += __shfl_xor(part, o);
  return part;
}

struct F0Out {
  double* freq;   // [B*nf][F0_MAXC]
  double* str;    // [B*nf][F0_MAXC]
  int* ncand;     // [B*nf]
  double* inten;  // [B*nf]
  int* cim;       // [B*nf][F0_MAXC] the lag of each candidate's autocorrelation peak (for the Brent refinement)
  double* rwin;   // [B*nf][rw] r at lags 0 .. rw - 1 (r is even: the Brent sums read |lag|)
  int rw;         // lags kept per frame: every lag a sinc(70) sum around a candidate peak can reach (iend + 72)
  int* work;      // [1 + B*nf*(F0_MAXC-1)]: work[0] = count, then the (frame * F0_MAXC + candidate) slots to refine
};

// Frame pass. tab: [win: nw][wR: bmax + 1][pad to even][twq: N/2 double2 = W_nfft^m, m < nfft/4] (f0_tables).
// LDS: the N complex points of the FFT, reused in turn for the power spectrum, r and the peak lists, and the quarter
// twiddle table: 24 N bytes (24 KiB at nfft 2048), so six frame workgroups share a CU.
template <int N>
__global__ __launch_bounds__(F0_NT) void f0_frame_kernel(const float* __restrict__ wav, int64_t n, F0Params P,
                                                         const double* __restrict__ tab,
                                                         const double* __restrict__ gpart, F0Out o,
                                                         const F0Utt* __restrict__ utt) {
  static_assert(2 * N == 512 || 2 * N == 1024 || 2 * N == 2048 || 2 * N == 4096, "nfft");
  constexpr int PR = (N + F0_NT - 1) / F0_NT;  // complex points per thread
  extern __shared__ __align__(16) unsigned char f0sm[];
  double2* zs = reinterpret_cast<double2*>(f0sm);              // [N]
  double* zf = reinterpret_cast<double*>(f0sm);                // the same, as 2N doubles
  double2* twq = reinterpret_cast<double2*>(f0sm + 16 * N);    // [N / 2]
  __shared__ double red[4];
  __shared__ int wcnt[4];
  __shared__ int npk_s, ncs;
  __shared__ double cf[F0_MAXC], cs[F0_MAXC];
  __shared__ int cim[F0_MAXC];
  const int fi = blockIdx.x, b = blockIdx.y;
  if (utt && fi >= utt[b].nf) return;  // past this utterance's frames (block-uniform, before any barrier)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double* win = tab;
  const double* winR = tab + P.nw;
  const double2* twg = reinterpret_cast<const double2*>(tab + ((P.nw + P.bmax + 2) & ~1));
  for (int i = tid; i < N / 2; i += F0_NT) twq[i] = twg[i];
  // W_nfft^m from the quarter table: m = q (N/2) + j -> (-i)^q W^j
  const auto tw = [twq](int m) {
    const double2 w = twq[m & (N / 2 - 1)];
    switch ((m / (N / 2)) & 3) {
      case 0: return w;
      case 1: return make_double2(w.y, -w.x);
      case 2: return make_double2(-w.x, -w.y);
      default: return make_double2(-w.y, w.x);
    }
  };
  const float* x = wav + (int64_t)b * n;
  const double t = (utt ? utt[b].t1 : P.t1) + fi * P.ts;
  const int left = (int)floor((t - P.x1) / P.dx) + 1;  // 1-based
  const int right = left + 1;
  // local mean: 1-based samples [right - nsp, left + nsp]
  double s = 0;
  for (int i = right - P.nsp + tid; i <= left + P.nsp; i += F0_NT) s += (double)x[i - 1];
  const double lmean = block_sum(s, red) / (2.0 * P.nsp);
  const int start = right - P.hnw;  // 1-based
  for (int j = tid; j < 2 * N; j += F0_NT) zf[j] = j < P.nw ? ((double)x[start - 1 + j] - lmean) * win[j] : 0.0;
  __syncthreads();
  int s0 = P.hnw + 1 - P.hnsp, s1 = P.hnw + P.hnsp;
  if (s0 < 1) s0 = 1;
  if (s1 > P.nw) s1 = P.nw;
  double lp = 0;
  for (int j = s0 - 1 + tid; j < s1; j += F0_NT) lp = fmax(lp, fabs(zf[j]));
  const double local_peak = block_max(lp, red);
  const int gf = b * P.nf + fi;
  if (tid == 0) {
    // global peak: max(xmax - mean, mean - xmin) over the partial blocks (summed in block order)
    const double* pp = gpart + (int64_t)b * F0_GP * 3;
    double tot = 0.0, mx = -INFINITY, mn = INFINITY;
    for (int g = 0; g < F0_GP; ++g) {
      tot += pp[3 * g];
      mx = fmax(mx, pp[3 * g + 1]);
      mn = fmin(mn, pp[3 * g + 2]);
    }
    const double mean = tot / (double)(utt ? utt[b].n : n);
    const double gp = fmax(mx - mean, mean - mn);
    o.inten[gf] = local_peak > gp ? 1.0 : local_peak / gp;
    o.freq[(int64_t)gf * F0_MAXC] = 0.0;  // candidate 0: unvoiced
    o.str[(int64_t)gf * F0_MAXC] = 0.0;
  }
  if (local_peak == 0.0) {
    if (tid == 0) o.ncand[gf] = 1;
    return;
  }
  // ---- autocorrelation by FFT (Praat: the frame zero-padded to nfft, |FFT|^2, inverse FFT)
  const auto fft = [&]() {
    fft_stage<N, 4, 1, F0_NT>(zs, tw, tid);
    fft_stage<N, 4, 4, F0_NT>(zs, tw, tid);
    fft_stage<N, 4, 16, F0_NT>(zs, tw, tid);
    fft_stage<N, 4, 64, F0_NT>(zs, tw, tid);
    if constexpr (N == 256) {
      // (4^4: done)
    } else if constexpr (N == 1024) {
      fft_stage<N, 4, 256, F0_NT>(zs, tw, tid);
    } else if constexpr (N == 2048) {
      fft_stage<N, 4, 256, F0_NT>(zs, tw, tid);
      fft_stage<N, 2, 1024, F0_NT>(zs, tw, tid);
    } else {
      fft_stage<N, 2, 256, F0_NT>(zs, tw, tid);
    }
  };
  fft();
  // real-input split X[k] = (Z[k] + Z*[N-k]) / 2 + W^k (Z[k] - Z*[N-k]) / 2i, power P[k] = |X[k]|^2, k = 0..N: a
  // thread takes the pair (k, N - k) (one read of Z[k], Z[N - k]) and writes P over zs's doubles after a barrier
  double pw[2][(N / 2 + F0_NT) / F0_NT];
  {
    int q = 0;
    for (int k = tid; k <= N / 2; k += F0_NT, ++q) {
      const double2 za = zs[k], zb = zs[k == 0 ? 0 : N - k];
      const auto power = [&](double2 zk, double2 zm, int kk) {
        const double2 e = make_double2(0.5 * (zk.x + zm.x), 0.5 * (zk.y - zm.y));
        const double2 od = make_double2(0.5 * (zk.y + zm.y), -0.5 * (zk.x - zm.x));
        const double2 X = cadd(e, cmul(od, tw(kk)));
        return X.x * X.x + X.y * X.y;
      };
      pw[0][q] = power(za, zb, k);       // X[k]: Z[k], Z[N-k]
      pw[1][q] = power(zb, za, N - k);   // X[N-k]: Z[N-k] (Z[0] for k = 0, i.e. Z[N]), Z[k]
    }
    __syncthreads();
    q = 0;
    for (int k = tid; k <= N / 2; k += F0_NT, ++q) {
      zf[k] = pw[0][q];
      zf[N - k] = pw[1][q];
    }
    __syncthreads();
  }
  // inverse real transform: the autocorrelation a (2N real, even) packed as y[m] = a[2m] + i a[2m+1] has the N-point
  // spectrum Y[k] = E[k] + i O[k], E = (P[k] + P[N-k]) / 2, O = (P[k] - P[N-k]) conj(W^k) / 2; y = conj(FFT(conj(Y)))
  // / N. The factors 1/2 and 1/N are exact powers of two and cancel in r, so they are left out.
  {
    double2 yv[PR];
#pragma unroll
    for (int q = 0; q < PR; ++q) {
      const int k = tid + q * F0_NT;
      if (k < N) {
        const double pk = zf[k], pm = zf[N - k];
        const double E = pk + pm, Pd = pk - pm;
        const double2 w = tw(k);
        yv[q] = make_double2(E + Pd * w.y, -Pd * w.x);  // conj(E + i Pd (w.x - i w.y))
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PR; ++q) {
      const int k = tid + q * F0_NT;
      if (k < N) zs[k] = yv[q];
    }
    __syncthreads();
  }
  fft();
  // a[2m] = Re, a[2m+1] = -Im of the transform; r[lag] = a[lag] / (a[0] wR[lag]), r[0] = 1, mirrored to negative lags
  // (r over zs's doubles after a barrier); lags < rw also to the frame's global row for the Brent pass
  const int rn = 2 * P.bmax + 1;
  {
    constexpr int LR = (2 * N / 3 + 2 + F0_NT) / F0_NT;  // bmax + 1 <= nw / 2 + 1 <= 2N / 3 + 1 lags
    double rv[LR];
    const double ac0 = zs[0].x;
#pragma unroll
    for (int q = 0; q < LR; ++q) {
      const int lag = tid + q * F0_NT;
      if (lag <= P.bmax) {
        const double2 zz = zs[lag >> 1];
        rv[q] = lag == 0 ? 1.0 : ((lag & 1) ? -zz.y : zz.x) / (ac0 * winR[lag]);
      }
    }
    __syncthreads();
    double* rg = o.rwin + (int64_t)gf * o.rw;
#pragma unroll
    for (int q = 0; q < LR; ++q) {
      const int lag = tid + q * F0_NT;
      if (lag <= P.bmax) {
        zf[P.bmax + lag] = rv[q];
        zf[P.bmax - lag] = rv[q];
        if (lag < o.rw) rg[lag] = rv[q];
      }
    }
    __syncthreads();
  }
  const double* r = zf;
  const auto ry = [r](int i) { return r[i]; };
  const int iend = P.maxlag < P.bmax ? P.maxlag : P.bmax;
  // ---- local maxima above half the voicing threshold, in lag order: frequency, strength and lag lists past r
  const int cap = (iend + 1) / 2 + 2;
  double* pk_f = zf + ((rn + 1) & ~1);
  double* pk_s = pk_f + cap;
  int* pk_i = reinterpret_cast<int*>(pk_s + cap);
  if (tid == 0) npk_s = 0;
  for (int base = 2; base < iend; base += F0_NT) {
    const int i = base + tid;
    bool peak = false;
    double freq = 0.0;
    if (i < iend) {
      const double ri = r[P.bmax + i], rm = r[P.bmax + i - 1], rp = r[P.bmax + i + 1];
      if (ri > 0.5 * P.voicing && ri > rm && ri >= rp) {
        peak = true;
        const double dr = 0.5 * (rp - rm), d2r = 2.0 * ri - rm - rp;
        freq = 1.0 / P.dx / (i + dr / d2r);
      }
    }
    const uint64_t m = __ballot(peak);
    const int rank = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wcnt[wave] = __popcll(m);
    __syncthreads();
    int off = npk_s;
    for (int w = 0; w < wave; ++w) off += wcnt[w];
    if (peak) {
      pk_i[off + rank] = i;
      pk_f[off + rank] = freq;
    }
    __syncthreads();
    if (tid == 0) npk_s += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    __syncthreads();
  }
  const int npk = npk_s;
  const int grp = tid / F0_G, gl = tid % F0_G;
  constexpr int NG = F0_NT / F0_G;
  // sinc(30) strength of every peak, a group per peak
  for (int p = grp; p < npk; p += NG) {
    double strength = sinc_group<F0_G, 30>(ry, rn, 1.0 / P.dx / pk_f[p] + P.bmax + 1, 30, gl);
    if (strength > 1.0) strength = 1.0 / strength;
    if (gl == 0) pk_s[p] = strength;
  }
  __syncthreads();
  if (tid == 0) {  // the candidate list in lag order (Praat's replacement rule is sequential)
    int nc = 1;
    cf[0] = 0.0;
    cs[0] = 0.0;
    cim[0] = 0;
    for (int p = 0; p < npk; ++p) {
      const double freq = pk_f[p], strength = pk_s[p];
      int place = 0;
      if (nc < P.maxc) {
        place = nc++;
      } else {
        double weakest = 2.0;
        for (int iw = 1; iw < P.maxc; ++iw) {
          const double ls = cs[iw] - P.octave_cost * log2(P.floor_hz / cf[iw]);
          if (ls < weakest) {
            weakest = ls;
            place = iw;
          }
        }
        if (strength - P.octave_cost * log2(P.floor_hz / freq) <= weakest) place = 0;
      }
      if (place) {
        cf[place] = freq;
        cs[place] = strength;
        cim[place] = pk_i[p];
      }
    }
    ncs = nc;
  }
  __syncthreads();
  const int nc = ncs;
  __shared__ int wbase;
  if (tid == 0) {
    o.ncand[gf] = nc;
    wbase = nc > 1 ? atomicAdd(o.work, nc - 1) : 0;  // the Brent pass's work list: one slot per voiced candidate
  }
  __syncthreads();
  if (tid < nc) o.cim[(int64_t)gf * F0_MAXC + tid] = cim[tid];
  if (tid >= 1 && tid < nc) o.work[1 + wbase + tid - 1] = gf * F0_MAXC + tid;
}

// Brent pass: NUMimproveExtremum of the sinc(70)-interpolated r around every candidate peak, a group of F0_G lanes per
// (frame, candidate) slot (F0_MAXC slots per frame, slot 0 is the unvoiced candidate): frames' candidates are
// independent, so this runs at full occupancy instead of inside the frame pass's workgroup (where one wave refined a
// frame's few candidates while its other waves waited).
template <int GB>
__global__ __launch_bounds__(F0_NT) void f0_brent_kernel(F0Params P, F0Out o) {
  const int grp = threadIdx.x / GB, gl = threadIdx.x % GB;
  const int64_t item = (int64_t)blockIdx.x * (F0_NT / GB) + grp;
  if (item >= o.work[0]) return;  // group-uniform (the grid covers the worst case, every frame voiced x maxc - 1)
  const int slot = o.work[1 + item];
  const int gf = slot / F0_MAXC, kc = slot % F0_MAXC;
  const double* rg = o.rwin + (int64_t)gf * o.rw;
  const int bmax = P.bmax, rn = 2 * bmax + 1;
  const auto ry = [rg, bmax](int i) { const int l = i - bmax; return rg[l < 0 ? -l : l]; };
  const int ixmid = o.cim[(int64_t)gf * F0_MAXC + kc] + bmax + 1;
  double xmid, ymid;
  if (ixmid <= 1) {
    xmid = 1.0;
    ymid = ry(0);
  } else if (ixmid >= rn) {
    xmid = rn;
    ymid = ry(rn - 1);
  } else {
    auto sg = [gl](decltype(ry) y, int nn, double xx, int depth) { return sinc_group<GB, 70>(y, nn, xx, depth, gl); };
    const double2 m = brent_neg_sinc(sg, ry, rn, 70, ixmid - 1, ixmid + 1, 1e-10);
    xmid = m.x;
    ymid = -m.y;
  }
  xmid -= bmax + 1;
  const double freq = 1.0 / P.dx / xmid;
  if (ymid > 1.0) ymid = 1.0 / ymid;
  if (gl == 0) {
    o.freq[(int64_t)gf * F0_MAXC + kc] = freq;
    o.str[(int64_t)gf * F0_MAXC + kc] = ymid;
  }
}

// Pitch_pathFinder + padding to T (one wave per utterance)
// ps_lds: the back-pointers of all frames fit in dynamic LDS as bytes (nf * F0_MAXC bytes), so the final serial
// backtrack chases LDS instead of global memory; otherwise they go to psi (global).
__global__ void f0_path_kernel(F0Params P, F0Out o, int* __restrict__ psi, int T, int pad, double* __restrict__ f0out,
                               int ps_lds, const F0Utt* __restrict__ utt) {
  extern __shared__ unsigned char psl[];
  const int b = blockIdx.x;
  // frame-array stride is the batch's P.nf; this utterance's own frame count / padding / length come from utt
  const int nf_stride = P.nf;
  const int Tb = utt ? utt[b].T : T;
  if (utt) {
    P.nf = utt[b].nf;
    pad = utt[b].pad;
  }
  const int j = threadIdx.x;
  const int jc = threadIdx.x >> 4, kk = threadIdx.x & 15;  // blockDim = 16 * F0_MAXC... at least F0_MAXC x 16
  // The Viterbi recursion is serial over frames, so each step must not wait on global memory: the candidates of
  // F0_PCH frames at a time are staged in LDS by the whole block (one load latency per chunk instead of several per
  // frame), and the previous frame's frequencies stay in LDS. Same arithmetic as before, value for value.
  constexpr int F0_PCH = 64;
  __shared__ double dprev[F0_MAXC], dcur[F0_MAXC], pfr[F0_MAXC], dlv[F0_MAXC];
  __shared__ double vals[F0_MAXC][16];
  __shared__ double cfr[F0_PCH][F0_MAXC], cst[F0_PCH][F0_MAXC], cin[F0_PCH];
  __shared__ int cnc[F0_PCH];
  __shared__ int pnc;
  const double tsc = 0.01 / P.ts;
  const double ojc = P.octave_jump * tsc, vuv = P.vuv_cost * tsc;
  const double ceil2 = P.ceiling;
  int* ps = psi + (int64_t)b * nf_stride * F0_MAXC;
  for (int i = 0; i < P.nf; ++i) {
    const int gf = b * nf_stride + i;
    const int li = i % F0_PCH;
    if (li == 0) {
      __syncthreads();
      const int nch = min(F0_PCH, P.nf - i);
      for (int q = j; q < nch * F0_MAXC; q += blockDim.x) {
        const int fi = q / F0_MAXC, c = q - fi * F0_MAXC;
        cfr[fi][c] = o.freq[(int64_t)(gf + fi) * F0_MAXC + c];
        cst[fi][c] = o.str[(int64_t)(gf + fi) * F0_MAXC + c];
      }
      for (int q = j; q < nch; q += blockDim.x) {
        cnc[q] = o.ncand[gf + q];
        cin[q] = o.inten[gf + q];
      }
      __syncthreads();
    }
    const int nc = cnc[li];
    // thread (jc, kk): jc = candidate of this frame, kk = candidate of the previous frame; the kk == 0 threads own jc
    if (kk == 0 && jc < nc) {
      const double inten = cin[li];
      double us = P.silence <= 0 ? 0 : 2.0 - inten / (P.silence / (1.0 + P.voicing));
      us = P.voicing + (us > 0 ? us : 0.0);
      const double f2 = cfr[li][jc];
      const bool voiced = f2 > 0.0 && f2 < ceil2;
      dlv[jc] = voiced ? cst[li][jc] - P.octave_cost * log2(P.ceiling / f2) : us;
    }
    __syncthreads();
    if (i == 0) {
      if (kk == 0 && jc < nc) dcur[jc] = dlv[jc];
    } else {
      const int np = pnc;
      if (jc < nc && kk < np) {  // every transition of the step at once (the log2s were the serial chain)
        const double f2 = cfr[li][jc];
        const bool v2 = f2 > 0.0 && f2 < ceil2;
        const double f1 = pfr[kk];
        const bool v1 = f1 > 0.0 && f1 < ceil2;
        double tc;
        if (!v2) tc = v1 ? vuv : 0.0;
        else tc = v1 ? ojc * fabs(log2(f1 / f2)) : vuv;
        vals[jc][kk] = dprev[kk] - tc + dlv[jc];
      }
      __syncthreads();
      if (kk == 0 && jc < nc) {  // best predecessor in kk order, first maximum wins (as the serial loop)
        double best = -1e30;
        int place = 0;
        for (int q = 0; q < np; ++q)
          if (vals[jc][q] > best) {
            best = vals[jc][q];
            place = q;
          }
        dcur[jc] = best;
        if (ps_lds)
          psl[i * F0_MAXC + jc] = (unsigned char)place;
        else
          ps[(int64_t)i * F0_MAXC + jc] = place;
      }
    }
    __syncthreads();
    if (kk == 0 && jc < nc) {
      dprev[jc] = dcur[jc];
      pfr[jc] = cfr[li][jc];
    }
    if (threadIdx.x == 0) pnc = nc;
    __syncthreads();
  }
  if (j == 0) {
    double* out = f0out + (int64_t)b * T;
    for (int t = 0; t < T; ++t) out[t] = 0.0;
    const int gl = b * nf_stride + P.nf - 1;
    int place = 0;
    double best = dprev[0];
    for (int kk = 1; kk < o.ncand[gl]; ++kk)
      if (dprev[kk] > best) {
        best = dprev[kk];
        place = kk;
      }
    for (int i = P.nf - 1; i >= 0; --i) {
      const int gf = b * nf_stride + i;
      const int t = pad + i;
      if (t >= 0 && t < Tb) out[t] = o.freq[(int64_t)gf * F0_MAXC + place];
      place = i > 0 ? (ps_lds ? (int)psl[i * F0_MAXC + place] : ps[(int64_t)i * F0_MAXC + place]) : 0;
    }
  }
}

// lags of r the Brent pass reads: a candidate peak lies below iend = min(maxlag, bmax), and a sinc(70) sum over x in
// [peak lag - 1, peak lag + 1] reaches 71 lags past it
// (and never past bmax: the sums stop at the end of r)
static int f0_rw(const F0Params& P) { return std::min((std::min(P.maxlag, P.bmax) + 72 + 1) & ~1, P.bmax + 1); }

size_t f0_workspace_bytes(int B, int64_t n, double fs, double ts, double floor_hz) {
  F0Params P = f0_params(n, fs, ts, floor_hz, 800.0);
  if (P.nf < 1) return 4096;
  const size_t nf = (size_t)B * P.nf;
  return nf * F0_MAXC * (8 + 8 + 4 + 4 + 4) + nf * (4 + 8) + nf * (size_t)f0_rw(P) * 8 + (size_t)B * F0_GP * 3 * 8 +
         9 * 4096;
}

// The context's per-parameter-set tables: [Hann window: nw][its normalised autocorrelation wR: bmax + 1][pad to even]
// [quarter twiddles W_nfft^m = (cos, -sin)(2 pi m / nfft), m < nfft / 4, as (re, im) pairs]
size_t f0_table_doubles(double fs, double floor_hz) {
  const F0Params P = f0_params(1 << 30, fs, 0.01, floor_hz, 800.0);
  return (size_t)((P.nw + P.bmax + 2) & ~1) + (size_t)P.nfft / 2;
}

int f0_tables(double fs, double floor_hz, double* out) {
  const F0Params P = f0_params(1 << 30, fs, 0.01, floor_hz, 800.0);
  SVC_REQUIRE(P.nw >= 4 && P.nw <= 2048, "f0: window of %d samples (pitch floor %g Hz at %g Hz)", P.nw, floor_hz, fs);
  const int nw = P.nw;
  double* w = out;
  for (int i = 0; i < nw; ++i) w[i] = 0.5 - 0.5 * cos((double)(i + 1) * 2.0 * M_PI / (nw + 1));
  double r0 = 0;
  for (int j = 0; j < nw; ++j) r0 = fma(w[j], w[j], r0);
  double* wr = out + nw;
  for (int lag = 0; lag <= P.bmax; ++lag) {
    double sacc = 0;
    for (int j = 0; j + lag < nw; ++j) sacc = fma(w[j], w[j + lag], sacc);
    wr[lag] = sacc / r0;
  }
  double* tq = out + ((nw + P.bmax + 2) & ~1);
  for (int m = 0; m < P.nfft / 4; ++m) {
    const double a = 2.0 * M_PI * (double)m / (double)P.nfft;
    tq[2 * m] = cos(a);
    tq[2 * m + 1] = -sin(a);
  }
  return SVC_OK;
}

template <int N>
static int launch_f0_frames(const float* wav, int B, int64_t n, const F0Params& P, const double* tab,
                            const double* gpart, const F0Out& o, const F0Utt* utt, hipStream_t s) {
  const size_t lds = (size_t)24 * N;
  if (int st = ensure_dyn_lds((const void*)f0_frame_kernel<N>, (int)lds)) return st;
  hipLaunchKernelGGL(f0_frame_kernel<N>, dim3(P.nf, B), dim3(F0_NT), lds, s, wav, n, P, tab, gpart, o, utt);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// n_b (host, [B], optional): ragged batches, utterance b has n_b[b] <= n samples and T_b[b] <= T mel frames; its F0
// is computed on its own samples exactly as a clip of that length, and written zero past T_b[b]. The per-utterance
// frame grids are staged to the device through `ring`. tab: the device copy of f0_tables(fs, floor_hz).
int f0_praat_ac(const float* wav, int B, int64_t n, double fs, double ts, double floor_hz, double ceiling_hz,
                double voicing, int T, double* f0_out, void* workspace, size_t ws_bytes, const double* tab,
                hipStream_t s, const int64_t* n_b, const int* T_b, StageRing* ring) {
  F0Params P = f0_params(n, fs, ts, floor_hz, ceiling_hz);
  SVC_REQUIRE(P.nf >= 1, "f0: sound (%lld samples) shorter than the 3-period window", (long long)n);
  const int hop = (int)llround(ts * fs);
  // utils/f0.py:156-157: pad = (len(audio)//hop - len(f0) + 1)//2 (python floor division)
  auto pad_of = [&](int64_t nn, int nf) {
    const int64_t num = nn / hop - nf + 1;
    return (int)(num >= 0 ? num / 2 : -((-num + 1) / 2));
  };
  const F0Utt* utt = nullptr;
  if (n_b) {
    std::vector<F0Utt> u((size_t)B);
    for (int b = 0; b < B; ++b) {
      SVC_REQUIRE(n_b[b] >= 1 && n_b[b] <= n && T_b[b] >= 1 && T_b[b] <= T, "f0: utterance %d: %lld samples", b,
                  (long long)n_b[b]);
      const F0Params Pb = f0_params(n_b[b], fs, ts, floor_hz, ceiling_hz);
      SVC_REQUIRE(Pb.nf >= 1, "f0: utterance %d (%lld samples) shorter than the 3-period window", b,
                  (long long)n_b[b]);
      u[b] = F0Utt{n_b[b], Pb.t1, Pb.nf, pad_of(n_b[b], Pb.nf), T_b[b]};
    }
    void* dev = nullptr;
    int st = ring->put(u.data(), u.size() * sizeof(F0Utt), s, &dev);
    if (st) return st;
    utt = (const F0Utt*)dev;
  }
  SVC_REQUIRE(P.nw <= 2048 && P.maxc <= F0_MAXC, "f0: window %d / candidates %d too large", P.nw, P.maxc);
  SVC_REQUIRE(P.nfft == 512 || P.nfft == 1024 || P.nfft == 2048 || P.nfft == 4096,
              "f0: autocorrelation FFT of %d points (window %d samples)", P.nfft, P.nw);
  P.voicing = voicing;
  P.silence = 0.03;
  P.octave_cost = 0.01;
  P.octave_jump = 0.35;
  P.vuv_cost = 0.14;
  SVC_REQUIRE(ws_bytes >= f0_workspace_bytes(B, n, fs, ts, floor_hz), "f0: workspace too small");
  char* w = (char*)workspace;
  auto take = [&](size_t bytes) {
    char* p = w;
    w += (bytes + 255) & ~(size_t)255;
    return p;
  };
  const size_t nf = (size_t)B * P.nf;
  F0Out o;
  o.freq = (double*)take(nf * F0_MAXC * 8);
  o.str = (double*)take(nf * F0_MAXC * 8);
  int* psi = (int*)take(nf * F0_MAXC * 4);
  o.ncand = (int*)take(nf * 4);
  o.inten = (double*)take(nf * 8);
  o.cim = (int*)take(nf * F0_MAXC * 4);
  o.rw = f0_rw(P);
  o.rwin = (double*)take(nf * (size_t)o.rw * 8);
  o.work = (int*)take((1 + nf * (F0_MAXC - 1)) * 4);
  double* gpart = (double*)take((size_t)B * F0_GP * 3 * 8);
  // the frame pass's LDS holds r (2 bmax + 1 doubles) and the peak lists (3 x (iend + 1) / 2 + 6 words) in the FFT's
  // 2 * nfft / 2 doubles and the quarter twiddle table after it (nfft / 2 doubles, dead after the inverse FFT)
  SVC_REQUIRE((2 * P.bmax + 2) + 3 * ((std::min(P.maxlag, P.bmax) + 1) / 2 + 2) <= 3 * P.nfft / 2,
              "f0: r and peak lists exceed the FFT buffer");
  hipLaunchKernelGGL(f0_global_kernel, dim3(F0_GP, B), dim3(256), 0, s, wav, n, utt, gpart, o.work);
  SVC_LAUNCH_CHECK();
  int st = P.nfft == 2048   ? launch_f0_frames<1024>(wav, B, n, P, tab, gpart, o, utt, s)
           : P.nfft == 1024 ? launch_f0_frames<512>(wav, B, n, P, tab, gpart, o, utt, s)
           : P.nfft == 512  ? launch_f0_frames<256>(wav, B, n, P, tab, gpart, o, utt, s)
                            : launch_f0_frames<2048>(wav, B, n, P, tab, gpart, o, utt, s);
  if (st) return st;
  const int64_t items = (int64_t)nf * (P.maxc - 1);
  // 8-lane groups: 396 us per 32 x 10 s batch against 488 (4 lanes, 162 VGPRs) and 435 (16 lanes) (r05g)
  hipLaunchKernelGGL(f0_brent_kernel<F0_G>, dim3((unsigned)cdiv64(items, F0_NT / F0_G)), dim3(F0_NT), 0, s, P, o);
  SVC_LAUNCH_CHECK();
  const int pad = pad_of(n, P.nf);
  const int ps_lds = (size_t)P.nf * F0_MAXC <= 32768 ? 1 : 0;  // 10 s: 934 frames -> 15 KB
  hipLaunchKernelGGL(f0_path_kernel, dim3(B), dim3(16 * F0_MAXC), ps_lds ? (size_t)P.nf * F0_MAXC : 0, s, P, o, psi, T,
                     pad, f0_out, ps_lds, utt);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
