// Praat autocorrelation pitch (parselmouth Sound.to_pitch_ac, utils/f0.py:120-161) on gfx950.
//
// Restates Praat's Sound_to_Pitch (AC, Hanning window, 3 periods) + Pitch_pathFinder, the same
// algorithm as oracle/praat_ac.py, in float64:
//   1. per utterance: global mean and peak |x - mean|
//   2. per frame (one workgroup): local mean over one longest period each side, windowed frame,
//      local peak, normalised autocorrelation r[lag] = ac[lag] / (ac[0] * wR[lag]) for lags
//      0..nsamp_window/2 (direct sums in f64 == Praat's zero-padded FFT autocorrelation), peak
//      candidates with parabolic frequency + sinc(30) strength, then per-candidate Brent refinement
//      of the sinc(70) interpolated maximum (one lane per candidate)
//   3. per utterance: Viterbi path over candidates (voiced/unvoiced and octave-jump costs), then the
//      chosen frequencies are written zero-padded to the mel length (utils/f0.py:156-157).
#include <math.h>

#include <algorithm>
#include <vector>

#include "common.h"

namespace svc {

constexpr int F0_MAXC = 16;  // >= max candidates (15 for the parselmouth defaults)
constexpr int F0_LB = 9;     // autocorrelation lags per thread (register window)
constexpr int F0_SEG = 4;    // autocorrelation sample segments (partial sums per lag)

struct F0Params {
  int nsp, hnsp, nw, hnw, maxlag, nf, bmax, maxc;
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
  return P;
}

// ---------------------------------------------------------------------------- NUM helpers (1-based y)
__device__ double sinc_interp(const double* y, int n, double x, int depth) {
  const int midleft = (int)floor(x), midright = midleft + 1;
  if (x > n) return y[n - 1];
  if (x < 1) return y[0];
  if (x == (double)midleft) return y[midleft - 1];
  if (depth > midright - 1) depth = midright - 1;
  if (depth > n - midleft) depth = n - midleft;
  if (depth <= 0) return y[(int)floor(x + 0.5) - 1];
  if (depth == 1) return y[midleft - 1] + (x - midleft) * (y[midright - 1] - y[midleft - 1]);
  if (depth == 2) {
    double yl = y[midleft - 1], yr = y[midright - 1];
    double dyl = 0.5 * (yr - y[midleft - 2]), dyr = 0.5 * (y[midright] - yl);
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
    result += y[ix - 1] * d;
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
    result += y[ix - 1] * d;
    a += M_PI;
    double h = cosaa * cosdaa - sinaa * sindaa;
    sinaa = cosaa * sindaa + sinaa * cosdaa;
    cosaa = h;
    halfsina = -halfsina;
  }
  return result;
}

// sinc_interp evaluated by a whole wave (x and depth wave-uniform; every lane returns the same value): the 2 * depth
// terms are spread over the lanes, each lane computing its terms' angles directly (cos(aa + q * daa)) instead of by
// the serial rotation recurrence, then a wave sum. Equal to sinc_interp up to rounding (~1e-16 relative).
__device__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ double sinc_interp_wave(const double* y, int n, double x, int depth, int lane) {
  const int midleft = (int)floor(x), midright = midleft + 1;
  if (x > n) return y[n - 1];
  if (x < 1) return y[0];
  if (x == (double)midleft) return y[midleft - 1];
  if (depth > midright - 1) depth = midright - 1;
  if (depth > n - midleft) depth = n - midleft;
  if (depth <= 2) return sinc_interp(y, n, x, depth);
  const int left = midright - depth, right = midleft + depth;
  double part = 0.0;
  {  // left terms ix = midleft - q, q < depth
    const double a0 = M_PI * (x - midleft);
    const double hs = 0.5 * sin(a0);
    const double aa = a0 / (x - left + 1.0), daa = M_PI / (x - left + 1.0);
    for (int q = lane; q < depth; q += 64) {
      const double a = a0 + q * M_PI;
      const double d = ((q & 1) ? -hs : hs) / a * (1.0 + cos(aa + q * daa));
      part += y[midleft - q - 1] * d;
    }
  }
  {  // right terms ix = midright + q
    const double a0 = M_PI * (midright - x);
    const double hs = 0.5 * sin(a0);
    const double aa = a0 / (right - x + 1.0), daa = M_PI / (right - x + 1.0);
    for (int q = lane; q < depth; q += 64) {
      const double a = a0 + q * M_PI;
      const double d = ((q & 1) ? -hs : hs) / a * (1.0 + cos(aa + q * daa));
      part += y[midright + q - 1] * d;
    }
  }
  return wave_sum(part);
}

// NUMminimize_brent on f(x) = -sinc(y, x, depth) over [a, b]; returns x, *fx = f(x). SINC is sinc_interp (one lane)
// or sinc_interp_wave (a whole wave, uniform control flow).
template <typename SINC>
__device__ double brent_neg_sinc(SINC sinc, const double* y, int n, int depth, double a, double b, double tol,
                                 double* fxo) {
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
  *fxo = fx;
  return x;
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
__global__ void f0_global_kernel(const float* __restrict__ wav, int64_t stride, const F0Utt* __restrict__ utt,
                                 double* __restrict__ gpeak) {
  const float* x = wav + (int64_t)blockIdx.x * stride;
  const int64_t n = utt ? utt[blockIdx.x].n : stride;
  __shared__ double red[16];
  double s = 0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) s += (double)x[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  double tot = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += red[w];
  const double mean = tot / (double)n;
  __syncthreads();
  double m = 0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) m = fmax(m, fabs((double)x[i] - mean));
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) r = fmax(r, red[w]);
    gpeak[blockIdx.x] = r;
  }
}

// Hanning window (Praat: 0.5 - 0.5 cos(2 pi i / (nw+1)), i = 1..nw) and its normalised autocorrelation
// Hann window and its normalised autocorrelation winR[lag] = sum_j w[j] w[j + lag] / sum_j w[j]^2, one lag per
// thread over F0_WIN_WG-thread workgroups (each recomputes the window in LDS); serial sums as the frame kernel's lags
constexpr int F0_WIN_WG = 64;
__global__ __launch_bounds__(F0_WIN_WG) void f0_window_kernel(int nw, int bmax, double* __restrict__ win,
                                                              double* __restrict__ winR) {
  __shared__ double w[2048];
  __shared__ double r0;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) {
    double v = 0.5 - 0.5 * cos((double)(i + 1) * 2.0 * M_PI / (nw + 1));
    w[i] = v;
    if (blockIdx.x == 0) win[i] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0;
    for (int j = 0; j < nw; ++j) s += w[j] * w[j];
    r0 = s;
  }
  __syncthreads();
  const int lag = blockIdx.x * blockDim.x + threadIdx.x;
  if (lag <= bmax) {
    double s = 0;
    for (int j = 0; j + lag < nw; ++j) s += w[j] * w[j + lag];
    winR[lag] = s / r0;
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

struct F0Out {
  double* freq;   // [B*nf][F0_MAXC]
  double* str;    // [B*nf][F0_MAXC]
  int* ncand;     // [B*nf]
  double* inten;  // [B*nf]
};

__global__ __launch_bounds__(256) void f0_frame_kernel(const float* __restrict__ wav, int64_t n, F0Params P,
                                                       const double* __restrict__ win, const double* __restrict__ winR,
                                                       const double* __restrict__ gpeak, F0Out o,
                                                       const F0Utt* __restrict__ utt) {
  extern __shared__ double sm[];
  double* frame = sm;                   // [nw + bmax + 2 F0_LB], zero past nw
  double* red = frame + P.nw + P.bmax + 2 * F0_LB;  // [8]
  double* r = red + 8;                  // [2*bmax+1], lag L at r[L + bmax]
  double* pkf = r + 2 * P.bmax + 1;     // [bmax + 1] first pass: peak frequency at lag i (0 = not a candidate peak)
  double* pks = pkf + P.bmax + 1;       // [bmax + 1] ... and its sinc(30) strength
  double* part = r;                     // [F0_SEG - 1][bmax + 1] autocorrelation partial sums (before r is written)
  __shared__ double cf[F0_MAXC], cs[F0_MAXC];
  __shared__ int cim[F0_MAXC];
  __shared__ int ncs;
  const int fi = blockIdx.x, b = blockIdx.y;
  if (utt && fi >= utt[b].nf) return;  // past this utterance's frames (block-uniform, before any barrier)
  const float* x = wav + (int64_t)b * n;
  const double t = (utt ? utt[b].t1 : P.t1) + fi * P.ts;
  const int left = (int)floor((t - P.x1) / P.dx) + 1;  // 1-based
  const int right = left + 1;
  // local mean: 1-based samples [right - nsp, left + nsp]
  double s = 0;
  for (int i = right - P.nsp + threadIdx.x; i <= left + P.nsp; i += blockDim.x) s += (double)x[i - 1];
  const double lmean = block_sum(s, red) / (2.0 * P.nsp);
  const int start = right - P.hnw;  // 1-based
  for (int j = threadIdx.x; j < P.nw; j += blockDim.x) frame[j] = ((double)x[start - 1 + j] - lmean) * win[j];
  for (int j = P.nw + threadIdx.x; j < P.nw + P.bmax + 2 * F0_LB; j += blockDim.x) frame[j] = 0.0;
  __syncthreads();
  int s0 = P.hnw + 1 - P.hnsp, s1 = P.hnw + P.hnsp;
  if (s0 < 1) s0 = 1;
  if (s1 > P.nw) s1 = P.nw;
  double lp = 0;
  for (int j = s0 - 1 + threadIdx.x; j < s1; j += blockDim.x) lp = fmax(lp, fabs(frame[j]));
  const double local_peak = block_max(lp, red);
  const int gf = b * P.nf + fi;
  if (threadIdx.x == 0) {
    const double gp = gpeak[b];
    o.inten[gf] = local_peak > gp ? 1.0 : local_peak / gp;
  }
  if (local_peak == 0.0) {
    if (threadIdx.x == 0) {
      o.ncand[gf] = 1;
      o.freq[(int64_t)gf * F0_MAXC] = 0.0;
      o.str[(int64_t)gf * F0_MAXC] = 0.0;
    }
    return;
  }
  // autocorrelation for lags 0..bmax (the zero padding to nfft >= 1.5 nw means no circular wrap): thread (g, sg)
  // sums lags [F0_LB g, F0_LB (g + 1)) over samples j of segment sg, with the F0_LB frame values x[j + lag] in a
  // sliding register window (one broadcast and one lane read per F0_LB fmas; zeros past nw stand in for j + lag >= nw)
  {
    const int ng = (P.bmax + F0_LB) / F0_LB;  // lag groups
    const int nseg = min(F0_SEG, (int)blockDim.x / ng);
    const int seg = (P.nw + nseg - 1) / nseg;
    const int g = threadIdx.x % ng, sg = threadIdx.x / ng;
    double acc[F0_LB];
#pragma unroll
    for (int q = 0; q < F0_LB; ++q) acc[q] = 0.0;
    if (sg < nseg) {
      const int L0 = g * F0_LB, j0 = sg * seg, j1 = min(j0 + seg, P.nw);
      double wv[F0_LB];
#pragma unroll
      for (int q = 0; q < F0_LB; ++q) wv[q] = frame[j0 + L0 + q];
      int j = j0;
      for (; j + F0_LB <= j1; j += F0_LB) {
        double nv[F0_LB];
#pragma unroll
        for (int q = 0; q < F0_LB; ++q) nv[q] = frame[j + L0 + F0_LB + q];
#pragma unroll
        for (int u = 0; u < F0_LB; ++u) {
          const double fj = frame[j + u];
#pragma unroll
          for (int q = 0; q < F0_LB; ++q) acc[q] = fma(fj, u + q < F0_LB ? wv[u + q] : nv[u + q - F0_LB], acc[q]);
        }
#pragma unroll
        for (int q = 0; q < F0_LB; ++q) wv[q] = nv[q];
      }
      for (; j < j1; ++j) {
        const double fj = frame[j];
#pragma unroll
        for (int q = 0; q < F0_LB; ++q) acc[q] = fma(fj, frame[j + L0 + q], acc[q]);
      }
      if (sg > 0) {
#pragma unroll
        for (int q = 0; q < F0_LB; ++q)
          if (L0 + q <= P.bmax) part[(sg - 1) * (P.bmax + 1) + L0 + q] = acc[q];
      }
    }
    __syncthreads();
    if (sg == 0) {
#pragma unroll
      for (int q = 0; q < F0_LB; ++q) {
        const int lag = g * F0_LB + q;
        if (lag <= P.bmax)
          for (int t = 1; t < nseg; ++t) acc[q] += part[(t - 1) * (P.bmax + 1) + lag];
      }
    }
    __syncthreads();  // partial sums read before r (which they alias) is written
    if (sg == 0) {
#pragma unroll
      for (int q = 0; q < F0_LB; ++q) {
        const int lag = g * F0_LB + q;
        if (lag <= P.bmax) r[P.bmax + lag] = acc[q];
      }
    }
  }
  __syncthreads();
  const double ac0 = r[P.bmax];
  __syncthreads();
  for (int lag = 1 + threadIdx.x; lag <= P.bmax; lag += blockDim.x) {
    double v = r[P.bmax + lag] / (ac0 * winR[lag]);
    r[P.bmax + lag] = v;
    r[P.bmax - lag] = v;
  }
  if (threadIdx.x == 0) r[P.bmax] = 1.0;
  __syncthreads();
  const int rn = 2 * P.bmax + 1;
  const int iend = P.maxlag < P.bmax ? P.maxlag : P.bmax;
  // first pass, in parallel over lags: local maxima above half the voicing threshold and their sinc(30) strengths
  for (int i = 2 + threadIdx.x; i < iend; i += blockDim.x) {
    const double ri = r[P.bmax + i], rm = r[P.bmax + i - 1], rp = r[P.bmax + i + 1];
    double freq = 0.0, strength = 0.0;
    if (ri > 0.5 * P.voicing && ri > rm && ri >= rp) {
      const double dr = 0.5 * (rp - rm), d2r = 2.0 * ri - rm - rp;
      freq = 1.0 / P.dx / (i + dr / d2r);
      strength = sinc_interp(r, rn, 1.0 / P.dx / freq + P.bmax + 1, 30);
      if (strength > 1.0) strength = 1.0 / strength;
    }
    pkf[i] = freq;
    pks[i] = strength;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // ... then the candidate list in lag order (Praat's replacement rule is sequential)
    int nc = 1;
    cf[0] = 0.0;
    cs[0] = 0.0;
    cim[0] = 0;
    for (int i = 2; i < iend; ++i) {
      if (pkf[i] != 0.0) {
        const double freq = pkf[i];
        const double strength = pks[i];
        int place = 0;
        if (nc < P.maxc) {
          place = nc++;
        } else {
          double weakest = 2.0;
          for (int iw = 1; iw < P.maxc; ++iw) {
            double ls = cs[iw] - P.octave_cost * log2(P.floor_hz / cf[iw]);
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
          cim[place] = i;
        }
      }
    }
    ncs = nc;
  }
  __syncthreads();
  const int nc = ncs;
  const int k = threadIdx.x;
  // second pass: sinc(70) maximum by Brent, one WAVE per candidate (the sinc sums spread over its lanes)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int kc = 1 + wave; kc < nc; kc += (int)(blockDim.x >> 6)) {
    const int ixmid = cim[kc] + P.bmax + 1;
    double xmid, ymid;
    if (ixmid <= 1) {
      xmid = 1.0;
      ymid = r[0];
    } else if (ixmid >= rn) {
      xmid = rn;
      ymid = r[rn - 1];
    } else {
      double fx;
      auto sw = [lane](const double* y, int n, double x, int depth) { return sinc_interp_wave(y, n, x, depth, lane); };
      xmid = brent_neg_sinc(sw, r, rn, 70, ixmid - 1, ixmid + 1, 1e-10, &fx);
      ymid = -fx;
    }
    xmid -= P.bmax + 1;
    double freq = 1.0 / P.dx / xmid;
    if (ymid > 1.0) ymid = 1.0 / ymid;
    if (lane == 0) {
      cf[kc] = freq;
      cs[kc] = ymid;
    }
  }
  __syncthreads();
  if (k < nc) {
    o.freq[(int64_t)gf * F0_MAXC + k] = cf[k];
    o.str[(int64_t)gf * F0_MAXC + k] = cs[k];
  }
  if (k == 0) o.ncand[gf] = nc;
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

size_t f0_workspace_bytes(int B, int64_t n, double fs, double ts, double floor_hz) {
  F0Params P = f0_params(n, fs, ts, floor_hz, 800.0);
  if (P.nf < 1) return 4096;
  const size_t nf = (size_t)B * P.nf;
  return nf * F0_MAXC * (8 + 8 + 4) + nf * (4 + 8) + (size_t)B * 8 + (size_t)(P.nw + P.bmax + 2) * 8 + 8 * 4096;
}

// n_b (host, [B], optional): ragged batches, utterance b has n_b[b] <= n samples and T_b[b] <= T mel frames; its F0
// is computed on its own samples exactly as a clip of that length, and written zero past T_b[b]. The per-utterance
// frame grids are staged to the device through `ring`.
int f0_praat_ac(const float* wav, int B, int64_t n, double fs, double ts, double floor_hz, double ceiling_hz,
                double voicing, int T, double* f0_out, void* workspace, size_t ws_bytes, hipStream_t s,
                const int64_t* n_b, const int* T_b, StageRing* ring) {
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
  double* gpeak = (double*)take((size_t)B * 8);
  double* win = (double*)take((size_t)P.nw * 8);
  double* winR = (double*)take((size_t)(P.bmax + 1) * 8);
  hipLaunchKernelGGL(f0_global_kernel, dim3(B), dim3(1024), 0, s, wav, n, utt, gpeak);
  SVC_LAUNCH_CHECK();
  hipLaunchKernelGGL(f0_window_kernel, dim3(cdiv(P.bmax + 1, F0_WIN_WG)), dim3(F0_WIN_WG), 0, s, P.nw, P.bmax, win, winR);
  SVC_LAUNCH_CHECK();
  // every lag group needs a thread of the 256-thread workgroup (nw <= 2048: at most 114 groups, >= 2 segments); the
  // F0_SEG - 1 partial-sum rows fit the r / pkf / pks region (4 bmax + 3 doubles)
  SVC_REQUIRE((P.bmax + F0_LB) / F0_LB <= 256, "f0: %d lags do not fit the autocorrelation blocking", P.bmax + 1);
  const size_t lds = (size_t)(P.nw + P.bmax + 2 * F0_LB + 8 + 2 * P.bmax + 1 + 2 * (P.bmax + 1)) * sizeof(double);
  hipLaunchKernelGGL(f0_frame_kernel, dim3(P.nf, B), dim3(256), lds, s, wav, n, P, win, winR, gpeak, o, utt);
  SVC_LAUNCH_CHECK();
  const int pad = pad_of(n, P.nf);
  const int ps_lds = (size_t)P.nf * F0_MAXC <= 32768 ? 1 : 0;  // 10 s: 934 frames -> 15 KB
  hipLaunchKernelGGL(f0_path_kernel, dim3(B), dim3(16 * F0_MAXC), ps_lds ? (size_t)P.nf * F0_MAXC : 0, s, P, o, psi, T,
                     pad, f0_out, ps_lds, utt);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
