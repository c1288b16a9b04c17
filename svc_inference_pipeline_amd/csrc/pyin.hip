// pYIN F0 (utils/f0.py:95-117 get_f0_features_using_pyin -> librosa.pyin with its defaults; unvoiced frames 0),
// SURVEY.md §8(f) F4. infer.py never selects it (utils/acoustic_feature_extraction.py hard-wires Praat); it is the
// config-selectable alternative, built as two launches:
//   1. pyin_frame_kernel, one workgroup per (utterance, frame): the centred frame (frame_length / 2 zeros before the
//      clip) in LDS as f64; acf(tau) = sum_{j=1..W} x[j] x[j + tau] and the window energy E(tau) = sum x[j + tau]^2
//      for tau = 0..max_period, register-tiled 8 lags per thread over a sliding 16-sample window (the j range split
//      across threads, partials summed in a fixed order); librosa's 1e-6 zeroing; d(tau) = E(0) + E(tau) - 2 acf(tau);
//      the cumulative mean normalised difference (CMND) rows min_period..max_period; parabolic shifts; troughs and
//      their probabilities (beta threshold prior x Boltzmann trough prior through a [trough][threshold] count table,
//      the global minimum's share below every trough); the observation row log(p + tiny) over the n_bins voiced
//      states and the unvoiced states' log((1 - voiced) / n_bins + tiny);
//   2. pyin_viterbi_kernel, one workgroup per utterance, thread per state: Viterbi over the 2 n_bins-state HMM in the
//      log domain as librosa.sequence.viterbi does. Every state is a source: in the band of the local transition
//      (2 x (2 half_width + 1) sources) from the log table, outside it log(0 + tiny) applied to the block's prefix /
//      suffix maximum (Hillis-Steele scans in LDS); argmax ties go to the lowest source, back-pointers as u16 in HBM,
//      backtracking by one thread, f0 = the decoded bin's frequency (0 when unvoiced).
// Restated from librosa 0.10's published algorithm (oracle/pyin.py): librosa is absent here, so PARITY IS UNPINNED;
// tests/test_f0.py holds the kernel to the oracle and both to known-answer tones.
#include <math.h>

#include <algorithm>
#include <vector>

#include "common.h"

namespace svc {

constexpr int PY_NT = 256;
constexpr int PY_MAXP = 1024;   // bound of max_period + 8 (LDS rows)
constexpr int PY_MAXTR = 240;   // troughs below threshold 1 (the count table is u16 [240][100])
constexpr int PY_NTH = 100;     // thresholds (librosa n_thresholds)
constexpr int PY_MAXBINS = 512;
constexpr int PY_XS = 2048 + 32;
constexpr double PY_TINY = 2.2250738585072014e-308;

struct PyinArgs {
  const float* wav;  // [B][ld]
  int64_t ld;
  const int64_t* nvalid;  // [B] samples per utterance (device), or NULL (all ld)
  int B, F;               // utterances, output frames per utterance
  int frame_length, win_length, hop, min_period, max_period;
  int n_bins, half_width, tau_groups, j_parts;
  double sr, fmin, bins_per_octave;
  const double* beta_probs;  // [100]
  const double* log_band;    // [2 (switch: same block, other block)][n_bins source][2 half_width + 1] log(trans + tiny)
  const double* freqs;       // [n_bins]
  double no_trough_prob;
  double* logobs;     // [B][F][n_bins] log(observation + tiny) of the voiced states
  double* logunv;     // [B][F] the unvoiced states'
  uint16_t* ptr;      // [B][F][2 n_bins]
  double* f0;         // [B][F]
};

__device__ __forceinline__ double py_boltzmann(int k, int n) {
  // scipy.stats.boltzmann.pmf(k, 2, N=n)
  if (k < 0 || k >= n) return 0.0;
  return (1.0 - exp(-2.0)) * exp(-2.0 * k) / (1.0 - exp(-2.0 * n));
}
// np.linspace(0, 1, 101)[i]: i * 0.01, the endpoint exactly 1
__device__ __forceinline__ double py_thr(int i) { return i == PY_NTH ? 1.0 : i * 0.01; }

__global__ __launch_bounds__(PY_NT) void pyin_frame_kernel(PyinArgs a) {
  // raw: xs [PY_XS] | pac [2048] | pe [2048] (f64); after the lag sums, the u16 count table [PY_MAXTR][100]
  __shared__ double raw[PY_XS + 4096];
  __shared__ double yin[PY_MAXP];  // d(tau), then the CMND rows (index tau - min_period)
  __shared__ double sh[PY_MAXP];   // parabolic shifts
  __shared__ double en[PY_MAXP];   // E(tau), then the cumulative mean, then the observation row
  __shared__ double pr[PY_MAXP / 2 + 2];
  __shared__ int tr[PY_MAXP / 2 + 2];   // trough rows
  __shared__ int fth[PY_MAXP / 2 + 2];  // first threshold index each trough is below (100: none)
  __shared__ int ntr_s, nlow_s;
  double* xs = raw;
  double* pac = raw + PY_XS;
  double* pe = pac + 2048;
  uint16_t* cnt = reinterpret_cast<uint16_t*>(raw);
  const int b = blockIdx.y, t = blockIdx.x, tid = threadIdx.x;
  const int FL = a.frame_length, W = a.win_length, maxp = a.max_period, minp = a.min_period;
  const int nbn = a.n_bins;
  const int64_t nb = a.nvalid ? a.nvalid[b] : a.ld;
  const int64_t o = (int64_t)b * a.F + t;
  double* lrow = a.logobs + o * nbn;
  if (t >= 1 + nb / a.hop) return;  // past this utterance's frames (the Viterbi stops before them)
  const float* w = a.wav + (int64_t)b * a.ld;
  for (int j = tid; j < PY_XS; j += PY_NT) {
    const int64_t i = (int64_t)t * a.hop + j - FL / 2;
    xs[j] = (j < FL && i >= 0 && i < nb) ? (double)w[i] : 0.0;
  }
  __syncthreads();
  // lag sums: thread (g, part) covers lags 8g..8g+7 over its j chunk
  const int G = a.tau_groups, P = a.j_parts;
  const int nblk = (W + 7) / 8, per = (nblk + P - 1) / P;
  if (tid < G * P) {
    const int g = tid % G, part = tid / G, tau0 = 8 * g;
    const int j0 = 1 + part * per * 8, j1 = min(W + 1, j0 + per * 8);
    double ac[8], e[8], win[16];
#pragma unroll
    for (int r = 0; r < 8; ++r) ac[r] = e[r] = 0.0;
    int j = j0;
    if (j0 < j1) {
#pragma unroll
      for (int r = 0; r < 8; ++r) win[r] = xs[j + tau0 + r];
      for (; j + 8 <= j1; j += 8) {
#pragma unroll
        for (int r = 0; r < 8; ++r) win[8 + r] = xs[j + 8 + tau0 + r];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const double xj = xs[j + q];
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            ac[r] = fma(xj, win[q + r], ac[r]);
            e[r] = fma(win[q + r], win[q + r], e[r]);
          }
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) win[r] = win[8 + r];
      }
      for (; j < j1; ++j) {
        const double xj = xs[j];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const double v = xs[j + tau0 + r];
          ac[r] = fma(xj, v, ac[r]);
          e[r] = fma(v, v, e[r]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      pac[part * G * 8 + tau0 + r] = ac[r];
      pe[part * G * 8 + tau0 + r] = e[r];
    }
  }
  __syncthreads();
  for (int tau = tid; tau <= maxp; tau += PY_NT) {
    double ac = 0.0, e = 0.0;
    for (int part = 0; part < P; ++part) {
      ac += pac[part * G * 8 + tau];
      e += pe[part * G * 8 + tau];
    }
    yin[tau] = fabs(ac) < 1e-6 ? 0.0 : ac;  // acf, for now
    en[tau] = fabs(e) < 1e-6 ? 0.0 : e;
  }
  __syncthreads();
  if (tid == 0) {
    // d(tau) and the cumulative mean over tau = 1..max_period (sequential: numpy's cumsum order)
    const double e0 = en[0];
    double cum = 0.0;
    for (int tau = 1; tau <= maxp; ++tau) {
      const double d = e0 + en[tau] - 2.0 * yin[tau];
      cum += d;
      en[tau] = cum / tau;
      yin[tau] = d;
    }
  }
  __syncthreads();
  const int np_ = maxp - minp + 1;
  for (int i = tid; i < np_; i += PY_NT) sh[i] = yin[minp + i] / (en[minp + i] + PY_TINY);
  __syncthreads();
  for (int i = tid; i < np_; i += PY_NT) yin[i] = sh[i];  // CMND rows 0..np_-1
  __syncthreads();
  for (int i = tid; i < np_; i += PY_NT) {
    double s = 0.0;
    if (i > 0 && i < np_ - 1) {
      const double pa = yin[i + 1] + yin[i - 1] - 2.0 * yin[i];
      const double pb = (yin[i + 1] - yin[i - 1]) / 2.0;
      s = fabs(pb) >= fabs(pa) ? 0.0 : -pb / pa;
    }
    sh[i] = s;
  }
  for (int s = tid; s < nbn; s += PY_NT) en[s] = 0.0;  // observation row
  if (tid == 0) {
    // troughs: x[i] < x[i-1] and x[i] <= x[i+1] (edge-padded); the first row by x[0] < x[1]
    int n = 0;
    for (int i = 0; i < np_; ++i) {
      bool is;
      if (i == 0) {
        is = yin[0] < yin[1];
      } else {
        const double r = i + 1 < np_ ? yin[i + 1] : yin[i];
        is = yin[i] < yin[i - 1] && yin[i] <= r;
      }
      if (is) tr[n++] = i;
    }
    ntr_s = n;
  }
  __syncthreads();
  const int ntr = ntr_s;
  if (ntr == 0) {
    // no trough: every voiced observation 0, voiced probability 0
    for (int s = tid; s < nbn; s += PY_NT) lrow[s] = log(PY_TINY);
    if (tid == 0) a.logunv[o] = log(1.0 / nbn + PY_TINY);
    return;
  }
  for (int k = tid; k < ntr; k += PY_NT) {
    const double h = yin[tr[k]];
    int f = PY_NTH;
    for (int th = PY_NTH - 1; th >= 0; --th)
      if (h < py_thr(th + 1)) f = th;
    fth[k] = f;
  }
  __syncthreads();
  if (tid == 0) {
    int m = 0;
    for (int k = 0; k < ntr; ++k) m += fth[k] < PY_NTH;
    nlow_s = m;
  }
  __syncthreads();
  // count table cnt[q][th] = #{below-1 troughs q' <= q below threshold th + 1}, q over the below-1 troughs in order
  // (the host bounds the trough count by PY_MAXTR)
  const int m = nlow_s;
  if (tid < PY_NTH) {
    int c = 0, q = 0;
    for (int k = 0; k < ntr; ++k) {
      if (fth[k] >= PY_NTH) continue;
      c += fth[k] <= tid;
      cnt[q * PY_NTH + tid] = (uint16_t)c;
      ++q;
    }
  }
  __syncthreads();
  // probability of trough k (thread per trough): sum_th boltzmann(pos, count) beta[th] over the thresholds it is below
  for (int k = tid; k < ntr; k += PY_NT) {
    double p = 0.0;
    if (fth[k] < PY_NTH) {
      int q = 0;
      for (int k2 = 0; k2 < k; ++k2) q += fth[k2] < PY_NTH;
      for (int th = fth[k]; th < PY_NTH; ++th) {
        const int pos = cnt[q * PY_NTH + th] - 1, count = cnt[(m - 1) * PY_NTH + th];
        p += py_boltzmann(pos, count) * a.beta_probs[th];
      }
    }
    pr[k] = p;
  }
  __syncthreads();
  if (tid == 0) {
    int g = 0;
    for (int k = 1; k < ntr; ++k)
      if (yin[tr[k]] < yin[tr[g]]) g = k;
    const double hg = yin[tr[g]];
    int below_min = 0;
    for (int th = 0; th < PY_NTH; ++th) below_min += !(hg < py_thr(th + 1));
    double s = 0.0;
    for (int th = 0; th < below_min; ++th) s += a.beta_probs[th];
    pr[g] += a.no_trough_prob * s;
    // observations in increasing period (a later trough in the same bin overwrites, as numpy's assignment does);
    // bin n_bins is the unvoiced block's first row, which librosa then overwrites
    for (int k = 0; k < ntr; ++k) {
      const double p = pr[k];
      if (p == 0.0) continue;
      const int i = tr[k];
      const double period = (double)(minp + i) + sh[i];
      const double f0c = a.sr / period;
      double bi = rint(a.bins_per_octave * log2(f0c / a.fmin));
      bi = bi < 0.0 ? 0.0 : (bi > nbn ? (double)nbn : bi);
      const int bin = (int)bi;
      if (bin < nbn) en[bin] = p;
    }
    double v = 0.0;
    for (int s2 = 0; s2 < nbn; ++s2) v += en[s2];
    v = v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);
    a.logunv[o] = log((1.0 - v) / nbn + PY_TINY);
  }
  __syncthreads();
  for (int s = tid; s < nbn; s += PY_NT) lrow[s] = log(en[s] + PY_TINY);
}

constexpr int PY_VT = 1024;

__global__ __launch_bounds__(PY_VT) void pyin_viterbi_kernel(PyinArgs a) {
  __shared__ double val[2 * PY_MAXBINS];
  __shared__ double pv[2][2 * PY_MAXBINS], qv[2][2 * PY_MAXBINS];  // prefix / suffix max (double-buffered)
  __shared__ int pi[2][2 * PY_MAXBINS], qi[2][2 * PY_MAXBINS];
  const int nbn = a.n_bins, S = 2 * nbn, hw = a.half_width, BW = 2 * hw + 1;
  const int b = blockIdx.x, d = threadIdx.x;
  const int64_t nb = a.nvalid ? a.nvalid[b] : a.ld;
  const int Fb = (int)min((int64_t)a.F, 1 + nb / a.hop);
  const double LOG_TINY = log(PY_TINY);
  const bool act = d < S;
  const int vd = d >= nbn, dd = d - vd * nbn;  // dest block and bin
  const double* lobs = a.logobs + (int64_t)b * a.F * nbn;
  const double* lunv = a.logunv + (int64_t)b * a.F;
  // t = 0: log observation + log(p_init): 1 / n_bins on the unvoiced states, 0 on the voiced
  if (act) val[d] = (vd ? lunv[0] : lobs[dd]) + (vd ? log(1.0 / nbn + PY_TINY) : LOG_TINY);
  __syncthreads();
  uint16_t* ptr = a.ptr + (int64_t)b * a.F * S;
  for (int t = 1; t < Fb; ++t) {
    // prefix (ties: first) and suffix (ties: lowest) maxima of val within each block, Hillis-Steele
    int cur = 0;
    if (act) {
      pv[0][d] = qv[0][d] = val[d];
      pi[0][d] = qi[0][d] = d;
    }
    __syncthreads();
    for (int off = 1; off < nbn; off <<= 1) {
      if (act) {
        double v = pv[cur][d], u = qv[cur][d];
        int iv = pi[cur][d], iu = qi[cur][d];
        if (dd >= off) {  // left element d - off: the current (right) one wins only when strictly greater
          const double lv = pv[cur][d - off];
          if (!(v > lv)) v = lv, iv = pi[cur][d - off];
        }
        if (dd + off < nbn) {  // right element d + off: the current (left) one wins ties
          const double rv = qv[cur][d + off];
          if (!(u >= rv)) u = rv, iu = qi[cur][d + off];
        }
        pv[cur ^ 1][d] = v;
        pi[cur ^ 1][d] = iv;
        qv[cur ^ 1][d] = u;
        qi[cur ^ 1][d] = iu;
      }
      cur ^= 1;
      __syncthreads();
    }
    double nv = 0.0;
    if (act) {
      double best = -INFINITY;
      int bi = 0x7fffffff;
      auto offer = [&](double v, int s) {
        if (v > best || (v == best && s < bi)) best = v, bi = s;
      };
      const int lo = max(0, dd - hw), hi = min(nbn - 1, dd + hw);
      for (int vs = 0; vs < 2; ++vs) {
        const int base = vs * nbn;
        const double* lb = a.log_band + (size_t)(vs == vd ? 0 : 1) * nbn * BW;
        for (int s = lo; s <= hi; ++s) offer(val[base + s] + lb[(size_t)s * BW + (dd - s + hw)], base + s);
        if (lo > 0) offer(pv[cur][base + lo - 1] + LOG_TINY, pi[cur][base + lo - 1]);
        if (hi < nbn - 1) offer(qv[cur][base + hi + 1] + LOG_TINY, qi[cur][base + hi + 1]);
      }
      nv = (vd ? lunv[t] : lobs[(int64_t)t * nbn + dd]) + best;
      ptr[(int64_t)t * S + d] = (uint16_t)bi;
    }
    __syncthreads();
    if (act) val[d] = nv;
    __syncthreads();
  }
  if (d == 0) {
    int st = 0;
    for (int s = 1; s < S; ++s)
      if (val[s] > val[st]) st = s;
    double* f0 = a.f0 + (int64_t)b * a.F;
    for (int t = Fb - 1; t >= 0; --t) {
      f0[t] = st < nbn ? a.freqs[st] : 0.0;
      if (t > 0) st = ptr[(int64_t)t * S + st];
    }
    for (int t = Fb; t < a.F; ++t) f0[t] = 0.0;
  }
}

namespace {
double py_beta_cdf(double x, int aa, int bb) {  // regularised incomplete beta for integer a, b
  const int n = aa + bb - 1;
  double s = 0.0, c = 1.0;  // c = C(n, j)
  for (int j = 0; j < aa; ++j) {
    s += c * pow(x, j) * pow(1.0 - x, n - j);
    c = c * (n - j) / (j + 1);
  }
  return 1.0 - s;
}
double py_triang(int m, int i) {  // scipy.signal.windows.triang(m, sym=True)[i]
  const int half = (m + 1) / 2;
  const int n = i < half ? i + 1 : m - i;
  return m % 2 == 0 ? (2.0 * n - 1.0) / m : 2.0 * n / (m + 1.0);
}

struct PyinPlan {
  int min_period, max_period, n_bins, bps, width, half_width, G, P;
};

int pyin_plan(double sr, double fmin, double fmax, int frame_length, int win_length, int hop, PyinPlan* p) {
  SVC_REQUIRE(sr > 0 && fmin > 0 && fmax > fmin && hop > 0, "pyin: sr %g fmin %g fmax %g hop %d", sr, fmin, fmax, hop);
  SVC_REQUIRE(frame_length > 0 && frame_length <= 2048 && win_length > 0 && win_length < frame_length,
              "pyin: frame_length %d win_length %d", frame_length, win_length);
  p->min_period = std::max((int)floor(sr / fmax), 1);
  p->max_period = std::min((int)ceil(sr / fmin), frame_length - win_length - 1);
  const int np_ = p->max_period - p->min_period + 1;
  // at most (np_ + 1) / 2 + 1 troughs; the count table holds PY_MAXTR of them
  SVC_REQUIRE(np_ >= 3 && p->max_period + 8 <= PY_MAXP && (np_ + 1) / 2 + 1 <= PY_MAXTR,
              "pyin: periods %d..%d unsupported", p->min_period, p->max_period);
  p->bps = 10;  // ceil(1 / resolution), resolution 0.1
  p->n_bins = (int)floor(12 * p->bps * log2(fmax / fmin)) + 1;
  const int max_semitones = (int)nearbyint(35.92 * 12 * hop / sr);  // Python round: half to even
  p->width = max_semitones * p->bps + 1;
  p->half_width = p->width / 2;
  SVC_REQUIRE(p->n_bins <= PY_MAXBINS && p->width <= p->n_bins, "pyin: %d pitch bins, transition width %d",
              p->n_bins, p->width);
  p->G = (p->max_period + 1 + 7) / 8;
  p->P = std::max(1, std::min(PY_NT / p->G, 16));
  return SVC_OK;
}
}  // namespace

size_t pyin_table_doubles(double sr, double fmin, double fmax, int frame_length, int win_length, int hop) {
  PyinPlan p;
  if (pyin_plan(sr, fmin, fmax, frame_length, win_length, hop, &p)) return 0;
  return PY_NTH + 2 * (size_t)p.n_bins * (2 * p.half_width + 1) + p.n_bins;
}

size_t pyin_workspace_bytes(int B, int F, double sr, double fmin, double fmax, int frame_length, int win_length,
                            int hop) {
  PyinPlan p;
  if (pyin_plan(sr, fmin, fmax, frame_length, win_length, hop, &p)) return 0;
  const size_t fr = (size_t)B * F;
  return fr * ((size_t)p.n_bins * 8 + 8 + 2 * (size_t)p.n_bins * 2) + 4 * 256;
}

// host tables (f64, computed as librosa computes them): beta threshold prior [100], log(transition + tiny) over the
// band [2][n_bins][2 hw + 1], the bin frequencies [n_bins]
int pyin_tables(double sr, double fmin, double fmax, int frame_length, int win_length, int hop, double* out) {
  PyinPlan p;
  if (int st = pyin_plan(sr, fmin, fmax, frame_length, win_length, hop, &p)) return st;
  const int nbn = p.n_bins, BW = 2 * p.half_width + 1, width = p.width;
  for (int th = 0; th < PY_NTH; ++th) {
    const double x0 = th * 0.01, x1 = th + 1 == PY_NTH ? 1.0 : (th + 1) * 0.01;  // np.linspace(0, 1, 101)
    out[th] = py_beta_cdf(x1, 2, 18) - py_beta_cdf(x0, 2, 18);
  }
  // transition_local(n_bins, width, 'triangle', wrap=False): row i = the centred window rolled to i and cut to
  // [i - width / 2, i + width / 2], row-normalised; kron with [[1 - p, p], [p, 1 - p]], p = switch_prob 0.01
  double* band = out + PY_NTH;
  std::vector<double> padded(nbn, 0.0), row(nbn);
  const int lpad = (nbn - width) / 2;
  for (int q = 0; q < width; ++q) padded[lpad + q] = py_triang(width, q);
  for (int i = 0; i < nbn; ++i) {
    const int shift = (nbn / 2 + i + 1) % nbn;
    for (int q = 0; q < nbn; ++q) row[(q + shift) % nbn] = padded[q];
    for (int q = std::min(nbn, i + width / 2 + 1); q < nbn; ++q) row[q] = 0.0;
    for (int q = 0; q < std::max(0, i - width / 2); ++q) row[q] = 0.0;
    double sum = 0.0;
    for (int q = 0; q < nbn; ++q) sum += row[q];
    for (int sw = 0; sw < 2; ++sw) {
      const double ps = sw == 0 ? 1.0 - 0.01 : 0.01;
      for (int q = -p.half_width; q <= p.half_width; ++q) {
        const int d = i + q;
        const double v = (d >= 0 && d < nbn) ? ps * (row[d] / sum) : 0.0;
        band[((size_t)sw * nbn + i) * BW + (q + p.half_width)] = log(v + PY_TINY);
      }
    }
  }
  double* freqs = band + 2 * (size_t)nbn * BW;
  for (int k = 0; k < nbn; ++k) freqs[k] = fmin * pow(2.0, (double)k / (12 * p.bps));
  return SVC_OK;
}

// wav f32 [B][ld]; nvalid_dev: per-utterance samples (device) or NULL; nvalid_host the same on the host (frame count
// checks); tables_dev: pyin_tables() on the device, alive until the launches have run; f0 f64 [B][F] out
int f0_pyin(const float* wav, int B, int64_t ld, const int64_t* nvalid_dev, const int64_t* nvalid_host, double sr,
            double fmin, double fmax, int frame_length, int win_length, int hop, int F, double* f0, void* ws,
            size_t ws_bytes, const double* tables_dev, hipStream_t s) {
  PyinPlan p;
  if (int st = pyin_plan(sr, fmin, fmax, frame_length, win_length, hop, &p)) return st;
  SVC_REQUIRE(wav && f0 && ws && tables_dev && B > 0 && ld > 0 && B <= 65535, "pyin: bad args");
  int64_t fmax_frames = 0;
  for (int b = 0; b < B; ++b) {
    const int64_t n = nvalid_host ? nvalid_host[b] : ld;
    SVC_REQUIRE(n > 0 && n <= ld, "pyin: utterance %d has %lld samples (batch length %lld)", b, (long long)n,
                (long long)ld);
    fmax_frames = std::max(fmax_frames, 1 + n / hop);
  }
  SVC_REQUIRE(F >= fmax_frames && F <= (1 << 24), "pyin: %d output frames for %lld", F, (long long)fmax_frames);
  const size_t need = pyin_workspace_bytes(B, F, sr, fmin, fmax, frame_length, win_length, hop);
  SVC_REQUIRE(ws_bytes >= need, "pyin: workspace %zu < %zu", ws_bytes, need);
  PyinArgs a{};
  a.wav = wav;
  a.ld = ld;
  a.nvalid = nvalid_dev;
  a.B = B;
  a.F = F;
  a.frame_length = frame_length;
  a.win_length = win_length;
  a.hop = hop;
  a.min_period = p.min_period;
  a.max_period = p.max_period;
  a.n_bins = p.n_bins;
  a.half_width = p.half_width;
  a.tau_groups = p.G;
  a.j_parts = p.P;
  a.sr = sr;
  a.fmin = fmin;
  a.bins_per_octave = 12.0 * p.bps;
  a.no_trough_prob = 0.01;
  a.beta_probs = tables_dev;
  a.log_band = tables_dev + PY_NTH;
  a.freqs = a.log_band + 2 * (size_t)p.n_bins * (2 * p.half_width + 1);
  const size_t fr = (size_t)B * F;
  char* q = reinterpret_cast<char*>(ws);
  auto take = [&](size_t bytes) {
    char* r = q;
    q += (bytes + 255) & ~(size_t)255;
    return r;
  };
  a.logobs = reinterpret_cast<double*>(take(fr * p.n_bins * 8));
  a.logunv = reinterpret_cast<double*>(take(fr * 8));
  a.ptr = reinterpret_cast<uint16_t*>(take(fr * 2 * p.n_bins * 2));
  a.f0 = f0;
  const int tok = prof_begin("pyin_frame", 0.0, 0.0, s);
  hipLaunchKernelGGL(pyin_frame_kernel, dim3((unsigned)F, (unsigned)B), dim3(PY_NT), 0, s, a);
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  const int tok2 = prof_begin("pyin_viterbi", 0.0, 0.0, s);
  hipLaunchKernelGGL(pyin_viterbi_kernel, dim3((unsigned)B), dim3(PY_VT), 0, s, a);
  prof_end(tok2, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
