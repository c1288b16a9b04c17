"""CPU restatement of librosa.pyin (TEST INFRASTRUCTURE ONLY: the product never imports this module).

The reference's `get_f0_features_using_pyin` (/root/reference/utils/f0.py:95-117) calls
`librosa.pyin(y=audio, fmin=f0_min, fmax=f0_max, sr=fs, win_length=win_length, hop_length=hop_length)` and zeroes the
unvoiced frames. librosa is not installed here and the reference pins no version; its files date from
2023-06, i.e. librosa 0.10.x. This module restates the published algorithm of librosa 0.10 `pyin` (Mauch & Dixon 2014,
"pYIN", as librosa implements it: YIN cumulative mean normalized difference, beta-distributed thresholds with the
Boltzmann trough prior of the official pYIN software, a 2 x n_pitch_bins HMM decoded by Viterbi) with the library's
defaults for every argument the reference leaves unset (frame_length 2048, n_thresholds 100, beta (2, 18),
boltzmann 2, resolution 0.1 semitone, max_transition_rate 35.92 octaves/s, switch_prob 0.01, no_trough_prob 0.01,
center=True with constant padding). PARITY UNPINNED: no librosa output exists in this container or the reference to
check it against; tests/test_f0.py checks it with known-answer tones and silence.
"""
import math

import numpy as np

TINY64 = np.finfo(np.float64).tiny


def frame(y, frame_length, hop_length):
    """librosa.util.frame for 1-D y: [frame_length, n_frames] (frames as columns)."""
    n = 1 + (len(y) - frame_length) // hop_length
    idx = np.arange(frame_length)[:, None] + hop_length * np.arange(n)[None, :]
    return y[idx]


def cumulative_mean_normalized_difference(y_frames, frame_length, win_length, min_period, max_period):
    """librosa.core.pitch._cumulative_mean_normalized_difference: rows min_period..max_period of the CMND."""
    a = np.fft.rfft(y_frames, frame_length, axis=0)
    b = np.fft.rfft(y_frames[win_length:0:-1, :], frame_length, axis=0)
    acf = np.fft.irfft(a * b, frame_length, axis=0)[win_length:, :]
    acf[np.abs(acf) < 1e-6] = 0
    energy = np.cumsum(y_frames ** 2, axis=0)
    energy = energy[win_length:, :] - energy[:-win_length, :]
    energy[np.abs(energy) < 1e-6] = 0
    yin = energy[:1, :] + energy - 2 * acf
    num = yin[min_period:max_period + 1, :]
    tau = np.arange(1, max_period + 1)[:, None]
    cm = np.cumsum(yin[1:max_period + 1, :], axis=0) / tau
    den = cm[min_period - 1:max_period, :]
    return num / (den + TINY64)


def parabolic_interpolation(x):
    """librosa 0.10 _parabolic_interpolation along axis 0: -b / a with a = x[i+1] + x[i-1] - 2 x[i],
    b = (x[i+1] - x[i-1]) / 2, zero where |b| >= |a| and at both ends."""
    s = np.zeros_like(x)
    a = x[2:] + x[:-2] - 2 * x[1:-1]
    b = (x[2:] - x[:-2]) / 2
    with np.errstate(divide="ignore", invalid="ignore"):
        sh = np.where(np.abs(b) >= np.abs(a), 0.0, -b / a)
    s[1:-1] = sh
    return s


def localmin(x):
    """librosa.util.localmin along axis 0 (edge padding): x[i] < x[i-1] and x[i] <= x[i+1]."""
    xp = np.pad(x, [(1, 1)] + [(0, 0)] * (x.ndim - 1), mode="edge")
    return (x < xp[:-2]) & (x <= xp[2:])


def beta_cdf(x, a, b):
    """Regularised incomplete beta I_x(a, b) for integer a, b (the prior's (2, 18)): 1 - sum_{j<a} C(n, j) x^j (1-x)^(n-j)
    with n = a + b - 1 (exact for integer parameters)."""
    n = a + b - 1
    x = np.asarray(x, dtype=np.float64)
    s = np.zeros_like(x)
    for j in range(a):
        s += math.comb(n, j) * x ** j * (1 - x) ** (n - j)
    return 1.0 - s


def boltzmann_pmf(k, lam, n):
    """scipy.stats.boltzmann.pmf(k, lam, N=n) = (1 - e^-lam) e^(-lam k) / (1 - e^(-lam N)) for 0 <= k < N, else 0."""
    k = np.asarray(k, dtype=np.float64)
    n = np.asarray(n, dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        p = (1 - math.exp(-lam)) * np.exp(-lam * k) / (1 - np.exp(-lam * n))
    return np.where((k >= 0) & (k < n), p, 0.0)


def triang(m):
    """scipy.signal.windows.triang(m, sym=True)."""
    n = np.arange(1, (m + 1) // 2 + 1)
    if m % 2 == 0:
        w = (2 * n - 1.0) / m
        return np.r_[w, w[::-1]]
    w = 2 * n / (m + 1.0)
    return np.r_[w, w[-2::-1]]


def transition_local(n_states, width):
    """librosa.sequence.transition_local(n_states, width, window='triangle', wrap=False)."""
    t = np.zeros((n_states, n_states))
    win = triang(width)
    for i in range(n_states):
        row = np.zeros(n_states)
        lpad = (n_states - width) // 2
        row[lpad:lpad + width] = win  # util.pad_center
        row = np.roll(row, n_states // 2 + i + 1)
        row[min(n_states, i + width // 2 + 1):] = 0
        row[:max(0, i - width // 2)] = 0
        t[i] = row
    return t / t.sum(axis=1, keepdims=True)


def viterbi(prob, transition, p_init):
    """librosa.sequence.viterbi (log domain, argmax ties to the lowest state): prob [n_states, T] -> states [T]."""
    log_trans = np.log(transition + TINY64)
    log_prob = np.log(prob.T + TINY64)
    log_p = np.log(p_init + TINY64)
    T, S = log_prob.shape
    value = log_prob[0] + log_p
    ptr = np.zeros((T, S), dtype=np.int64)
    for t in range(1, T):
        trans_out = value[None, :] + log_trans.T  # [dest, src]
        ptr[t] = np.argmax(trans_out, axis=1)
        value = log_prob[t] + trans_out[np.arange(S), ptr[t]]
    state = np.zeros(T, dtype=np.int64)
    state[-1] = int(np.argmax(value))
    for t in range(T - 2, -1, -1):
        state[t] = ptr[t + 1, state[t + 1]]
    return state


def pyin_params(sr, fmin, fmax, frame_length=2048, win_length=None, hop_length=None, resolution=0.1,
                max_transition_rate=35.92):
    win_length = frame_length // 2 if win_length is None else win_length
    hop_length = frame_length // 4 if hop_length is None else hop_length
    min_period = max(int(np.floor(sr / fmax)), 1)
    max_period = min(int(np.ceil(sr / fmin)), frame_length - win_length - 1)
    bps = int(np.ceil(1.0 / resolution))
    n_bins = int(np.floor(12 * bps * np.log2(fmax / fmin))) + 1
    max_semitones = round(max_transition_rate * 12 * hop_length / sr)
    width = max_semitones * bps + 1
    return dict(win_length=win_length, hop_length=hop_length, min_period=min_period, max_period=max_period, bps=bps,
                n_bins=n_bins, width=width)


def observations(yin, shifts, sr, fmin, min_period, n_bins, bps, n_thresholds=100, beta=(2, 18), boltzmann=2.0,
                 no_trough_prob=0.01):
    """librosa's __pyin_helper: per frame, the trough probabilities (threshold prior x Boltzmann trough prior, the
    global minimum's share for thresholds below every trough) -> [2 n_bins, T] observation probabilities and the
    voiced probability [T]."""
    thresholds = np.linspace(0, 1, n_thresholds + 1)
    beta_probs = np.diff(beta_cdf(thresholds, *beta))
    yin_probs = np.zeros_like(yin)
    for i in range(yin.shape[1]):
        f = yin[:, i]
        is_trough = localmin(f)
        is_trough[0] = f[0] < f[1]
        (idx,) = np.nonzero(is_trough)
        if len(idx) == 0:
            continue
        heights = f[idx]
        below = np.less.outer(heights, thresholds[1:])
        pos = np.cumsum(below, axis=0) - 1
        n_tr = np.count_nonzero(below, axis=0)
        prior = boltzmann_pmf(pos, boltzmann, n_tr)
        prior[~below] = 0
        probs = prior.dot(beta_probs)
        gmin = int(np.argmin(heights))
        n_below_min = np.count_nonzero(~below[gmin, :])
        probs[gmin] += no_trough_prob * np.sum(beta_probs[:n_below_min])
        yin_probs[idx, i] = probs
    period, fi = np.nonzero(yin_probs)
    cand = min_period + period + shifts[period, fi]
    f0c = sr / cand
    bi = 12 * bps * np.log2(f0c / fmin)
    bi = np.clip(np.round(bi), 0, n_bins).astype(int)
    obs = np.zeros((2 * n_bins, yin.shape[1]))
    obs[bi, fi] = yin_probs[period, fi]  # (assignment: with two candidates in one bin the later period wins)
    voiced = np.clip(np.sum(obs[:n_bins, :], axis=0), 0, 1)
    obs[n_bins:, :] = (1 - voiced) / n_bins
    return obs, voiced


def pyin(y, fmin, fmax, sr, frame_length=2048, win_length=None, hop_length=None, switch_prob=0.01):
    """librosa.pyin(y, fmin=, fmax=, sr=, frame_length=2048, win_length=, hop_length=) -> (f0 [T] with NaN where
    unvoiced, voiced_flag [T], voiced_prob [T]); center=True (constant padding of frame_length // 2 each side)."""
    p = pyin_params(sr, fmin, fmax, frame_length, win_length, hop_length)
    y = np.pad(np.asarray(y, dtype=np.float64), (frame_length // 2, frame_length // 2), mode="constant")
    frames = frame(y, frame_length, p["hop_length"])
    yin = cumulative_mean_normalized_difference(frames, frame_length, p["win_length"], p["min_period"],
                                                p["max_period"])
    shifts = parabolic_interpolation(yin)
    obs, voiced = observations(yin, shifts, sr, fmin, p["min_period"], p["n_bins"], p["bps"])
    n_bins = p["n_bins"]
    trans = np.kron(np.array([[1 - switch_prob, switch_prob], [switch_prob, 1 - switch_prob]]),
                    transition_local(n_bins, p["width"]))
    p_init = np.zeros(2 * n_bins)
    p_init[n_bins:] = 1 / n_bins
    states = viterbi(obs, trans, p_init)
    freqs = fmin * 2 ** (np.arange(n_bins) / (12 * p["bps"]))
    f0 = freqs[states % n_bins]
    flag = states < n_bins
    f0 = np.where(flag, f0, np.nan)
    return f0, flag, voiced


def f0_pyin(audio, fs, win_length, hop_length, f0_min, f0_max):
    """utils/f0.py:95-117 get_f0_features_using_pyin: pyin with NaN (unvoiced) frames set to 0."""
    f0, flag, _ = pyin(audio, f0_min, f0_max, fs, win_length=win_length, hop_length=hop_length)
    f0 = f0.copy()
    f0[~flag] = 0
    return f0
