"""ORACLE (test infrastructure only) — Praat autocorrelation pitch (Sound: To Pitch (ac)...).

The reference calls parselmouth (Praat) at utils/f0.py:144-153:
    parselmouth.Sound(audio, fs).to_pitch_ac(time_step=hop/fs, voicing_threshold=0.6,
                                             pitch_floor=65, pitch_ceiling=800).selected_array["frequency"]
and pads the result to the mel length at :156-157. parselmouth/Praat (unpinned dependency, Praat
6.x via parselmouth 0.4.x era, 2023) is NOT installed here, so this module restates Praat's published
algorithm (Boersma 1993, "Accurate short-term analysis of the fundamental frequency and the
harmonics-to-noise ratio of a sampled sound"; Praat sources Sound_to_Pitch.cpp, Pitch.cpp
Pitch_pathFinder, NUM.cpp NUM_interpolate_sinc / NUMimproveExtremum / NUMminimize_brent) with the
parselmouth defaults for the arguments the reference leaves unset (max candidates 15, very_accurate
False -> Hanning window, 3 periods, silence 0.03, octave cost 0.01, octave-jump cost 0.35,
voiced/unvoiced cost 0.14). PARITY UNPINNED: checked by known-answer tests on synthetic tones
(tests/test_f0.py), not against Praat output.
"""
import math

import numpy as np

EPS_SQRT = math.sqrt(np.finfo(np.float64).eps)
GOLDEN = 1.0 - 0.6180339887498949  # 1 - NUM_goldenSection


# ----------------------------------------------------------------------------- NUM helpers (1-based y)


def interpolate_sinc(y, x, max_depth):
    """NUM_interpolate_sinc: y is a 0-based array standing for Praat's 1-based vector y[1..n]."""
    n = len(y)
    midleft = math.floor(x)
    midright = midleft + 1
    if n < 1:
        return float("nan")
    if x > n:
        return y[n - 1]
    if x < 1:
        return y[0]
    if x == midleft:
        return y[midleft - 1]
    if max_depth > midright - 1:
        max_depth = midright - 1
    if max_depth > n - midleft:
        max_depth = n - midleft
    if max_depth <= 0:
        return y[math.floor(x + 0.5) - 1]
    if max_depth == 1:
        return y[midleft - 1] + (x - midleft) * (y[midright - 1] - y[midleft - 1])
    if max_depth == 2:
        yl, yr = y[midleft - 1], y[midright - 1]
        dyl = 0.5 * (yr - y[midleft - 2])
        dyr = 0.5 * (y[midright] - yl)
        fil, fir = x - midleft, midright - x
        return yl * fir + yr * fil - fil * fir * (0.5 * (dyr - dyl) + (fil - 0.5) * (dyl + dyr - 2 * (yr - yl)))
    left = midright - max_depth
    right = midleft + max_depth
    result = 0.0
    a = math.pi * (x - midleft)
    halfsina = 0.5 * math.sin(a)
    aa = a / (x - left + 1.0)
    daa = math.pi / (x - left + 1.0)
    cosaa, sinaa, cosdaa, sindaa = math.cos(aa), math.sin(aa), math.cos(daa), math.sin(daa)
    for ix in range(midleft, left - 1, -1):
        d = halfsina / a * (1.0 + cosaa)
        result += y[ix - 1] * d
        a += math.pi
        help_ = cosaa * cosdaa - sinaa * sindaa
        sinaa = cosaa * sindaa + sinaa * cosdaa
        cosaa = help_
        halfsina = -halfsina
    a = math.pi * (midright - x)
    halfsina = 0.5 * math.sin(a)
    aa = a / (right - x + 1.0)
    daa = math.pi / (right - x + 1.0)
    cosaa, sinaa, cosdaa, sindaa = math.cos(aa), math.sin(aa), math.cos(daa), math.sin(daa)
    for ix in range(midright, right + 1):
        d = halfsina / a * (1.0 + cosaa)
        result += y[ix - 1] * d
        a += math.pi
        help_ = cosaa * cosdaa - sinaa * sindaa
        sinaa = cosaa * sindaa + sinaa * cosdaa
        cosaa = help_
        halfsina = -halfsina
    return result


def minimize_brent(f, a, b, tol):
    """NUMminimize_brent: returns (xmin, fmin); golden section + parabolic steps, 60 iterations max."""
    v = a + GOLDEN * (b - a)
    fv = f(v)
    x = w = v
    fx = fw = fv
    for _ in range(60):
        rng = b - a
        middle = (a + b) / 2
        tol_act = EPS_SQRT * abs(x) + tol / 3
        if abs(x - middle) + rng / 2 <= 2 * tol_act:
            return x, fx
        new_step = GOLDEN * (b - x if x < middle else a - x)
        if abs(x - w) >= tol_act:
            t = (x - w) * (fx - fv)
            q = (x - v) * (fx - fw)
            p = (x - v) * q - (x - w) * t
            q = 2 * (q - t)
            if q > 0:
                p = -p
            else:
                q = -q
            if abs(p) < abs(new_step * q) and p > q * (a - x + 2 * tol_act) and p < q * (b - x - 2 * tol_act):
                new_step = p / q
        if abs(new_step) < tol_act:
            new_step = tol_act if new_step > 0 else -tol_act
        t = x + new_step
        ft = f(t)
        if ft <= fx:
            if t < x:
                b = x
            else:
                a = x
            v, w, x = w, x, t
            fv, fw, fx = fw, fx, ft
        else:
            if t < x:
                a = t
            else:
                b = t
            if ft <= fw or w == x:
                v, w = w, t
                fv, fw = fw, ft
            elif ft <= fv or v == x or v == w:
                v, fv = t, ft
    return x, fx


def improve_maximum(y, ixmid, depth):
    """NUMimproveExtremum(isMaximum=true) with sinc interpolation: returns (x_real, value)."""
    n = len(y)
    if ixmid <= 1:
        return 1.0, y[0]
    if ixmid >= n:
        return float(n), y[n - 1]
    xr, fr = minimize_brent(lambda xx: -interpolate_sinc(y, xx, depth), ixmid - 1, ixmid + 1, 1e-10)
    return xr, -fr


# ----------------------------------------------------------------------------- analysis


def analysis_params(n_samples, fs, time_step, floor, ceiling, max_cands=15, periods=3.0):
    dx = 1.0 / fs
    if max_cands < ceiling / floor:
        max_cands = int(math.floor(ceiling / floor))
    nsamp_period = int(math.floor(1.0 / dx / floor))
    halfnsamp_period = nsamp_period // 2 + 1
    if ceiling > 0.5 / dx:
        ceiling = 0.5 / dx
    dt_window = periods / floor
    nsamp_window = int(math.floor(dt_window / dx))
    halfnsamp_window = nsamp_window // 2 - 1
    nsamp_window = halfnsamp_window * 2
    maximum_lag = min(int(math.floor(nsamp_window / periods)) + 2, nsamp_window)
    duration = n_samples * dx
    n_frames = int(math.floor((duration - dt_window) / time_step)) + 1
    x1 = 0.5 * dx
    mid = x1 - 0.5 * dx + 0.5 * duration
    t1 = mid - 0.5 * n_frames * time_step + 0.5 * time_step
    nfft = 1
    while nfft < nsamp_window * 1.5:
        nfft *= 2
    brent_ixmax = int(math.floor(nsamp_window * 0.5))
    return dict(dx=dx, max_cands=max_cands, nsamp_period=nsamp_period, halfnsamp_period=halfnsamp_period,
                ceiling=ceiling, nsamp_window=nsamp_window, halfnsamp_window=halfnsamp_window, maximum_lag=maximum_lag,
                n_frames=n_frames, t1=t1, x1=x1, nfft=nfft, brent_ixmax=brent_ixmax, time_step=time_step)


def hanning(nw):
    i = np.arange(1, nw + 1, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(i * 2 * math.pi / (nw + 1))


def window_autocorr(window, nfft):
    w = np.zeros(nfft)
    w[: len(window)] = window
    p = np.abs(np.fft.rfft(w)) ** 2
    r = np.fft.irfft(p, nfft)
    return r / r[0]


def frame_candidates(x, i_frame, P, global_peak, window, windowR, voicing, octave_cost, floor):
    """Sound_into_PitchFrame (AC, Hanning): returns (intensity, [(freq, strength), ...])."""
    dx = P["dx"]
    t = P["t1"] + i_frame * P["time_step"]
    left = int(math.floor((t - P["x1"]) / dx)) + 1  # Sampled_xToLowIndex (1-based)
    right = left + 1
    nsp, hnw, nw = P["nsamp_period"], P["halfnsamp_window"], P["nsamp_window"]
    # local mean over one longest period each side (1-based [right-nsp, left+nsp])
    local_mean = x[right - nsp - 1: left + nsp].sum() / (2 * nsp)
    start = right - hnw  # 1-based
    frame = (x[start - 1: start - 1 + nw] - local_mean) * window
    s0 = max(1, hnw + 1 - P["halfnsamp_period"])
    s1 = min(nw, hnw + P["halfnsamp_period"])
    local_peak = np.abs(frame[s0 - 1: s1]).max()
    intensity = 1.0 if local_peak > global_peak else local_peak / global_peak
    cands = [(0.0, 0.0)]
    if local_peak == 0.0:
        return intensity, cands
    nfft = P["nfft"]
    buf = np.zeros(nfft)
    buf[:nw] = frame
    ac = np.fft.irfft(np.abs(np.fft.rfft(buf)) ** 2, nfft)
    bmax = P["brent_ixmax"]
    r = np.empty(2 * bmax + 1)  # r[-bmax..bmax] stored at index lag + bmax
    r[bmax] = 1.0
    lags = np.arange(1, bmax + 1)
    vals = ac[lags] / (ac[0] * windowR[lags])
    r[bmax + lags] = vals
    r[bmax - lags] = vals
    R = lambda lag: r[bmax + lag]
    imax = [0]
    max_cands = P["max_cands"]
    for i in range(2, min(P["maximum_lag"], bmax)):
        ri = R(i)
        if ri > 0.5 * voicing and ri > R(i - 1) and ri >= R(i + 1):
            dr = 0.5 * (R(i + 1) - R(i - 1))
            d2r = 2.0 * ri - R(i - 1) - R(i + 1)
            freq = 1.0 / dx / (i + dr / d2r)
            # vector coordinate of lag L is L + bmax + 1 (1-based)
            strength = interpolate_sinc(r, 1.0 / dx / freq + bmax + 1, 30)
            if strength > 1.0:
                strength = 1.0 / strength
            place = 0
            if len(cands) < max_cands:
                cands.append(None)
                imax.append(0)
                place = len(cands) - 1
            else:
                weakest = 2.0
                for iw in range(1, max_cands):
                    fq, st = cands[iw]
                    ls = st - octave_cost * math.log2(floor / fq)
                    if ls < weakest:
                        weakest = ls
                        place = iw
                if strength - octave_cost * math.log2(floor / freq) <= weakest:
                    place = 0
            if place:
                cands[place] = (freq, strength)
                imax[place] = i
    for k in range(1, len(cands)):
        xmid, ymid = improve_maximum(r, imax[k] + bmax + 1, 70)
        xmid -= bmax + 1
        freq = 1.0 / dx / xmid
        if ymid > 1.0:
            ymid = 1.0 / ymid
        cands[k] = (freq, ymid)
    return intensity, cands


def path_finder(frames, time_step, silence, voicing, octave_cost, octave_jump, vuv_cost, ceiling):
    """Pitch_pathFinder (Viterbi over candidates): returns the chosen candidate index per frame."""
    tsc = 0.01 / time_step
    octave_jump *= tsc
    vuv_cost *= tsc
    nf = len(frames)
    voiced = lambda f: f > 0.0 and f < ceiling
    delta = []
    for inten, cands in frames:
        us = 0.0 if silence <= 0 else 2.0 - inten / (silence / (1.0 + voicing))
        us = voicing + (us if us > 0 else 0.0)
        delta.append([us if not voiced(f) else st - octave_cost * math.log2(ceiling / f) for f, st in cands])
    psi = [[0] * len(c) for _, c in frames]
    for i in range(1, nf):
        prev, cur = frames[i - 1][1], frames[i][1]
        nd = []
        for j, (f2, _) in enumerate(cur):
            best, place = -1e30, 0
            v2 = voiced(f2)
            for k, (f1, _) in enumerate(prev):
                v1 = voiced(f1)
                if not v2:
                    tc = 0.0 if not v1 else vuv_cost
                else:
                    tc = vuv_cost if not v1 else octave_jump * abs(math.log2(f1 / f2))
                val = delta[i - 1][k] - tc + delta[i][j]
                if val > best:
                    best, place = val, k
            nd.append(best)
            psi[i][j] = place
        delta[i] = nd
    place = 0
    best = delta[-1][0]
    for j in range(1, len(delta[-1])):
        if delta[-1][j] > best:
            best, place = delta[-1][j], j
    path = [0] * nf
    for i in range(nf - 1, -1, -1):
        path[i] = place
        place = psi[i][place]
    return path


def to_pitch_ac(x, fs, time_step, floor=65.0, ceiling=800.0, voicing=0.6, silence=0.03, octave_cost=0.01,
                octave_jump=0.35, vuv_cost=0.14, max_cands=15):
    """parselmouth.Sound(x, fs).to_pitch_ac(...).selected_array['frequency'] (f64[n_frames])."""
    x = np.asarray(x, dtype=np.float64)
    P = analysis_params(len(x), fs, time_step, floor, ceiling, max_cands)
    if P["n_frames"] < 1:
        raise ValueError("sound shorter than the analysis window")
    global_peak = np.abs(x - x.sum() / len(x)).max()
    if global_peak == 0.0:
        return np.zeros(P["n_frames"])
    window = hanning(P["nsamp_window"])
    windowR = window_autocorr(window, P["nfft"])
    frames = [frame_candidates(x, i, P, global_peak, window, windowR, voicing, octave_cost, floor)
              for i in range(P["n_frames"])]
    path = path_finder(frames, time_step, silence, voicing, octave_cost, octave_jump, vuv_cost, P["ceiling"])
    return np.array([frames[i][1][path[i]][0] for i in range(len(frames))], dtype=np.float64)


def f0_features(audio, mel_len, fs=24000, hop=256, floor=65.0, ceiling=800.0):
    """utils/f0.py:120-161 (f0 part; f0_to_coarse's result is discarded by the reference)."""
    f0 = to_pitch_ac(audio, fs, hop / fs, floor=floor, ceiling=ceiling, voicing=0.6)
    pad = (int(len(audio) // hop) - len(f0) + 1) // 2
    return np.pad(f0, [[pad, mel_len - len(f0) - pad]], mode="constant")
