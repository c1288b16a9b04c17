"""ORACLE (test infrastructure only) — acoustic/content feature front-end, CPU restatement.

Reference rows A2, A3(energy), A4, A5, A7, A13, A15 of SURVEY.md §8(a).
"""
import numpy as np
import torch

# ----------------------------------------------------------------------------- librosa slaney mel


def _hz_to_mel(freqs):
    """librosa.hz_to_mel(htk=False) as used by librosa.filters.mel (utils/mel.py:14,140)."""
    freqs = np.asanyarray(freqs, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = freqs / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if freqs.ndim:
        log_t = freqs >= min_log_hz
        mels[log_t] = min_log_mel + np.log(freqs[log_t] / min_log_hz) / logstep
    elif freqs >= min_log_hz:
        mels = min_log_mel + np.log(freqs / min_log_hz) / logstep
    return mels


def _mel_to_hz(mels):
    mels = np.asanyarray(mels, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * mels
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    log_t = mels >= min_log_mel
    freqs[log_t] = min_log_hz * np.exp(logstep * (mels[log_t] - min_log_mel))
    return freqs


def slaney_mel_filterbank(sr, n_fft, n_mels, fmin=0.0, fmax=None):
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax, htk=False, norm='slaney') -> f32[n_mels, 1+n_fft//2].
    Known-answer: utils/whisper_extractor/assets/mel_filters.npz (mel_80 = mel(16000, 400, 80))."""
    if fmax is None:
        fmax = float(sr) / 2
    weights = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2: n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


# ----------------------------------------------------------------------------- 24 kHz mel + energy


def mel_frames(n_samples, n_fft=1024, hop=256):
    """Frame count of utils/mel.py:148-167 (reflect pad (n_fft-hop)/2 both sides, center=False)."""
    return (n_samples + (n_fft - hop) - n_fft) // hop + 1


def mel_spectrogram(y, cfg):
    """utils/mel.py:130-174. y: f32[B, N] torch -> log-mel f32[B, n_mels, T]."""
    mel = torch.from_numpy(slaney_mel_filterbank(cfg.fs, cfg.n_fft, cfg.n_mels, cfg.fmin, cfg.fmax)).float()
    win = torch.hann_window(cfg.win_length)
    pad = int((cfg.n_fft - cfg.hop_length) / 2)
    y = torch.nn.functional.pad(y.unsqueeze(1), (pad, pad), mode="reflect").squeeze(1)
    spec = torch.stft(y, cfg.n_fft, hop_length=cfg.hop_length, win_length=cfg.win_length, window=win,
                      center=False, pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    spec = torch.view_as_real(spec)
    spec = torch.sqrt(spec.pow(2).sum(-1) + (1e-9))
    spec = torch.matmul(mel, spec)
    return torch.log(torch.clamp(spec, min=1e-5))


def energy_from_mel(mel):
    """utils/mel.py:199: (mel.exp() ** 2).sum(0).sqrt() per utterance; mel [B, n_mels, T] -> [B, T]."""
    return (mel.exp() ** 2).sum(1).sqrt()


# ----------------------------------------------------------------------------- Whisper log-mel (16 kHz)

WHISPER_N_SAMPLES = 480000


def pad_or_trim(audio, length=WHISPER_N_SAMPLES):
    """utils/whisper_extractor/audio.py:52-73 (numpy branch)."""
    if audio.shape[-1] > length:
        audio = audio[..., :length]
    if audio.shape[-1] < length:
        pad = [(0, 0)] * audio.ndim
        pad[-1] = (0, length - audio.shape[-1])
        audio = np.pad(audio, pad)
    return audio


def whisper_mel_filters():
    return slaney_mel_filterbank(16000, 400, 80)


def whisper_log_mel(audio16k):
    """utils/whisper_extractor/audio.py:92-124. audio16k: f32[B, 480000] torch -> f32[B, 80, 3000].
    The max-8 clamp is per utterance (the reference processes one utterance per call)."""
    window = torch.hann_window(400)
    stft = torch.stft(audio16k, 400, 160, window=window, return_complex=True)
    magnitudes = stft[..., :-1].abs() ** 2
    filters = torch.from_numpy(whisper_mel_filters())
    mel_spec = filters @ magnitudes
    log_spec = torch.clamp(mel_spec, min=1e-10).log10()
    mx = log_spec.amax(dim=(-2, -1), keepdim=True)
    log_spec = torch.maximum(log_spec, mx - 8.0)
    return (log_spec + 4.0) / 4.0


def quantize_16k(audio16k):
    """utils/whisper_extractor/audio.py:41-49: ffmpeg s16le decode -> int16 / 32768."""
    q = np.clip(np.round(np.asarray(audio16k, dtype=np.float64) * 32768.0), -32768, 32767).astype(np.int16)
    return q.astype(np.float32) / 32768.0


# ----------------------------------------------------------------------------- content mapping


def map_whisper_features(raw_feats, target_len_in, fast_mapping=True):
    """utils/whisper.py:31-81 (numpy, f32). raw_feats [1500, D] -> [min(T, 2812), D]."""
    source_hop, target_hop = 480, 256
    g = np.gcd(source_hop, target_hop)
    source_hop //= g
    target_hop //= g
    max_source_len = 1500
    target_len = min(target_len_in, max_source_len * source_hop // target_hop)
    width = raw_feats.shape[-1]
    if fast_mapping:
        source_len = target_len * target_hop // source_hop + 1
        raw_feats = raw_feats[:source_len]
    else:
        source_len = max_source_len
    const = source_len * source_hop // target_hop * target_hop
    up = np.repeat(raw_feats, source_hop, axis=0)
    down = np.average(up[:const].reshape(-1, target_hop, width), axis=1)
    assert len(down) >= target_len
    return down[:target_len]


class MappingError(RuntimeError):
    """utils/hubert.py:114-120: the reference calls exit() when the mapped length is off by more than 3."""


def map_hubert_features(raw_feats, target_len):
    """utils/hubert.py:83-134 (get_mapped_features, numpy f32). raw_feats [src_len, D] -> [target_len, D]:
    the same 15:8 repeat/average as Whisper but without the 2812 cap or the fast_mapping truncation;
    a shortfall of at most 3 rows is filled with the last mapped row, anything larger is an error."""
    source_hop, target_hop = 480, 256
    g = np.gcd(source_hop, target_hop)
    source_hop //= g
    target_hop //= g
    source_len, width = raw_feats.shape
    const = source_len * source_hop // target_hop * target_hop
    up = np.repeat(raw_feats, source_hop, axis=0)
    down = np.average(up[:const].reshape(-1, target_hop, width), axis=1)
    err = abs(target_len - len(down))
    if err > 3:
        raise MappingError(f"content vector maps to {len(down)} frames, mel has {target_len}")
    if len(down) < target_len:
        down = np.concatenate([down, down[-1][None, :].repeat(err, axis=0)], axis=0)
    return down[:target_len]


# ----------------------------------------------------------------------------- F0 pitch shift, mel denorm


def pitch_shift(raw_f0, target_median):
    """utils/acoustic_feature_extraction.py:33-52 (target median precomputed from config/f0.pkl)."""
    voiced = np.where(raw_f0 != 0)
    factor = target_median / np.median(raw_f0[voiced])
    return raw_f0 * factor


def denormalize_mel_channel(mel, mel_min, mel_max):
    """utils/acoustic_feature_extraction.py:83-97. mel f32[n_mel, T] numpy."""
    ZERO = 1e-12
    mn = np.expand_dims(mel_min, -1)
    mx = np.expand_dims(mel_max, -1)
    return (mel + 1) / 2 * (mx - mn + ZERO) + mn


def synthesis_fade(audio, T, hop=256):
    """modules/bigvgan_inference.py:33-44: trim to T*hop, linear fade-out on the last 20*hop samples."""
    fade = torch.linspace(1, 0, steps=20 * hop)
    audio = audio[..., : T * hop].clone()
    audio[..., -20 * hop:] *= fade
    return audio


def save_audio_pcm16(waveform, fs, volume_peak=0.9):
    """utils/util.py:20-37 -> int16 samples (peak 0.9, fs//20 zeros both sides, PCM_S16 = round(x*32768))."""
    ratio = volume_peak / max(waveform.max(), abs(waveform.min()))
    waveform = waveform * ratio
    sil = np.zeros((fs // 20,), dtype=waveform.dtype)
    w = np.concatenate([sil, waveform, sil]).astype(np.float32)
    return np.clip(np.round(w.astype(np.float64) * 32768.0), -32768, 32767).astype(np.int16)
