"""Audio I/O for the conversion path, mirroring the reference's host functions.

    load_audio_torch(wave_file, fs)   utils/audio.py:10-55            -> load_audio (+ resample on the GPU)
    load_audio(file, sr=16000)        utils/whisper_extractor/audio.py:22-49 (ffmpeg s16le decode)
                                                                      -> load_whisper_audio
    save_audio(path, waveform, fs)    utils/util.py:20-37              -> save_audio

The reference reads wavs with soundfile, resamples with librosa (soxr) and decodes Whisper's 16 kHz input with
an ffmpeg subprocess; none of the three is in this image. Here a RIFF/WAVE reader gives soundfile's float
conversion (PCM int / 2^(bits-1), IEEE float as stored), and resampling runs in libsvc_hip.so
(`svc_resample`: scipy.signal.resample_poly's Kaiser(5) polyphase filter; parity pinned to scipy, unpinned
against soxr / ffmpeg's swresample). Only WAV input is supported (the reference's non-wav branch uses
librosa.load).
"""
import ctypes
import os
import struct

import numpy as np
import torch

from . import _lib

WHISPER_SR = 16000  # utils/whisper_extractor/audio.py:12


class AudioError(ValueError):
    pass


def read_wav(path):
    """RIFF/WAVE -> (float64 [n, channels], sample_rate), with soundfile.read's float scaling.
    PCM 8 (unsigned), 16, 24, 32-bit and IEEE float 32/64, WAVE_FORMAT_EXTENSIBLE included."""
    with open(path, "rb") as fh:
        data = fh.read()
    if len(data) < 12 or data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise AudioError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, payload = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, sr, _, align, bits = struct.unpack("<HHIIHH", body[:16])
            if tag == 0xFFFE and len(body) >= 26:  # WAVE_FORMAT_EXTENSIBLE: sub-format GUID's first 2 bytes
                tag = struct.unpack("<H", body[24:26])[0]
            fmt = (tag, ch, sr, align, bits)
        elif cid == b"data":
            payload = body
        pos += 8 + size + (size & 1)
    if fmt is None or payload is None:
        raise AudioError(f"{path}: missing fmt or data chunk")
    tag, ch, sr, align, bits = fmt
    if ch < 1 or align != ch * bits // 8:
        raise AudioError(f"{path}: unsupported layout ({ch} channels, block align {align}, {bits} bits)")
    n = len(payload) // align
    raw = np.frombuffer(payload[:n * align], dtype=np.uint8)
    if tag == 1 and bits == 8:
        x = (raw.astype(np.float64) - 128.0) / 128.0
    elif tag == 1 and bits == 16:
        x = raw.view("<i2").astype(np.float64) / 32768.0
    elif tag == 1 and bits == 24:
        b3 = raw.reshape(-1, 3).astype(np.int32)
        v = b3[:, 0] | (b3[:, 1] << 8) | (b3[:, 2] << 16)
        x = (np.where(v >= 1 << 23, v - (1 << 24), v)).astype(np.float64) / float(1 << 23)
    elif tag == 1 and bits == 32:
        x = raw.view("<i4").astype(np.float64) / float(1 << 31)
    elif tag == 3 and bits == 32:
        x = raw.view("<f4").astype(np.float64)
    elif tag == 3 and bits == 64:
        x = raw.view("<f8").copy()
    else:
        raise AudioError(f"{path}: unsupported sample format (tag {tag}, {bits} bits)")
    return x.reshape(n, ch), sr


def _normalise(audio):
    """utils/audio.py:31-45: float data scaled by 1, 2^15+1 or 2^31+1 by its peak, then float32."""
    mx = max(float(np.amax(audio)), float(-np.amin(audio))) if audio.size else 0.0
    max_mag = (2 ** 31) + 1 if mx > 2 ** 15 else ((2 ** 15) + 1 if mx > 1.01 else 1.0)
    return (torch.from_numpy(audio.astype(np.float32)) / max_mag).numpy()


def resample(x, sr_in, sr_out, device="cuda", quantize16=False):
    """f32 [B, n] or [n] (host or device) -> device f32 at sr_out, on the current stream (svc_resample)."""
    xt = torch.as_tensor(x, dtype=torch.float32, device=device)
    squeeze = xt.dim() == 1
    if squeeze:
        xt = xt[None]
    xt = xt.contiguous()
    B, n_in = xt.shape
    n_out = _lib.load().svc_resample_len(n_in, sr_in, sr_out)
    y = torch.empty(B, n_out, device=xt.device, dtype=torch.float32)
    _lib.call("svc_resample", ctypes.c_void_p(xt.data_ptr()), B, n_in, sr_in, sr_out, 1 if quantize16 else 0,
              ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream(xt.device).cuda_stream))
    return y[0] if squeeze else y


def load_audio(path, fs, device="cuda"):
    """utils/audio.py:10-55 for a wav: channel 0, peak-class normalisation, resample to fs on the GPU.
    Returns a device f32 tensor, or None where the reference returns [] (NaN / Inf samples)."""
    audio, sr = read_wav(path)
    audio = audio[:, 0]
    if len(audio) <= 2:
        raise AudioError(f"{path}: {len(audio)} samples")
    x = _normalise(audio)
    if not np.isfinite(x).all():
        return None
    if sr == fs:
        return torch.as_tensor(x, device=device)
    return resample(x, sr, fs, device=device)


def load_whisper_audio(path, sr=WHISPER_SR, device="cuda"):
    """utils/whisper_extractor/audio.py:22-49: mono down-mix (ffmpeg ac=1 averages the channels), resample to
    16 kHz and quantise to int16 / 32768 (the s16le pipe)."""
    audio, sr_in = read_wav(path)
    mono = audio.mean(axis=1).astype(np.float32)
    return resample(mono, sr_in, sr, device=device, quantize16=True)


def to_pcm16(waveform, fs, add_silence=True, turn_up=True, volume_peak=0.9):
    """utils/util.py:20-37 sample conversion: peak to volume_peak, fs//20 zeros both sides,
    PCM_S16 = clip(round(x * 32768)) (matches gen/1100000814_svcc_CDF1.wav: peak -29491)."""
    w = np.asarray(waveform, dtype=np.float32)
    if turn_up:
        w = w * (volume_peak / max(float(w.max()), abs(float(w.min()))))
    if add_silence:
        sil = np.zeros((fs // 20,), dtype=w.dtype)
        w = np.concatenate([sil, w, sil])
    return np.clip(np.round(w.astype(np.float64) * 32768.0), -32768, 32767).astype(np.int16)


def write_wav_pcm16(path, pcm, fs):
    pcm = np.asarray(pcm, dtype="<i2")
    body = pcm.tobytes()
    hdr = b"RIFF" + struct.pack("<I", 36 + len(body)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, fs, fs * 2, 2, 16)
    hdr += b"data" + struct.pack("<I", len(body))
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "wb") as fh:
        fh.write(hdr + body)


def save_audio(path, waveform, fs, add_silence=True, turn_up=True, volume_peak=0.9):
    """utils/util.py:20-37: 16-bit PCM mono wav."""
    write_wav_pcm16(path, to_pcm16(waveform, fs, add_silence, turn_up, volume_peak), fs)
