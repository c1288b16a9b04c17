"""Command-line counterpart of the reference's infer.py (infer.py:24-91): source wav + target singer ->
converted wav, on one MI355X through libsvc_hip.so.

    python -m svc_inference_pipeline_amd.infer --wav test_set/1100000814.wav --singer svcc_CDF1 \\
        --mapper-ckpt mapper.pt --vocoder-ckpt vocoder.pt --whisper-ckpt medium.pt [--fast] [--out gen/x.wav]
    python -m svc_inference_pipeline_amd.infer --wav a.wav b.wav c.wav ...   # several files: one ragged batch

Same sequence as the reference: acoustic features (mel, energy, Praat F0) -> pitch shift to the target
singer -> Whisper content features -> DiffSVC sampler (DDPM-1000 by default, PLMS with --fast, as
svc_model_inference's fast_inference) -> de-normalisation -> BigVGAN -> fade -> 16-bit wav (peak 0.9, 50 ms of
silence each side). Checkpoint paths default to the config's svc_model_path / vocoder_model_path. Without
checkpoints the run needs --random-weights (seeded weights of the reference architectures: plumbing and
timing only, the audio is noise).
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

from . import audio as A
from . import config as C
from . import weights as W
from .pipeline import SVCPipeline
from .runtime import SVCEngine


def build_engine(cfg, device=0, mapper_ckpt=None, vocoder_ckpt=None, whisper_ckpt=None, random_weights=None, seed=0):
    """Engine from the reference's checkpoints, or from seeded random weights when random_weights names a
    Whisper size ("medium" or "tiny-test"); checkpoints and random weights do not mix."""
    if random_weights:
        dims = W.WHISPER_DIMS[random_weights]
        if dims["n_audio_state"] != cfg.mapper.input_content_dim["whisper"]:
            cfg.mapper.input_content_dim["whisper"] = dims["n_audio_state"]
        return SVCEngine(cfg, device, whisper_state=W.make_whisper_state(dims, seed),
                         mapper_state=W.make_mapper_state(cfg.mapper, seed),
                         vocoder_state=W.make_vocoder_state(cfg.vocoder, seed))
    if not (mapper_ckpt and vocoder_ckpt and whisper_ckpt):
        raise SystemExit("need --mapper-ckpt, --vocoder-ckpt and --whisper-ckpt (or --random-weights)")
    st = W.load_checkpoints(mapper_ckpt, vocoder_ckpt, whisper_ckpt)
    return SVCEngine(cfg, device, whisper_state=st["whisper"], mapper_state=st["mapper"], vocoder_state=st["vocoder"])


def convert_file(engine, cfg, wav_path, singer_name, fast_inference=False, speedup=10, seed=0, device="cuda",
                 f0_method="parselmouth"):
    """One file through the GPU path -> (f32 waveform [T*hop] before save_audio's normalisation, T)."""
    wav24 = A.load_audio(wav_path, cfg.fs, device=device)          # utils/audio.py:10-55
    if wav24 is None:
        raise A.AudioError(f"{wav_path}: non-finite samples")
    wav16 = A.load_whisper_audio(wav_path, device=device)          # whisper_extractor/audio.py:22-49
    singers = C.load_singers(cfg)
    if singer_name not in singers:
        raise KeyError(f"unknown singer {singer_name!r}; known: {sorted(singers)}")
    singer = torch.tensor([int(singers[singer_name])], dtype=torch.int32, device=device)  # utils/util.py:49-54
    utt = torch.zeros(1, dtype=torch.int32, device=device)
    res = SVCPipeline(engine, f0_method=f0_method).convert(wav24[None].contiguous(), wav16[None].contiguous(), singer,
                                      fast_inference=fast_inference, speedup=speedup, seed=seed, utt_ids=utt)
    return res.wav[0].cpu().numpy(), res.mel.shape[1]


def convert_files(engine, cfg, wav_paths, singer_name, fast_inference=False, speedup=10, seed=0, device="cuda",
                  f0_method="parselmouth"):
    """Several files as ONE ragged batch (SVCPipeline.convert_many, per-utterance lengths through the C-ABI) ->
    list of (f32 waveform [T_i*hop], T_i); file i uses utterance id i, so file 0 equals convert_file's result."""
    singers = C.load_singers(cfg)
    if singer_name not in singers:
        raise KeyError(f"unknown singer {singer_name!r}; known: {sorted(singers)}")
    w24, w16 = [], []
    for p in wav_paths:
        w = A.load_audio(p, cfg.fs, device=device)
        if w is None:
            raise A.AudioError(f"{p}: non-finite samples")
        w24.append(w)
        w16.append(A.load_whisper_audio(p, device=device))
    sid = int(singers[singer_name])
    wavs = SVCPipeline(engine, f0_method=f0_method).convert_many(w24, w16, [sid] * len(w24), fast_inference=fast_inference,
                                            speedup=speedup, seed=seed)
    hop = cfg.hop_length
    return [(w.cpu().numpy(), int(w.shape[0]) // hop) for w in wavs]


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--wav", required=True, nargs="+",
                    help="one or more source files; several are converted as one ragged GPU batch")
    ap.add_argument("--singer", default="svcc_CDF1")
    ap.add_argument("--out", default=None, help="default gen/<wav stem>_<singer>.wav (infer.py:28); one file only")
    ap.add_argument("--config", default=None, help="reference-format config.json (default: the packaged one)")
    ap.add_argument("--fast", action="store_true", help="PLMS (fast_inference=True) instead of DDPM-1000")
    ap.add_argument("--speedup", type=int, default=10)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--mapper-ckpt", default=None)
    ap.add_argument("--vocoder-ckpt", default=None)
    ap.add_argument("--whisper-ckpt", default=None)
    ap.add_argument("--random-weights", default=None, choices=sorted(W.WHISPER_DIMS))
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--f0-method", default="parselmouth", choices=("parselmouth", "pyin"),
                    help="F0 extractor: Praat AC (the reference's infer.py) or pYIN (utils/f0.py:95-117; follows "
                         "librosa 0.10.1's pyin, parity-unpinned: librosa is not installed here)")
    args = ap.parse_args(argv)

    cfg = C.load_config(args.config) if args.config else C.load_config()
    mapper = args.mapper_ckpt or getattr(cfg, "svc_model_path", None)
    vocoder = args.vocoder_ckpt or getattr(cfg, "vocoder_model_path", None)
    print("Loading mapper and vocoder...", flush=True)
    engine = build_engine(cfg, args.device, mapper, vocoder, args.whisper_ckpt, args.random_weights, args.seed)
    if args.out and len(args.wav) > 1:
        raise SystemExit("--out names one output file: omit it when converting several files")
    t0 = time.time()
    print("Converting...", flush=True)
    dev = f"cuda:{args.device}"
    if len(args.wav) == 1:
        results = [convert_file(engine, cfg, args.wav[0], args.singer, args.fast, args.speedup, args.seed, device=dev,
                                f0_method=args.f0_method)]
    else:
        results = convert_files(engine, cfg, args.wav, args.singer, args.fast, args.speedup, args.seed, device=dev,
                                f0_method=args.f0_method)
    print(f"Using time: {time.time() - t0:.3f}s ({sum(T for _, T in results)} frames, {len(results)} file(s))",
          flush=True)
    for path, (wav, _) in zip(args.wav, results):
        out = args.out or os.path.join("gen", f"{os.path.splitext(os.path.basename(path))[0]}_{args.singer}.wav")
        A.save_audio(out, wav, cfg.fs)
        print("Saving", out, flush=True)
    engine.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
