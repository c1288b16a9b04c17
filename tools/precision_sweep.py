"""mel-L1 tolerance sweep: content encoder (Whisper-medium, the headline, or HuBERT/ContentVec, BASELINE config 5)
+ DDPM-1000 + BigVGAN, fp16 vs bf16 operands, and the HIP path's precision modes.

The reference runs in fp32. The HIP path feeds MFMA with fp16 operands and accumulates in fp32 (DESIGN.md,
"Dtypes"); bf16 runs at the same gfx950 MFMA rate but keeps 8 instead of 11 significand bits. This tool measures
what that choice costs on the config-5 path, against the fp32 oracle on identical inputs, weights, x_T and
per-step noise:

  fp16-emu / bf16-emu : the oracle with every dense conv / linear / attention matmul rounding its operands to
                        that type (oracle.models.OperandRounding), fp32 accumulation — the operand precision a
                        bf16 build of the same kernels would have.
  gpu-fp16            : the actual HIP path (--gpu; needs an MI355X), through the C-ABI.
  gpu-bf16            : the same kernels with bfloat16 operands on v_mfma_f32_16x16x32_bf16 (--gpu --bf16;
                        SVCEngine(operands="bf16")), plain and in the default split modes.

Metrics, per SURVEY.md §7.3: mel-L1 = mean |delta| of the de-normalised natural-log mel fed to the vocoder (the
north-star target is <= 1e-3), plus the same in normalised units, the content features' and the waveform's
relative L2. Random weights (no checkpoints offline) make BigVGAN chaotic, so the waveform figure is
informational. Usage: python tools/precision_sweep.py [--content whisper|contentvec] [--gpu] [--no-emu] [--no-vocoder]
[--seconds 1.0] > profiles/<round>_precision_sweep.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oracle import features as OF  # noqa: E402
from oracle import models as OM  # noqa: E402
from oracle import noise as ON  # noqa: E402
from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd import weights as W  # noqa: E402


def rel_l2(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def oracle_chain(cfg, ws, hs, ms, vs, w24, w16, f0, xT, noise_fn, stats, vocoder=True):
    from oracle import pipeline as OP
    mel = OF.mel_spectrogram(torch.from_numpy(w24)[None], cfg)
    en = OF.energy_from_mel(mel)
    T = mel.shape[-1]
    f0s = torch.from_numpy(OF.pitch_shift(f0, stats["target_f0_median"]))[None]
    with torch.no_grad():
        if hs is not None:
            content = OP.hubert_content(hs, w16, T)
            ctype = "contentvec"
        else:
            content = OP.whisper_content(ws, w16, T)
            ctype = "whisper"
        content = torch.from_numpy(np.asarray(content, np.float32))[None]
        cond = OM.conditioner(ms, {ctype: content}, f0s, en, torch.tensor([[2]]))
        table = W.step_embedding_table(1000)
        consts = OM.schedule_constants(C.noise_schedule(cfg.mapper))
        den = lambda x, t: OM.diffsvc_forward(ms, cfg.mapper, x, cond, t, table)  # noqa: E731
        x0 = OM.sample_ddpm(den, torch.from_numpy(xT), 1, T, 1000, consts, noise_fn)
        mel_d = OF.denormalize_mel_channel(x0[0].numpy().T, stats["mel_min"], stats["mel_max"]).astype(np.float32)
        wav = None
        if vocoder:
            wav = OM.bigvgan_forward(vs, cfg.vocoder, torch.from_numpy(mel_d)[None])
            wav = OF.synthesis_fade(wav[0, 0], T).numpy()
    return dict(content=content[0].numpy(), x0=x0[0].numpy(), mel=mel_d.T, wav=wav)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--content", choices=["whisper", "contentvec"], default="contentvec")
    ap.add_argument("--whisper-dims", default="medium")
    ap.add_argument("--no-emu", action="store_true", help="skip the fp16 / bf16 operand emulations")
    ap.add_argument("--no-vocoder", action="store_true", help="mel-L1 only (skip BigVGAN)")
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--wsplit-variants", default="",
                    help="with --gpu, only these weight-split Whisper variants: comma-separated attn_mask:mlp_mask "
                         "or attn:mlp:qk:v:out masks "
                         "(content.wsplit_attn / content.wsplit_mlp, bit i = block i; e.g. 16777215:0 = attention "
                         "linears of all 24 blocks, no MLP linear)")
    ap.add_argument("--seed", type=int, default=7, help="synthetic clip seed")
    ap.add_argument("--bf16", action="store_true", help="with --gpu: the fp16-vs-bf16 operand sweep (BASELINE "
                    "configs[4]): plain and default-mode fp16 against plain and default-mode bf16")
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    cfg = C.load_config()
    ws = hs = None
    if args.content == "contentvec":
        cfg.mapper.content_feature = ["contentvec"]
        cfg.mapper.input_content_dim["contentvec"] = W.HUBERT_DIMS["contentvec"]["final_dim"]
        hs = W.make_hubert_state(W.HUBERT_DIMS["contentvec"], 0)
        w16 = ON.synth_clip(args.seed, args.seconds, 16000).astype(np.float32)
    else:
        dims = W.WHISPER_DIMS[args.whisper_dims]
        cfg.mapper.input_content_dim["whisper"] = dims["n_audio_state"]
        ws = W.make_whisper_state(dims, 0)
        w16 = ON.synth_clip_16k_quantised(args.seed, args.seconds)
    ms = W.make_mapper_state(cfg.mapper, 0)
    vs = W.make_vocoder_state(cfg.vocoder, 0)
    stats = C.load_stats(cfg)
    w24 = ON.synth_clip(args.seed, args.seconds, 24000).astype(np.float32)
    T = OF.mel_frames(len(w24))
    f0 = ON.synth_f0(4, T)
    seed = 17
    xT = ON.x_T(seed, 1, T)
    noise_fn = lambda i: torch.from_numpy(ON.step_noise(seed, i, 1, T))  # noqa: E731
    voc = not args.no_vocoder

    results = {}
    t0 = time.time()
    ref = oracle_chain(cfg, ws, hs, ms, vs, w24, w16, f0, xT, noise_fn, stats, voc)
    timing = {"fp32": round(time.time() - t0, 1)}
    runs = {}
    for name, dt in (() if args.no_emu else (("fp16-emu", torch.float16), ("bf16-emu", torch.bfloat16))):
        t0 = time.time()
        with OM.OperandRounding(dt, linear=True):
            runs[name] = oracle_chain(cfg, ws, hs, ms, vs, w24, w16, f0, xT, noise_fn, stats, voc)
        timing[name] = round(time.time() - t0, 1)
    if args.gpu:
        from svc_inference_pipeline_amd.pipeline import SVCPipeline
        from svc_inference_pipeline_amd.runtime import SVCEngine
        variants = [("gpu-fp16", False, False, None), ("gpu, split-fp16 content encoder", True, False, None),
                    ("gpu, split-fp16 DiffSVC head", False, True, None),
                    ("gpu, split-fp16 content encoder + DiffSVC head", True, True, None),
                    ("gpu, weight-split content linears + split-fp16 DiffSVC head (default)", 2, True, None)]
        if args.bf16:
            variants = [("gpu-fp16 (plain fp16 operands)", 0, False, None),
                        ("gpu-fp16, default precision mode", 2, True, None),
                        ("gpu-bf16 (plain bf16 operands)", 0, False, {"operands": "bf16"}),
                        ("gpu-bf16, default precision mode (split bf16 operands)", 2, True, {"operands": "bf16"})]
        if args.wsplit_variants:
            variants = []
            for v in args.wsplit_variants.split(","):
                f = [int(x, 0) for x in v.split(":")]
                extra = {"content.wsplit_attn": f[0], "content.wsplit_mlp": f[1]}
                name = f"gpu, weight-split attention {f[0]:#x} MLP {f[1]:#x}"
                if len(f) == 5:  # att:mlp:qk:v:out
                    extra.update({"content.wsplit_qk": f[2], "content.wsplit_v": f[3], "content.wsplit_out": f[4]})
                    name += f" (qk {f[2]:#x} v {f[3]:#x} out {f[4]:#x})"
                variants.append((name + " + split-fp16 DiffSVC head", 2, True, extra))
        for name, split, head, extra in variants:
            extra = dict(extra or {})
            operands = extra.pop("operands", "fp16")
            e = SVCEngine(cfg, 0, whisper_state=ws, mapper_state=ms, vocoder_state=vs, hubert_state=hs,
                          content_split=split, head_split=head, config=extra or None, operands=operands)
            d = lambda a, t=torch.float32: torch.as_tensor(np.ascontiguousarray(a)).to(t).cuda()  # noqa: E731
            noise = np.stack([ON.step_noise(seed, i, 1, T) for i in reversed(range(1000))])
            pipe = SVCPipeline(e)
            w16f = d(w16[None]) if hs is not None else None
            content = pipe.content(d(w16[None]), T, w16f).float().cpu().numpy()[0]
            res = pipe.convert(d(w24[None]), d(w16[None]), d(np.array([2]), torch.int32), fast_inference=False,
                               x_T=d(xT), noise=d(noise), f0=d(f0[None], torch.float64), wav16_float=w16f)
            _, mel_d = e.bigvgan(res.x0, return_mel=True)
            runs[name] = dict(content=content, x0=res.x0[0].cpu().numpy(), mel=mel_d[0].cpu().numpy(),
                              wav=res.wav[0].cpu().numpy())
            e.close()
    for name, r in runs.items():
        results[name] = {
            "mel_l1_denorm_ln": float(np.mean(np.abs(r["mel"] - ref["mel"]))),
            "mel_l1_normalised": float(np.mean(np.abs(r["x0"] - ref["x0"]))),
            "mel_l1_target_1e-3_met": bool(np.mean(np.abs(r["mel"] - ref["mel"])) <= 1e-3),
            "content_rel_l2": rel_l2(r["content"], ref["content"]),
            "wav_rel_l2": rel_l2(r["wav"], ref["wav"]) if voc else None,
        }
    enc = ("Whisper-" + args.whisper_dims) if hs is None else "ContentVec (layer 9)"
    print(json.dumps({"config": f"{enc} + DDPM-1000 + BigVGAN, seeded random weights, "
                                f"{args.seconds:g} s synthetic clip (T={T}), shared x_T and step noise; reference = "
                                "fp32 oracle", "cpu_seconds": timing, "results": results}, indent=1))


if __name__ == "__main__":
    main()
