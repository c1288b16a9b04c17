"""Generate the HuBERT/ContentVec-variant goldens (BASELINE config 5) in tests/golden/.

Build container only. What pins what:
  * hubert_map.npz      — the REFERENCE's own utils/hubert.py:get_mapped_features (imported with sys.modules
                          shims for fairseq/librosa, which it imports but this function never touches), over
                          source/target lengths that exercise exact fit, <=3-row padding, truncation and the
                          >3 exit() branch.
  * conditioner_multi_content.npz — the REFERENCE's modules/encoder.py EncoderFramework with
                          content_feature = ["whisper", "contentvec"] (both ContentEncoders summed) and with
                          ["contentvec"] alone.
  * hubert_encoder_tiny.npz — fairseq (which the reference loads ContentVec with, utils/hubert.py:14-28) is
                          not installed and the reference pins no version, so the encoder cannot be pinned to
                          the reference itself. The fixture comes from an independent implementation of the
                          same published model, transformers.HubertModel (installed here), with our
                          fairseq-named weights mapped onto it; oracle.models.hubert_content must match it.
Outputs are data only. Usage:  python tools/make_goldens_hubert.py
"""
import os
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_goldens import OUT, REF, install_shims, load_into  # noqa: E402
from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd import weights as W  # noqa: E402
from oracle import noise as ON  # noqa: E402


def hf_from_fairseq(sd, d):
    """transformers.HubertModel carrying the weights of a fairseq-named HuBERT state dict."""
    from transformers import HubertConfig, HubertModel
    c = HubertConfig(hidden_size=d["embed_dim"], num_hidden_layers=d["n_layer"], num_attention_heads=d["n_head"],
                     intermediate_size=d["ffn_dim"], conv_dim=(d["conv_dim"],) * 7, feat_extract_norm="group",
                     do_stable_layer_norm=False, conv_bias=False, num_conv_pos_embeddings=d["conv_pos"],
                     num_conv_pos_embedding_groups=d["conv_pos_groups"], hidden_act="gelu",
                     feat_proj_layer_norm=True, layer_norm_eps=1e-5)
    m = HubertModel(c).eval()
    hs = {}
    for i in range(7):
        hs[f"feature_extractor.conv_layers.{i}.conv.weight"] = sd[f"feature_extractor.conv_layers.{i}.0.weight"]
    hs["feature_extractor.conv_layers.0.layer_norm.weight"] = sd["feature_extractor.conv_layers.0.2.weight"]
    hs["feature_extractor.conv_layers.0.layer_norm.bias"] = sd["feature_extractor.conv_layers.0.2.bias"]
    hs["feature_projection.layer_norm.weight"] = sd["layer_norm.weight"]
    hs["feature_projection.layer_norm.bias"] = sd["layer_norm.bias"]
    hs["feature_projection.projection.weight"] = sd["post_extract_proj.weight"]
    hs["feature_projection.projection.bias"] = sd["post_extract_proj.bias"]
    hs["encoder.pos_conv_embed.conv.bias"] = sd["encoder.pos_conv.0.bias"]
    hs["encoder.pos_conv_embed.conv.parametrizations.weight.original0"] = sd["encoder.pos_conv.0.weight_g"]
    hs["encoder.pos_conv_embed.conv.parametrizations.weight.original1"] = sd["encoder.pos_conv.0.weight_v"]
    hs["encoder.layer_norm.weight"] = sd["encoder.layer_norm.weight"]
    hs["encoder.layer_norm.bias"] = sd["encoder.layer_norm.bias"]
    for i in range(d["n_layer"]):
        p = f"encoder.layers.{i}."
        for proj in ("q_proj", "k_proj", "v_proj", "out_proj"):
            for n in ("weight", "bias"):
                hs[p + f"attention.{proj}.{n}"] = sd[p + f"self_attn.{proj}.{n}"]
        for n in ("weight", "bias"):
            hs[p + f"layer_norm.{n}"] = sd[p + f"self_attn_layer_norm.{n}"]
            hs[p + f"feed_forward.intermediate_dense.{n}"] = sd[p + f"fc1.{n}"]
            hs[p + f"feed_forward.output_dense.{n}"] = sd[p + f"fc2.{n}"]
            hs[p + f"final_layer_norm.{n}"] = sd[p + f"final_layer_norm.{n}"]
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in hs.items()},
                                            strict=False)
    assert set(missing) <= {"masked_spec_embed"} and not unexpected, (missing, unexpected)
    return m


def main():
    import transformers  # noqa: F401  (before the shims: it probes torchaudio/librosa specs at import)
    from transformers import HubertConfig, HubertModel  # noqa: F401
    install_shims()
    sys.modules["fairseq"] = types.ModuleType("fairseq")
    sys.modules["fairseq"].checkpoint_utils = None
    sys.modules["tqdm"] = sys.modules.get("tqdm") or types.ModuleType("tqdm")
    sys.modules["tqdm"].tqdm = getattr(sys.modules["tqdm"], "tqdm", None)
    torch.set_num_threads(8)
    import contextlib
    import io
    from utils import hubert as RH  # noqa: E402

    # ---------------------------------------------------------------- A8 mapping (reference's own function)
    rng = np.random.default_rng(21)
    cases = [(499, 937), (499, 935), (499, 934), (499, 938), (49, 93), (10, 18), (1, 1), (3, 8), (37, 66)]
    maps = {}
    for s, t in cases:
        raw = rng.standard_normal((s, 24)).astype(np.float32)
        with contextlib.redirect_stdout(io.StringIO()):
            out = RH.get_mapped_features(raw, np.zeros((t, 100)))
        maps[f"raw_{s}_{t}"] = raw
        maps[f"out_{s}_{t}"] = out
    # the exit() branch: |target - mapped| > 3
    bad = []
    for s, t in [(499, 939), (499, 930), (49, 96)]:
        raw = rng.standard_normal((s, 4)).astype(np.float32)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                RH.get_mapped_features(raw, np.zeros((t, 100)))
            bad.append((s, t, 0))
        except SystemExit:
            bad.append((s, t, 1))
    np.savez_compressed(os.path.join(OUT, "hubert_map.npz"), cases=np.array(cases), exits=np.array(bad), **maps)
    print("hubert map", len(cases), "cases; exit branch", bad)

    # ---------------------------------------------------------------- A8 encoder (independent implementation)
    d = W.HUBERT_DIMS["tiny-test"]
    sd = W.make_hubert_state(d, seed=0)
    wav = np.stack([ON.synth_clip(3, 1.0, 16000), ON.synth_clip(4, 1.0, 16000)]).astype(np.float32)
    m = hf_from_fairseq(sd, d)
    with torch.no_grad():
        h = m(torch.from_numpy(wav), output_hidden_states=True).hidden_states[d["output_layer"]]
        feats = torch.nn.functional.linear(h, torch.from_numpy(sd["final_proj.weight"]),
                                           torch.from_numpy(sd["final_proj.bias"]))
    import transformers
    np.savez_compressed(os.path.join(OUT, "hubert_encoder_tiny.npz"), wav16=wav, feats=feats.numpy(),
                        source=np.array(f"transformers {transformers.__version__} HubertModel (fairseq stand-in)"))
    print("hubert encoder", feats.shape)

    # ---------------------------------------------------------------- A10 with ContentVec content (reference)
    from modules.encoder import EncoderFramework  # noqa: E402
    cfg = C.load_config(os.path.join(REF, "config/config.json"))
    out = {}
    T = 93
    f0 = ON.synth_f0(2, T)[None]
    energy = rng.uniform(0.0, 1.4, (1, T)).astype(np.float32)
    cw = rng.standard_normal((1, T, 128)).astype(np.float32)
    cv = rng.standard_normal((1, T, 32)).astype(np.float32)
    singer = np.array([[3]], dtype=np.int32)
    for tag, types_ in (("multi", ["whisper", "contentvec"]), ("cv", ["contentvec"])):
        mcfg = C.load_config(os.path.join(REF, "config/config.json")).mapper
        mcfg.content_feature = types_
        mcfg.input_content_dim = C.JsonHParams(**{"whisper": 128, "contentvec": 32})
        msd = W.make_mapper_state(mcfg, seed=0)
        enc = EncoderFramework(mcfg)
        load_into(enc, {k[len("0."):]: v for k, v in msd.items() if k.startswith("0.")})
        batch = {"content_whisper": torch.from_numpy(cw), "content_contentvec": torch.from_numpy(cv),
                 "melody": torch.from_numpy(f0), "loudness": torch.from_numpy(energy), "singer": torch.from_numpy(singer)}
        with torch.no_grad():
            out[f"cond_{tag}"] = enc(batch).numpy()
    np.savez_compressed(os.path.join(OUT, "conditioner_multi_content.npz"), f0=f0, energy=energy, content_whisper=cw,
                        content_contentvec=cv, singer=singer, **out)
    print("conditioner multi-content", out["cond_multi"].shape)


if __name__ == "__main__":
    main()
