"""Model parameters in the reference's own state_dict format.

No trained checkpoints exist offline (`/mnt/workspace/...` paths in config.json:7-10, Whisper
download at utils/whisper_extractor/__init__.py:26,103), so this module builds seeded random
parameters whose NAMES and SHAPES are exactly the reference's state_dict keys:

  mapper   : torch.nn.ModuleList([EncoderFramework, DiffSVC])   (utils/load_models.py:17-20)
  vocoder  : bigvgan.Generator                                   (modules/bigvgan.py:519-622)
  whisper  : Whisper.encoder (AudioEncoder)                      (utils/whisper_extractor/model.py:132-160)
  hubert   : fairseq HubertModel (ContentVec)                     (utils/hubert.py:14-47)

Random tensors come from numpy PCG64 keyed by (seed, crc32(name)), so any subset is reproducible
independently of generation order. Model BUFFERS the reference builds at construction time
(melody/energy bins, Kaiser-sinc filters, Whisper sinusoid positions, DiffSVC step table) are built
with torch-CPU float32 using the reference's own formulas, because that is how the reference
materialises them before `.cuda()` (they are then bit-identical).

`load_state_dict_checkpoint` is the loader for real checkpoints (utils/load_models.py:23-79) but,
unlike the reference, it fails loudly on missing/mismatched keys.
"""
import math
import zlib

import numpy as np
import torch

# ----------------------------------------------------------------------------- helpers


def _rng(seed, name):
    return np.random.Generator(np.random.PCG64([int(seed) & 0xFFFFFFFF, zlib.crc32(name.encode())]))


def _normal(seed, name, shape, std, mean=0.0):
    a = _rng(seed, name).standard_normal(size=shape, dtype=np.float32)
    a *= np.float32(std)
    if mean:
        a += np.float32(mean)
    return a


def _uniform(seed, name, shape, lo, hi):
    return _rng(seed, name).uniform(lo, hi, size=shape).astype(np.float32)


def note_to_hz(note):
    """librosa.note_to_hz for the two notes the reference uses (modules/encoder.py:38-39)."""
    midi = {"C1": 24, "C7": 96}[note]
    return float(440.0 * (2.0 ** ((midi - 69.0) / 12.0)))


# ----------------------------------------------------------------------------- buffers (torch-CPU f32)


def melody_bins(n_bins):
    """modules/encoder.py:47-57."""
    f0_min, f0_max = note_to_hz("C1"), note_to_hz("C7")
    return torch.exp(torch.linspace(np.log(f0_min - 0.1), np.log(f0_max), n_bins - 1))


def energy_bins(n_bins):
    """modules/encoder.py:89-102."""
    return torch.exp(torch.linspace(np.log(1e-30), np.log(1.5), n_bins - 1))


def step_embedding_table(max_steps):
    """modules/diffsvc.py:45-54 (StepEncoder.build_embedding)."""
    steps = torch.arange(max_steps).unsqueeze(1)
    dims = torch.arange(64).unsqueeze(0)
    table = steps * 10.0 ** (dims * 4.0 / 63.0)
    return torch.cat([torch.sin(table), torch.cos(table)], dim=1)


def kaiser_sinc_filter1d(cutoff, half_width, kernel_size):
    """modules/bigvgan.py:162-193 -> [1,1,kernel_size] f32."""
    even = kernel_size % 2 == 0
    half_size = kernel_size // 2
    delta_f = 4 * half_width
    A = 2.285 * (half_size - 1) * math.pi * delta_f + 7.95
    if A > 50.0:
        beta = 0.1102 * (A - 8.7)
    elif A >= 21.0:
        beta = 0.5842 * (A - 21) ** 0.4 + 0.07886 * (A - 21.0)
    else:
        beta = 0.0
    window = torch.kaiser_window(kernel_size, beta=beta, periodic=False)
    if even:
        time = torch.arange(-half_size, half_size) + 0.5
    else:
        time = torch.arange(kernel_size) - half_size
    filt = 2 * cutoff * window * torch.sinc(2 * cutoff * time)
    filt /= filt.sum()
    return filt.view(1, 1, kernel_size)


def sinusoids(length, channels, max_timescale=10000):
    """utils/whisper_extractor/model.py:48-54."""
    log_timescale_increment = np.log(max_timescale) / (channels // 2 - 1)
    inv_timescales = torch.exp(-log_timescale_increment * torch.arange(channels // 2))
    scaled_time = torch.arange(length)[:, np.newaxis] * inv_timescales[np.newaxis, :]
    return torch.cat([torch.sin(scaled_time), torch.cos(scaled_time)], dim=1)


def fade_out_table(n):
    """modules/bigvgan_inference.py:37-39: torch.linspace(1, 0, steps=n) (f32)."""
    return torch.linspace(1, 0, steps=n)


# ----------------------------------------------------------------------------- random parameter sets


def _conv(sd, seed, name, cout, cin, k, gain=1.0, bias_std=0.02):
    sd[name + ".weight"] = _normal(seed, name + ".weight", (cout, cin, k), gain / math.sqrt(cin * k))
    sd[name + ".bias"] = _normal(seed, name + ".bias", (cout,), bias_std)


def _linear(sd, seed, name, cout, cin, gain=1.0, bias=True, bias_std=0.02):
    sd[name + ".weight"] = _normal(seed, name + ".weight", (cout, cin), gain / math.sqrt(cin))
    if bias:
        sd[name + ".bias"] = _normal(seed, name + ".bias", (cout,), bias_std)


def make_mapper_state(mcfg, seed=0):
    """State dict of ModuleList([EncoderFramework, DiffSVC]) (utils/load_models.py:17-20;
    modules/encoder.py:138-163; modules/diffsvc.py:240-282). DiffSVC.output_projection is zero-
    initialised by the reference (diffsvc.py:282), which would make every epsilon prediction a
    constant; here it is random like every other layer."""
    sd = {}
    C = mcfg.residual_channels
    p = "0.registered_modules_dict."
    for ct in mcfg.content_feature:  # one ContentEncoder per content type (modules/encoder.py:144-148)
        _linear(sd, seed, p + f"content_{ct}.nn", mcfg.encoder_content_dim, mcfg.input_content_dim[ct])
    sd[p + "melody.melody_bins"] = melody_bins(mcfg.n_bins_melody).numpy()
    sd[p + "melody.nn.weight"] = _normal(seed, p + "melody.nn.weight", (mcfg.n_bins_melody, mcfg.encoder_melody_dim), 0.5)
    sd[p + "loudness.energy_bins"] = energy_bins(mcfg.n_bins_loudness).numpy()
    sd[p + "loudness.nn.weight"] = _normal(seed, p + "loudness.nn.weight", (mcfg.n_bins_loudness, mcfg.encoder_loudness_dim), 0.5)
    sd[p + "singer.nn.weight"] = _normal(seed, p + "singer.nn.weight", (mcfg.singer_table_size, mcfg.encoder_singer_dim), 0.5)
    q = "1."
    _conv(sd, seed, q + "mel_preprocess.projection", C, mcfg.n_mel, 1, gain=math.sqrt(2.0))
    _linear(sd, seed, q + "diffusion_embedding.projection1", mcfg.diffusion_fc_size, 128)
    _linear(sd, seed, q + "diffusion_embedding.projection2", mcfg.diffusion_fc_size, mcfg.diffusion_fc_size)
    for i in range(mcfg.residual_layer_num):
        r = q + f"residual_layers.{i}."
        _conv(sd, seed, r + "dilated_conv", 2 * C, C, mcfg.residual_kernel_size)
        _linear(sd, seed, r + "diffusion_projection", C, mcfg.diffusion_fc_size)
        _conv(sd, seed, r + "conditioner_projection", 2 * C, mcfg.conditioner_size, 1)
        _conv(sd, seed, r + "output_projection", 2 * C, C, 1)
    _conv(sd, seed, q + "skip_projection", C, C, 1, gain=math.sqrt(2.0))
    _conv(sd, seed, q + "output_projection", mcfg.n_mel, C, 1)
    return sd


def _wn_conv(sd, seed, name, w_shape, fan_in, bias_n):
    """weight_norm(Conv) params: weight_g [dim0,1,1], weight_v, bias (modules/bigvgan.py:529-593)."""
    v = _normal(seed, name + ".weight_v", w_shape, 1.0 / math.sqrt(fan_in))
    norm = np.sqrt((v.astype(np.float64) ** 2).reshape(w_shape[0], -1).sum(1)).astype(np.float32)
    g = norm * _uniform(seed, name + ".weight_g", (w_shape[0],), 0.8, 1.2)
    sd[name + ".weight_v"] = v
    sd[name + ".weight_g"] = g.reshape(w_shape[0], 1, 1)
    sd[name + ".bias"] = _normal(seed, name + ".bias", (bias_n,), 0.02)


def _act(sd, seed, name, ch, kind="snakebeta", logscale=True):
    """Activation1d params (modules/bigvgan.py:234-307): SnakeBeta has alpha and beta, Snake (:42-92) alpha only;
    log-scale parameters are drawn around 0, linear-scale ones around 1 (the reference's initialisations)."""
    f = kaiser_sinc_filter1d(0.25, 0.3, 12).numpy()
    mean = 0.0 if logscale else 1.0
    sd[name + ".act.alpha"] = _normal(seed, name + ".act.alpha", (ch,), 0.3 if logscale else 0.1, mean=mean)
    if kind == "snakebeta":
        sd[name + ".act.beta"] = _normal(seed, name + ".act.beta", (ch,), 0.3 if logscale else 0.1, mean=mean)
    sd[name + ".upsample.filter"] = f.copy()
    sd[name + ".downsample.lowpass.filter"] = f.copy()


# BigVGAN configurations infer.py does not use but the config can select: AMPBlock2
# (modules/bigvgan.py:442-516, dilations (1, 3)) and Snake (:42-92) in log or linear scale
VOCODER_VARIANTS = {
    "amp2_snake_log": dict(resblock="2", activation="snake", snake_logscale=True, dil=[[1, 3], [1, 3], [1, 3]]),
    "amp2_snake_lin": dict(resblock="2", activation="snake", snake_logscale=False, dil=[[1, 3], [1, 3], [1, 3]]),
    "amp1_snake_log": dict(resblock="1", activation="snake", snake_logscale=True, dil=None),
}


def vocoder_variant_cfg(vcfg, name):
    """A copy of the vocoder config with one of VOCODER_VARIANTS applied."""
    import copy
    v = VOCODER_VARIANTS[name]
    c = copy.deepcopy(vcfg)
    c.resblock = v["resblock"]
    c.activation = v["activation"]
    c.snake_logscale = v["snake_logscale"]
    if v["dil"] is not None:
        c.resblock_dilation_sizes = [list(d) for d in v["dil"]]
    return c


def make_vocoder_state(vcfg, seed=0):
    """State dict of bigvgan.Generator (modules/bigvgan.py:519-598): AMPBlock1 (convs1 / convs2, :336-440) or
    AMPBlock2 (convs, :442-516), SnakeBeta or Snake activations (log or linear scale)."""
    assert vcfg.resblock in ("1", "2") and vcfg.activation in ("snake", "snakebeta")
    kind, logscale = vcfg.activation, bool(vcfg.snake_logscale)
    sd = {}
    C0 = vcfg.upsample_initial_channel
    _wn_conv(sd, seed, "conv_pre", (C0, vcfg.input_dim, 7), vcfg.input_dim * 7, C0)
    nk = len(vcfg.resblock_kernel_sizes)
    for i, (u, k) in enumerate(zip(vcfg.upsample_rates, vcfg.upsample_kernel_sizes)):
        cin, cout = C0 // (2 ** i), C0 // (2 ** (i + 1))
        _wn_conv(sd, seed, f"ups.{i}.0", (cin, cout, k), cin * k // u, cout)
    for i in range(len(vcfg.upsample_rates)):
        ch = C0 // (2 ** (i + 1))
        for j, (k, d) in enumerate(zip(vcfg.resblock_kernel_sizes, vcfg.resblock_dilation_sizes)):
            rb = f"resblocks.{i * nk + j}."
            if vcfg.resblock == "1":
                for l in range(len(d)):
                    _wn_conv(sd, seed, rb + f"convs1.{l}", (ch, ch, k), ch * k, ch)
                    _wn_conv(sd, seed, rb + f"convs2.{l}", (ch, ch, k), ch * k, ch)
                n_act = 2 * len(d)
            else:
                for l in range(len(d)):
                    _wn_conv(sd, seed, rb + f"convs.{l}", (ch, ch, k), ch * k, ch)
                n_act = len(d)
            for a in range(n_act):
                _act(sd, seed, rb + f"activations.{a}", ch, kind, logscale)
    ch = C0 // (2 ** len(vcfg.upsample_rates))
    _act(sd, seed, "activation_post", ch, kind, logscale)
    _wn_conv(sd, seed, "conv_post", (1, ch, 7), ch * 7, 1)
    return sd


WHISPER_DIMS = {
    # utils/whisper_extractor/__init__.py:18-30 model table; medium = n_audio_state 1024, 16 heads, 24 layers
    "medium": dict(n_mels=80, n_audio_ctx=1500, n_audio_state=1024, n_audio_head=16, n_audio_layer=24),
    "tiny-test": dict(n_mels=80, n_audio_ctx=1500, n_audio_state=128, n_audio_head=2, n_audio_layer=2),
}


def make_whisper_state(dims, seed=0):
    """State dict of AudioEncoder with the 'encoder.' prefix Whisper uses
    (utils/whisper_extractor/model.py:132-142, 104-116)."""
    sd = {}
    D, L = dims["n_audio_state"], dims["n_audio_layer"]
    p = "encoder."
    _conv(sd, seed, p + "conv1", D, dims["n_mels"], 3)
    _conv(sd, seed, p + "conv2", D, D, 3)
    sd[p + "positional_embedding"] = sinusoids(dims["n_audio_ctx"], D).numpy()
    for i in range(L):
        b = p + f"blocks.{i}."
        _linear(sd, seed, b + "attn.query", D, D)
        _linear(sd, seed, b + "attn.key", D, D, bias=False)
        _linear(sd, seed, b + "attn.value", D, D)
        _linear(sd, seed, b + "attn.out", D, D, gain=0.5)
        for ln in ("attn_ln", "mlp_ln"):
            sd[b + ln + ".weight"] = _normal(seed, b + ln + ".weight", (D,), 0.05, mean=1.0)
            sd[b + ln + ".bias"] = _normal(seed, b + ln + ".bias", (D,), 0.02)
        _linear(sd, seed, b + "mlp.0", 4 * D, D)
        _linear(sd, seed, b + "mlp.2", D, 4 * D, gain=0.5)
    sd[p + "ln_post.weight"] = _normal(seed, p + "ln_post.weight", (D,), 0.05, mean=1.0)
    sd[p + "ln_post.bias"] = _normal(seed, p + "ln_post.bias", (D,), 0.02)
    return sd


def whisper_dims_from_state(sd):
    D = sd["encoder.conv1.weight"].shape[0]
    n_layer = 1 + max(int(k.split(".")[2]) for k in sd if k.startswith("encoder.blocks."))
    return dict(n_mels=sd["encoder.conv1.weight"].shape[1], n_audio_ctx=sd["encoder.positional_embedding"].shape[0],
                n_audio_state=D, n_audio_head=D // 64, n_audio_layer=n_layer)


HUBERT_DIMS = {
    # fairseq HubertModel as ContentVec ships it (utils/hubert.py:14-28 loads it through
    # fairseq.checkpoint_utils): conv extractor [(512,10,5)] + [(512,3,2)]*4 + [(512,2,2)]*2, 768-wide
    # post-LN transformer (12 heads, FFN 3072), conv_pos 128 / 16 groups, final_proj 768 -> 256.
    # utils/hubert.py:42 reads output_layer=9, so only layers 0..8 are evaluated.
    "contentvec": dict(conv_dim=512, embed_dim=768, n_head=12, ffn_dim=3072, n_layer=12, final_dim=256,
                       conv_pos=128, conv_pos_groups=16, output_layer=9),
    "tiny-test": dict(conv_dim=64, embed_dim=128, n_head=2, ffn_dim=256, n_layer=3, final_dim=32,
                      conv_pos=128, conv_pos_groups=16, output_layer=2),
}
HUBERT_CONV_LAYERS = [(10, 5)] + [(3, 2)] * 4 + [(2, 2)] * 2  # (kernel, stride) of the feature extractor


def make_hubert_state(dims, seed=0):
    """State dict of a fairseq HubertModel (ContentVec) with fairseq's own key names:
    feature_extractor.conv_layers.{i}.0.weight (bias-free convs; layer 0 adds Fp32GroupNorm at .2),
    layer_norm, post_extract_proj, encoder.pos_conv.0.{weight_g,weight_v,bias} (weight_norm over dim 2),
    encoder.layer_norm, encoder.layers.{i}.{self_attn.{q,k,v,out}_proj, self_attn_layer_norm, fc1, fc2,
    final_layer_norm}, final_proj. fairseq is not installed; names follow its published modules
    (fairseq/models/wav2vec/wav2vec2.py ConvFeatureExtractionModel / TransformerEncoder,
    fairseq/models/hubert/hubert.py HubertModel)."""
    sd = {}
    Cc, D, Fd = dims["conv_dim"], dims["embed_dim"], dims["ffn_dim"]
    cin = 1
    for i, (k, _s) in enumerate(HUBERT_CONV_LAYERS):
        name = f"feature_extractor.conv_layers.{i}.0.weight"
        sd[name] = _normal(seed, name, (Cc, cin, k), math.sqrt(2.0 / (cin * k)))
        cin = Cc
    for n in ("weight", "bias"):
        name = f"feature_extractor.conv_layers.0.2.{n}"
        sd[name] = _normal(seed, name, (Cc,), 0.05 if n == "weight" else 0.02, mean=1.0 if n == "weight" else 0.0)
    sd["layer_norm.weight"] = _normal(seed, "layer_norm.weight", (Cc,), 0.05, mean=1.0)
    sd["layer_norm.bias"] = _normal(seed, "layer_norm.bias", (Cc,), 0.02)
    _linear(sd, seed, "post_extract_proj", D, Cc)
    kp, G = dims["conv_pos"], dims["conv_pos_groups"]
    v = _normal(seed, "encoder.pos_conv.0.weight_v", (D, D // G, kp), math.sqrt(4.0 / (kp * D)))
    sd["encoder.pos_conv.0.weight_v"] = v
    # weight_norm(dim=2): g has shape [1, 1, k]; start from ||v|| over dims (0, 1) scaled like a trained model
    norm = np.sqrt((v.astype(np.float64) ** 2).sum(axis=(0, 1), keepdims=True))
    sd["encoder.pos_conv.0.weight_g"] = (norm * _uniform(seed, "encoder.pos_conv.0.weight_g", (1, 1, kp), 0.5, 1.5)).astype(np.float32)
    sd["encoder.pos_conv.0.bias"] = _normal(seed, "encoder.pos_conv.0.bias", (D,), 0.02)
    sd["encoder.layer_norm.weight"] = _normal(seed, "encoder.layer_norm.weight", (D,), 0.05, mean=1.0)
    sd["encoder.layer_norm.bias"] = _normal(seed, "encoder.layer_norm.bias", (D,), 0.02)
    for i in range(dims["n_layer"]):
        p = f"encoder.layers.{i}."
        for proj in ("q_proj", "k_proj", "v_proj"):
            _linear(sd, seed, p + "self_attn." + proj, D, D)
        _linear(sd, seed, p + "self_attn.out_proj", D, D, gain=0.5)
        for ln in ("self_attn_layer_norm", "final_layer_norm"):
            sd[p + ln + ".weight"] = _normal(seed, p + ln + ".weight", (D,), 0.05, mean=1.0)
            sd[p + ln + ".bias"] = _normal(seed, p + ln + ".bias", (D,), 0.02)
        _linear(sd, seed, p + "fc1", Fd, D)
        _linear(sd, seed, p + "fc2", D, Fd, gain=0.5)
    _linear(sd, seed, "final_proj", dims["final_dim"], D)
    return sd


def hubert_dims_from_state(sd, output_layer=9):
    Cc = sd["feature_extractor.conv_layers.0.0.weight"].shape[0]
    D = sd["post_extract_proj.weight"].shape[0]
    n_layer = 1 + max(int(k.split(".")[2]) for k in sd if k.startswith("encoder.layers."))
    kp = sd["encoder.pos_conv.0.weight_v"].shape[2]
    return dict(conv_dim=Cc, embed_dim=D, n_head=D // 64, ffn_dim=sd["encoder.layers.0.fc1.weight"].shape[0],
                n_layer=n_layer, final_dim=sd["final_proj.weight"].shape[0], conv_pos=kp,
                conv_pos_groups=D // sd["encoder.pos_conv.0.weight_v"].shape[1], output_layer=min(output_layer, n_layer))


def hubert_frames(n_samples):
    """Frames of the conv feature extractor for n 16 kHz samples (499 for 10 s)."""
    t = n_samples
    for k, s in HUBERT_CONV_LAYERS:
        t = (t - k) // s + 1
    return t


# ----------------------------------------------------------------------------- real checkpoints (F2)


def load_state_dict_checkpoint(path, key, expected):
    """utils/load_models.py:23-79 semantics (strip 'module.'), but every expected key must be present
    with the expected shape, or ValueError is raised (the reference silently keeps random init)."""
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    sd = ckpt[key] if key else ckpt
    sd = {k.split("module.")[-1]: v for k, v in sd.items()}
    missing = [k for k in expected if k not in sd]
    bad = [k for k in expected if k in sd and tuple(sd[k].shape) != tuple(expected[k].shape)]
    if missing or bad:
        raise ValueError(f"checkpoint {path}: missing {missing[:5]}..., shape-mismatch {bad[:5]}...")
    return {k: sd[k].float().numpy() for k in expected}


def _tensor_dict(sd, strip_module=True, prefix=None):
    out = {}
    for k, v in sd.items():
        if strip_module:
            k = k.split("module.")[-1]
        if prefix is not None and not k.startswith(prefix):
            continue
        if torch.is_tensor(v):
            out[k] = v.detach().float().cpu().numpy()
    return out


def load_checkpoints(mapper_path=None, vocoder_path=None, whisper_path=None):
    """The reference's three checkpoint formats -> {"mapper"|"vocoder"|"whisper": state dict of f32 arrays}.

    mapper  utils/load_models.py:23-49   ckpt["state_dict"], keys of ModuleList([EncoderFramework, DiffSVC])
    vocoder utils/load_models.py:52-79   ckpt["generator_state_dict"], keys of Generator
    whisper utils/whisper_extractor/__init__.py:72-120  {"dims", "model_state_dict"}; the encoder half is kept
    "module." prefixes are stripped as the reference does. Loading is weights_only (no unpickling of code).
    Unlike the reference, which keeps random init for missing or mis-shaped keys, SVCEngine's native
    finalize rejects them (svc_ctx_finalize)."""
    out = {}
    if mapper_path:
        ckpt = torch.load(mapper_path, map_location="cpu", weights_only=True)
        out["mapper"] = _tensor_dict(ckpt["state_dict"])
    if vocoder_path:
        ckpt = torch.load(vocoder_path, map_location="cpu", weights_only=True)
        out["vocoder"] = _tensor_dict(ckpt["generator_state_dict"])
    if whisper_path:
        ckpt = torch.load(whisper_path, map_location="cpu", weights_only=True)
        out["whisper"] = _tensor_dict(ckpt["model_state_dict"], strip_module=False, prefix="encoder.")
        dims = ckpt.get("dims", {})
        got = whisper_dims_from_state(out["whisper"])
        for k in ("n_mels", "n_audio_ctx", "n_audio_state", "n_audio_head", "n_audio_layer"):
            if k in dims and int(dims[k]) != int(got[k]):
                raise ValueError(f"whisper checkpoint {whisper_path}: dims[{k}]={dims[k]} but weights give {got[k]}")
    return out


def save_checkpoints(dirname, mapper_state=None, vocoder_state=None, whisper_state=None, module_prefix=False):
    """Write states in the reference's checkpoint formats (tests and tools; the inverse of load_checkpoints)."""
    import os
    os.makedirs(dirname, exist_ok=True)
    pre = "module." if module_prefix else ""
    paths = {}
    if mapper_state is not None:
        paths["mapper"] = os.path.join(dirname, "mapper.pt")
        torch.save({"state_dict": {pre + k: torch.from_numpy(np.asarray(v)) for k, v in mapper_state.items()}},
                   paths["mapper"])
    if vocoder_state is not None:
        paths["vocoder"] = os.path.join(dirname, "vocoder.pt")
        torch.save({"generator_state_dict": {pre + k: torch.from_numpy(np.asarray(v)) for k, v in vocoder_state.items()}},
                   paths["vocoder"])
    if whisper_state is not None:
        paths["whisper"] = os.path.join(dirname, "whisper.pt")
        torch.save({"dims": whisper_dims_from_state(whisper_state),
                    "model_state_dict": {k: torch.from_numpy(np.asarray(v)) for k, v in whisper_state.items()}},
                   paths["whisper"])
    return paths

