"""ORACLE (test infrastructure only) — network restatement in torch-CPU float32 (functional form).

Rows A6 (Whisper encoder), A8 (HuBERT/ContentVec variant), A10 (conditioner), A11 (DiffSVC), A12 (samplers), A14 (BigVGAN) of
SURVEY.md §8(a). Parameters are dicts in the reference's state_dict naming (see
svc_inference_pipeline_amd/weights.py); values may be numpy or torch.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


def _t(sd, k):
    v = sd[k]
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v))


# ============================================================================ Whisper AudioEncoder


def whisper_encoder(sd, mel, n_head):
    """utils/whisper_extractor/model.py:132-160 (AudioEncoder.forward) with
    MultiHeadAttention.qkv_attention :88-101 and ResidualAttentionBlock :104-129. mel f32[B,80,3000]."""
    x = F.gelu(F.conv1d(mel, _t(sd, "encoder.conv1.weight"), _t(sd, "encoder.conv1.bias"), padding=1))
    x = F.gelu(F.conv1d(x, _t(sd, "encoder.conv2.weight"), _t(sd, "encoder.conv2.bias"), stride=2, padding=1))
    x = x.permute(0, 2, 1)
    x = x + _t(sd, "encoder.positional_embedding")
    i = 0
    while f"encoder.blocks.{i}.attn.query.weight" in sd:
        p = f"encoder.blocks.{i}."
        h = F.layer_norm(x, (x.shape[-1],), _t(sd, p + "attn_ln.weight"), _t(sd, p + "attn_ln.bias"))
        q = F.linear(h, _t(sd, p + "attn.query.weight"), _t(sd, p + "attn.query.bias"))
        k = F.linear(h, _t(sd, p + "attn.key.weight"))
        v = F.linear(h, _t(sd, p + "attn.value.weight"), _t(sd, p + "attn.value.bias"))
        nb, nc, ns = q.shape
        scale = (ns // n_head) ** -0.25
        q = q.view(nb, nc, n_head, -1).permute(0, 2, 1, 3) * scale
        k = k.view(nb, nc, n_head, -1).permute(0, 2, 3, 1) * scale
        v = v.view(nb, nc, n_head, -1).permute(0, 2, 1, 3)
        w = F.softmax((q @ k).float(), dim=-1)
        wv = (w @ v).permute(0, 2, 1, 3).flatten(start_dim=2)
        x = x + F.linear(wv, _t(sd, p + "attn.out.weight"), _t(sd, p + "attn.out.bias"))
        h = F.layer_norm(x, (x.shape[-1],), _t(sd, p + "mlp_ln.weight"), _t(sd, p + "mlp_ln.bias"))
        h = F.gelu(F.linear(h, _t(sd, p + "mlp.0.weight"), _t(sd, p + "mlp.0.bias")))
        x = x + F.linear(h, _t(sd, p + "mlp.2.weight"), _t(sd, p + "mlp.2.bias"))
        i += 1
    return F.layer_norm(x, (x.shape[-1],), _t(sd, "encoder.ln_post.weight"), _t(sd, "encoder.ln_post.bias"))


# ============================================================================ HuBERT / ContentVec (variant, A8)


def hubert_content(sd, wav16, output_layer=9):
    """utils/hubert.py:31-47 (get_hubert_content): fairseq HubertModel.extract_features(source,
    padding_mask=all-False, output_layer=9) then final_proj, returned here time-major [B, frames, final_dim].

    fairseq is not installed and the reference pins no version; this restates its
    published modules (fairseq/models/wav2vec/wav2vec2.py ConvFeatureExtractionModel mode "default",
    TransformerEncoder + TransformerSentenceEncoderLayer with layer_norm_first=False;
    fairseq/models/hubert/hubert.py HubertModel.forward_features / forward(features_only=True)):
      conv_layers[0]: conv(1->C, k10 s5, no bias) -> Fp32GroupNorm(C, C) (per channel over time, eps 1e-5) -> GELU
      conv_layers[1..6]: conv(k3/k2, s2, no bias) -> GELU
      LayerNorm(C) -> post_extract_proj (C -> D)
      x += GELU(SamePad(weight_norm(dim=2) grouped conv k=128, pad 64)(x)); LayerNorm(D)
      layers 0..output_layer-1, post-LN: x = LN(x + MHA(x)); x = LN(x + fc2(GELU(fc1(x))))
      q = (x Wq + bq) * dh^-1/2, softmax in f32.
    Padding masks are all False (utils/hubert.py:37) so they drop out. wav16 f32 [B, N]."""
    x = wav16.unsqueeze(1)
    i = 0
    while f"feature_extractor.conv_layers.{i}.0.weight" in sd:
        w = _t(sd, f"feature_extractor.conv_layers.{i}.0.weight")
        stride = 5 if i == 0 else 2
        x = F.conv1d(x, w, stride=stride)
        if i == 0:
            x = F.group_norm(x, x.shape[1], _t(sd, "feature_extractor.conv_layers.0.2.weight"),
                             _t(sd, "feature_extractor.conv_layers.0.2.bias"), eps=1e-5)
        x = F.gelu(x)
        i += 1
    x = x.transpose(1, 2)
    x = F.layer_norm(x, (x.shape[-1],), _t(sd, "layer_norm.weight"), _t(sd, "layer_norm.bias"))
    x = F.linear(x, _t(sd, "post_extract_proj.weight"), _t(sd, "post_extract_proj.bias"))
    # weight_norm(name="weight", dim=2): w = g * v / ||v|| with the norm over dims (0, 1) per tap
    v = _t(sd, "encoder.pos_conv.0.weight_v")
    g = _t(sd, "encoder.pos_conv.0.weight_g")
    w = g * v / torch.sqrt((v * v).sum(dim=(0, 1), keepdim=True))
    kp = v.shape[2]
    groups = x.shape[-1] // v.shape[1]
    xc = F.conv1d(x.transpose(1, 2), w, _t(sd, "encoder.pos_conv.0.bias"), padding=kp // 2, groups=groups)
    if kp % 2 == 0:
        xc = xc[:, :, :-1]  # SamePad
    x = x + F.gelu(xc).transpose(1, 2)
    D = x.shape[-1]
    x = F.layer_norm(x, (D,), _t(sd, "encoder.layer_norm.weight"), _t(sd, "encoder.layer_norm.bias"))
    H = D // 64
    n_layers = 1 + max(int(k.split(".")[2]) for k in sd if k.startswith("encoder.layers."))
    for li in range(min(output_layer, n_layers)):  # fairseq runs every layer when output_layer exceeds them
        p = f"encoder.layers.{li}."
        B, L, _ = x.shape
        q = F.linear(x, _t(sd, p + "self_attn.q_proj.weight"), _t(sd, p + "self_attn.q_proj.bias")) * (64 ** -0.5)
        k = F.linear(x, _t(sd, p + "self_attn.k_proj.weight"), _t(sd, p + "self_attn.k_proj.bias"))
        vv = F.linear(x, _t(sd, p + "self_attn.v_proj.weight"), _t(sd, p + "self_attn.v_proj.bias"))
        q = q.view(B, L, H, 64).transpose(1, 2)
        k = k.view(B, L, H, 64).transpose(1, 2)
        vv = vv.view(B, L, H, 64).transpose(1, 2)
        a = F.softmax((q @ k.transpose(-1, -2)).float(), dim=-1)
        o = (a @ vv).transpose(1, 2).reshape(B, L, D)
        x = x + F.linear(o, _t(sd, p + "self_attn.out_proj.weight"), _t(sd, p + "self_attn.out_proj.bias"))
        x = F.layer_norm(x, (D,), _t(sd, p + "self_attn_layer_norm.weight"), _t(sd, p + "self_attn_layer_norm.bias"))
        h = F.gelu(F.linear(x, _t(sd, p + "fc1.weight"), _t(sd, p + "fc1.bias")))
        x = x + F.linear(h, _t(sd, p + "fc2.weight"), _t(sd, p + "fc2.bias"))
        x = F.layer_norm(x, (D,), _t(sd, p + "final_layer_norm.weight"), _t(sd, p + "final_layer_norm.bias"))
    return F.linear(x, _t(sd, "final_proj.weight"), _t(sd, "final_proj.bias"))


# ============================================================================ conditioner


def bucketize_indices(values, bins):
    """torch.bucketize(x, bins) (right=False) as in modules/encoder.py:70,115: count of bins < x."""
    return torch.bucketize(values, bins)


def conditioner(sd, content, f0, energy, singer, content_type="whisper"):
    """modules/encoder.py:165-201, merge_mode "add". content f32[B,T,D], f0 f64[B,T], energy f32[B,T],
    singer int[B,1]. Summation order: content, melody, loudness, singer (ModuleDict order)."""
    p = "0.registered_modules_dict."
    if not isinstance(content, dict):  # one content type; a dict {type: f32[B,T,D_type]} sums several
        content = {content_type: content}
    cs = [F.linear(x, _t(sd, p + f"content_{ct}.nn.weight"), _t(sd, p + f"content_{ct}.nn.bias"))
          for ct, x in content.items()]
    m = F.embedding(torch.bucketize(f0, _t(sd, p + "melody.melody_bins")), _t(sd, p + "melody.nn.weight"))
    l = F.embedding(torch.bucketize(energy, _t(sd, p + "loudness.energy_bins")), _t(sd, p + "loudness.nn.weight"))
    s = F.embedding(singer, _t(sd, p + "singer.nn.weight")).expand(-1, cs[0].shape[1], -1)
    return torch.sum(torch.cat([o[None] for o in (*cs, m, l, s)], dim=0), dim=0)


# ============================================================================ DiffSVC epsilon predictor


def diffsvc_forward(sd, mcfg, x, cond, t, step_table, cp_cache=None):
    """modules/diffsvc.py:284-321 (+ StepEncoder :67-94, ResidualBlock :192-232, Preprocessor :111-125).
    x f32[B,T,100], cond f32[B,T,384], t int64[B] -> eps f32[B,T,100]. cp_cache (a dict, optional, one per cond):
    the conditioner projections of cond computed once and reused by later calls on the same cond; they do not
    depend on x or t, so the result is bit-identical (a sampler's 1000 calls run ~20 % faster)."""
    q = "1."
    h = F.relu(F.conv1d(x.transpose(1, 2), _t(sd, q + "mel_preprocess.projection.weight"), _t(sd, q + "mel_preprocess.projection.bias")))
    e = step_table[t.unsqueeze(1)]  # [B,1,128]
    e = F.silu(F.linear(e, _t(sd, q + "diffusion_embedding.projection1.weight"), _t(sd, q + "diffusion_embedding.projection1.bias")))
    e = F.silu(F.linear(e, _t(sd, q + "diffusion_embedding.projection2.weight"), _t(sd, q + "diffusion_embedding.projection2.bias")))
    condT = cond.transpose(1, 2)
    skip = None
    n = mcfg.residual_layer_num
    for i in range(n):
        r = q + f"residual_layers.{i}."
        d = F.linear(e, _t(sd, r + "diffusion_projection.weight"), _t(sd, r + "diffusion_projection.bias"))
        y = h + d.transpose(1, 2)
        cp = cp_cache.get(i) if cp_cache is not None else None
        if cp is None:
            cp = F.conv1d(condT, _t(sd, r + "conditioner_projection.weight"), _t(sd, r + "conditioner_projection.bias"))
            if cp_cache is not None:
                cp_cache[i] = cp
        dil = 2 ** (i % mcfg.dilation_cycle_length)
        y = F.conv1d(y, _t(sd, r + "dilated_conv.weight"), _t(sd, r + "dilated_conv.bias"), padding=dil, dilation=dil) + cp
        gate, filt = torch.chunk(y, 2, dim=1)
        y = torch.sigmoid(gate) * torch.tanh(filt)
        y = F.conv1d(y, _t(sd, r + "output_projection.weight"), _t(sd, r + "output_projection.bias"))
        res, sk = torch.chunk(y, 2, dim=1)
        h = (h + res) / math.sqrt(2.0)
        skip = sk if skip is None else sk + skip
    h = skip / math.sqrt(n)
    h = F.relu(F.conv1d(h, _t(sd, q + "skip_projection.weight"), _t(sd, q + "skip_projection.bias")))
    h = F.conv1d(h, _t(sd, q + "output_projection.weight"), _t(sd, q + "output_projection.bias"))
    return h.transpose(1, 2)


# ============================================================================ samplers


def schedule_constants(betas):
    """modules/diffsvcrepo_inference.py:163-197: numpy f64 -> torch f32."""
    to = lambda a: torch.tensor(a, dtype=torch.float32)
    alphas = 1.0 - betas
    ac = np.cumprod(alphas, axis=0)
    ac_prev = np.append(1.0, ac[:-1])
    post_var = betas * (1.0 - ac_prev) / (1.0 - ac)
    return {
        "alphas_cumprod": to(ac),
        "sqrt_recip_alphas_cumprod": to(np.sqrt(1.0 / ac)),
        "sqrt_recipm1_alphas_cumprod": to(np.sqrt(1.0 / ac - 1)),
        "posterior_mean_coef1": to(betas * np.sqrt(ac_prev) / (1.0 - ac)),
        "posterior_mean_coef2": to((1.0 - ac_prev) * np.sqrt(alphas) / (1.0 - ac)),
        "posterior_log_variance_clipped": to(np.log(np.maximum(post_var, 1e-20))),
    }


def plms_x_pred(x, noise_t, t, interval, ac):
    """p_sample_plms.get_x_pred, modules/diffsvcrepo_inference.py:96-113 (x in [B,T,100] layout;
    the update is elementwise so the reference's [B,1,100,T] layout does not change values)."""
    a_t = ac[t].view(-1, 1, 1)
    a_prev = ac[torch.clamp(t - interval, min=0)].view(-1, 1, 1)
    a_t_sq, a_prev_sq = a_t.sqrt(), a_prev.sqrt()
    x_delta = (a_prev - a_t) * ((1 / (a_t_sq * (a_t_sq + a_prev_sq))) * x
                                - 1 / (a_t_sq * (((1 - a_prev) * a_t).sqrt() + ((1 - a_t) * a_prev).sqrt())) * noise_t)
    return x + x_delta


def sample_plms(denoise, x, B, T, steps, interval, consts):
    """modules/diffsvcrepo_inference.py:91-151,216-231 (fast_inference=True). `denoise(x, t)` returns
    the epsilon tensor (the reference's denoise_fn returns (eps, stats); A12 — the oracle takes [0]).
    x: x_T f32[B,T,100]. Returns x_0 f32[B,T,100]."""
    ac = consts["alphas_cumprod"]
    hist = []
    for i in reversed(range(0, steps, interval)):
        t = torch.full((B,), i, dtype=torch.long)
        eps = denoise(x, t)
        if len(hist) == 0:
            x_pred = plms_x_pred(x, eps, t, interval, ac)
            t_prev = torch.full((B,), max(i - interval, 0), dtype=torch.long)
            eps_prev = denoise(x_pred, t_prev)
            e = (eps + eps_prev) / 2
        elif len(hist) == 1:
            e = (3 * eps - hist[-1]) / 2
        elif len(hist) == 2:
            e = (23 * eps - 16 * hist[-1] + 5 * hist[-2]) / 12
        else:
            e = (55 * eps - 59 * hist[-1] + 37 * hist[-2] - 9 * hist[-3]) / 24
        x = plms_x_pred(x, e, t, interval, ac)
        hist.append(eps)
        hist = hist[-4:]
    return x


def ddpm_step(x, eps, t, z, consts):
    """p_sample / p_mean_variance / q_posterior (modules/diffsvcrepo_inference.py:36-88),
    clip_denoised=True. x, eps, z f32[B,T,100]; t python int (same for the whole batch)."""
    x_recon = consts["sqrt_recip_alphas_cumprod"][t] * x - consts["sqrt_recipm1_alphas_cumprod"][t] * eps
    x_recon = x_recon.clamp(-1.0, 1.0)
    mean = consts["posterior_mean_coef1"][t] * x_recon + consts["posterior_mean_coef2"][t] * x
    nonzero = 0.0 if t == 0 else 1.0
    return mean + nonzero * (0.5 * consts["posterior_log_variance_clipped"][t]).exp() * z


def sample_ddpm(denoise, x, B, T, steps, consts, noise_fn):
    """modules/diffsvcrepo_inference.py:233-235. noise_fn(i) -> z f32[B,T,100] for step i (the
    reference draws randn([B,1,100,T]) each step, t = 0 included; callers transpose to [B,T,100])."""
    for i in reversed(range(0, steps)):
        t = torch.full((B,), i, dtype=torch.long)
        eps = denoise(x, t)
        x = ddpm_step(x, eps, i, noise_fn(i), consts)
    return x


# ============================================================================ BigVGAN generator


def _wn(sd, name):
    """weight_norm fold, dim=0 (torch._weight_norm: v * g / ||v|| over all dims but 0)."""
    return torch._weight_norm(_t(sd, name + ".weight_v"), _t(sd, name + ".weight_g"), 0)


def activation1d(x, alpha_log, beta_log, filt, logscale=True):
    """modules/bigvgan.py:234-307 (Activation1d = UpSample1d(2,12) -> SnakeBeta -> DownSample1d(2,12)) with SnakeBeta
    :146-159; Snake (:42-92) is the same with beta = alpha. logscale=False: the parameters are alpha / beta themselves
    (`alpha_logscale=False`). x f32[B,C,T]."""
    C = x.shape[1]
    f = filt.view(1, 1, -1)
    # UpSample1d :277-287  (ratio 2, kernel 12: pad 5, pad_left 15, pad_right 15)
    xu = F.pad(x, (5, 5), mode="replicate")
    xu = 2 * F.conv_transpose1d(xu, f.expand(C, -1, -1), stride=2, groups=C)
    xu = xu[..., 15:-15]
    # SnakeBeta :146-159
    alpha = (torch.exp(alpha_log) if logscale else alpha_log).view(1, -1, 1)
    beta = (torch.exp(beta_log) if logscale else beta_log).view(1, -1, 1)
    xu = xu + (1.0 / (beta + 0.000000001)) * torch.pow(torch.sin(xu * alpha), 2)
    # DownSample1d -> LowPassFilter1d :224-231 (pad_left 5, pad_right 6, stride 2)
    xd = F.pad(xu, (5, 6), mode="replicate")
    return F.conv1d(xd, f.expand(C, -1, -1), stride=2, groups=C)


def _act(sd, name, x, logscale=True):
    """SnakeBeta when the state has `.act.beta`, else Snake (x + 1/(alpha+1e-9) sin^2(alpha x), :84-92)."""
    alpha = _t(sd, name + ".act.alpha")
    beta = _t(sd, name + ".act.beta") if name + ".act.beta" in sd else alpha
    return activation1d(x, alpha, beta, _t(sd, name + ".upsample.filter"), logscale)


def bigvgan_forward(sd, vcfg, mel):
    """modules/bigvgan.py:600-622 (Generator.forward) with AMPBlock1.forward :424-433 or AMPBlock2.forward :506-512
    (`resblock` "2": x = x + conv_d(act(x)) per dilation, one conv each). mel f32[B,100,T] -> f32[B,1,256T]."""
    ls = bool(getattr(vcfg, "snake_logscale", True))
    rb2 = str(getattr(vcfg, "resblock", "1")) == "2"
    x = F.conv1d(mel, _wn(sd, "conv_pre"), _t(sd, "conv_pre.bias"), padding=3)
    nk = len(vcfg.resblock_kernel_sizes)
    for i, (u, k) in enumerate(zip(vcfg.upsample_rates, vcfg.upsample_kernel_sizes)):
        x = F.conv_transpose1d(x, _wn(sd, f"ups.{i}.0"), _t(sd, f"ups.{i}.0.bias"), stride=u, padding=(k - u) // 2)
        xs = None
        for j, (kk, dd) in enumerate(zip(vcfg.resblock_kernel_sizes, vcfg.resblock_dilation_sizes)):
            rb = f"resblocks.{i * nk + j}."
            xr = x
            for l, d in enumerate(dd):
                if rb2:
                    xt = _act(sd, rb + f"activations.{l}", xr, ls)
                    xt = F.conv1d(xt, _wn(sd, rb + f"convs.{l}"), _t(sd, rb + f"convs.{l}.bias"), dilation=d,
                                  padding=(kk * d - d) // 2)
                    xr = xt + xr
                    continue
                xt = _act(sd, rb + f"activations.{2 * l}", xr, ls)
                xt = F.conv1d(xt, _wn(sd, rb + f"convs1.{l}"), _t(sd, rb + f"convs1.{l}.bias"), dilation=d, padding=(kk * d - d) // 2)
                if _STORE16[0]:  # (fp16 emulation only: the HIP path stores this intermediate as saturating f16)
                    xt = xt.clamp(-65504.0, 65504.0).half().float()
                xt = _act(sd, rb + f"activations.{2 * l + 1}", xt, ls)
                xt = F.conv1d(xt, _wn(sd, rb + f"convs2.{l}"), _t(sd, rb + f"convs2.{l}.bias"), padding=(kk - 1) // 2)
                xr = xt + xr
            xs = xr if xs is None else xs + xr
        x = xs / nk
    x = _act(sd, "activation_post", x, ls)
    x = F.conv1d(x, _wn(sd, "conv_post"), _t(sd, "conv_post.bias"), padding=3)
    return torch.tanh(x)


# ============================================================================ fp16-operand emulation
_STORE16 = [False]  # set inside Fp16Operands: BigVGAN's AMPBlock1 intermediate rounded to f16 as the HIP path stores it


class OperandRounding:
    """Context manager: dense convolutions (and, with `linear=True`, F.linear and the attention matmuls of
    the functional encoders) round their input and weight to `dtype` (float16 / bfloat16) and accumulate in
    fp32, emulating MFMA operand precision. Used to derive tolerances for chaotic random-weight regimes
    (tests/test_gpu_stages.py::test_bigvgan) and for the fp16-vs-bf16 sweep (tools/precision_sweep.py);
    depthwise (grouped) convs are untouched because the HIP path computes them in fp32."""

    def __init__(self, dtype=torch.float16, linear=False):
        self.dtype, self.linear = dtype, linear

    def __enter__(self):
        self._c, self._t, self._l, self._m = F.conv1d, F.conv_transpose1d, F.linear, torch.Tensor.__matmul__
        dt = self.dtype
        r = lambda t: t.to(dt).float()  # noqa: E731
        c, tr, li, mm = self._c, self._t, self._l, self._m

        def conv1d(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
            if groups > 1 and w.shape[1] == 1:
                return c(x, w, b, stride, padding, dilation, groups)
            return c(r(x), r(w), b, stride, padding, dilation, groups)

        def conv_t(x, w, b=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1):
            if groups > 1:
                return tr(x, w, b, stride, padding, output_padding, groups, dilation)
            return tr(r(x), r(w), b, stride, padding, output_padding, groups, dilation)

        F.conv1d, F.conv_transpose1d = conv1d, conv_t
        if self.linear:
            F.linear = lambda x, w, b=None: li(r(x), r(w), b)
            torch.Tensor.__matmul__ = lambda a, b: mm(r(a), r(b))
        return self

    def __exit__(self, *a):
        F.conv1d, F.conv_transpose1d, F.linear = self._c, self._t, self._l
        torch.Tensor.__matmul__ = self._m
        return False


class Fp16Operands(OperandRounding):
    """fp16 conv operands (the BigVGAN tolerance derivation), and the f16 storage of AMPBlock1's convs1 output that the
    HIP vocoder uses (engine.hip, round 3)."""

    def __init__(self, store16=True):
        super().__init__(torch.float16, linear=False)
        self.store16 = store16  # False: operand rounding only (the pre-round-3 emulation, tests/test_gpu_stages.py)

    def __enter__(self):
        self._prev_store16 = _STORE16[0]  # (nested / repeated contexts restore what they found)
        _STORE16[0] = self.store16
        return super().__enter__()

    def __exit__(self, *a):
        _STORE16[0] = self._prev_store16
        return super().__exit__(*a)
