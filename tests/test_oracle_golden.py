"""CPU: the oracle (CPU restatement) against golden vectors produced by the reference itself
(tools/make_goldens.py). These tests pin the oracle before it is trusted as the GPU checker."""
import numpy as np
import pytest
import torch

from oracle import features as OF
from oracle import models as OM
from oracle import noise as ON
from svc_inference_pipeline_amd import config as C
from svc_inference_pipeline_amd import weights as W


@pytest.fixture(scope="module")
def cfg():
    c = C.load_config()
    return c


@pytest.fixture(scope="module")
def mapper_sd(cfg):
    mcfg = C.load_config().mapper
    mcfg.input_content_dim["whisper"] = W.WHISPER_DIMS["tiny-test"]["n_audio_state"]
    return mcfg, W.make_mapper_state(mcfg, seed=0)


def test_mel_filterbank_kat(golden):
    kat = golden("mel_filters_kat")["mel_80"]
    assert np.array_equal(OF.slaney_mel_filterbank(16000, 400, 80), kat)


def test_mel24k_energy(golden, cfg):
    g = golden("mel24k")
    wav = torch.from_numpy(g["wav"]).unsqueeze(0)
    mel = OF.mel_spectrogram(wav, cfg)[0]
    assert mel.shape[-1] == OF.mel_frames(wav.shape[-1]) == g["mel"].shape[-1]
    np.testing.assert_allclose(mel.numpy(), g["mel"], rtol=0, atol=2e-5)
    en = OF.energy_from_mel(mel.unsqueeze(0))[0]
    np.testing.assert_allclose(en.numpy(), g["energy"], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("n,T", [(24000, 93), (240000, 937), (97197, 379), (4320000, 16875), (1024, 4), (768, 3)])
def test_mel_frame_count(n, T):
    assert OF.mel_frames(n) == T


def test_whisper_logmel(golden):
    g = golden("whisper_logmel")
    a = torch.from_numpy(OF.pad_or_trim(g["wav16"])).unsqueeze(0)
    lm = OF.whisper_log_mel(a)[0]
    np.testing.assert_allclose(lm.numpy(), g["logmel"], rtol=0, atol=1e-5)


def test_whisper_encoder_tiny(golden):
    g = golden("whisper_logmel")
    dims = W.WHISPER_DIMS["tiny-test"]
    sd = W.make_whisper_state(dims, seed=0)
    feats = OM.whisper_encoder(sd, torch.from_numpy(g["logmel"]).unsqueeze(0), dims["n_audio_head"])[0]
    ref = golden("whisper_encoder_tiny")["feats"]
    np.testing.assert_allclose(feats.numpy(), ref, rtol=0, atol=5e-4)
    assert np.abs(feats.numpy() - ref).mean() < 2e-5


def test_content_map_bit_exact(golden):
    g = golden("content_map")
    for tl in (1, 93, 379, 937, 2812, 3000):
        out = OF.map_whisper_features(g["raw"], tl)
        assert out.shape == g[f"T{tl}"].shape
        assert np.array_equal(out.astype(np.float32), g[f"T{tl}"].astype(np.float32)), tl


def test_pitch_shift_and_denorm(golden):
    g = golden("f0_denorm")
    stats = C.load_stats(C.load_config())
    assert abs(stats["target_f0_median"] - 223.2578) < 1e-3
    sh = OF.pitch_shift(g["f0"], stats["target_f0_median"])
    assert np.array_equal(sh, g["f0_shift"])
    den = OF.denormalize_mel_channel(g["x_norm"], stats["mel_min"], stats["mel_max"])
    assert np.array_equal(den.astype(np.float32), g["denorm"].astype(np.float32))


def test_conditioner_and_eps(golden, mapper_sd):
    mcfg, sd = mapper_sd
    g = golden("conditioner_diffsvc")
    cond = OM.conditioner(sd, torch.from_numpy(g["content"]).unsqueeze(0), torch.from_numpy(g["f0_shift"]).unsqueeze(0),
                          torch.from_numpy(g["energy"]).unsqueeze(0), torch.from_numpy(g["singer"].astype(np.int64)))
    np.testing.assert_allclose(cond.numpy(), g["cond"], rtol=0, atol=1e-5)
    table = W.step_embedding_table(1000)
    for t in (0, 500, 999):
        eps = OM.diffsvc_forward(sd, mcfg, torch.from_numpy(g["x_in"]), torch.from_numpy(g["cond"]), torch.tensor([t]), table)
        np.testing.assert_allclose(eps.numpy(), g[f"eps_t{t}"], rtol=0, atol=2e-5)


def _denoiser(sd, mcfg, cond):
    table = W.step_embedding_table(1000)
    return lambda x, t: OM.diffsvc_forward(sd, mcfg, x, cond, t, table)


def test_plms_samplers(golden, mapper_sd):
    mcfg, sd = mapper_sd
    g = golden("samplers")
    cond = torch.from_numpy(golden("conditioner_diffsvc")["cond"])
    consts = OM.schedule_constants(C.noise_schedule(mcfg))
    T = cond.shape[1]
    x4 = OM.sample_plms(_denoiser(sd, mcfg, cond), torch.from_numpy(g["x_T"]), 1, T, 1000, 250, consts)
    np.testing.assert_allclose(x4[0].numpy().T, g["plms4"], rtol=1e-4, atol=1e-3)
    x100 = OM.sample_plms(_denoiser(sd, mcfg, cond), torch.from_numpy(g["x_T"]), 1, T, 1000, 10, consts)
    ref = g["plms100"]
    # random weights make PLMS-100 grow (A12 in SURVEY.md); compare relative to the magnitude
    assert np.abs(x100[0].numpy().T - ref).max() <= 1e-4 * np.abs(ref).max()


def test_plms100_headline_shape(golden):
    """The oracle's PLMS-100 at the headline length (T = 937) against the reference's own svc_model_inference on the
    same seeded weights (eps head x 3), conditioning and x_T (tools/make_goldens_headline.py, utterance 0): max |d| <=
    1e-5 of max |x_0|, and the eps-induced part x_0 - x_0|eps=0 (the sampler run with a zero denoiser) within rel-L2
    1e-5."""
    import headline_golden as HG
    g = golden("plms100_headline")
    mcfg = C.load_config().mapper
    mcfg.input_content_dim["whisper"] = 1024
    sd = HG.headline_mapper_state(mcfg)
    consts = OM.schedule_constants(C.noise_schedule(mcfg))
    cond = torch.from_numpy(HG.headline_cond(0))
    table = W.step_embedding_table(1000)
    cache = {}
    den = lambda x, t: OM.diffsvc_forward(sd, mcfg, x, cond, t, table, cp_cache=cache)
    xT = torch.from_numpy(HG.headline_x_T(0))
    x = OM.sample_plms(den, xT, 1, HG.T, 1000, 10, consts)[0].numpy()
    x_triv = OM.sample_plms(lambda x, t: torch.zeros_like(x), xT, 1, HG.T, 1000, 10, consts)[0].numpy()
    ref = g["plms100_u0"]
    assert np.abs(x - ref).max() <= 1e-5 * np.abs(ref).max()
    d, r = (x - x_triv).ravel(), (ref - x_triv).ravel()
    assert np.linalg.norm(d - r) <= 1e-5 * np.linalg.norm(r), np.linalg.norm(d - r) / np.linalg.norm(r)


@pytest.mark.slow
def test_ddpm1000(golden, mapper_sd):
    mcfg, sd = mapper_sd
    g = golden("samplers")
    cond = torch.from_numpy(golden("conditioner_diffsvc")["cond"])
    consts = OM.schedule_constants(C.noise_schedule(mcfg))
    T = cond.shape[1]
    seed = int(g["seed"])
    noise = lambda i: torch.from_numpy(ON.step_noise(seed, i, 1, T))
    x = OM.sample_ddpm(_denoiser(sd, mcfg, cond), torch.from_numpy(g["x_T"]), 1, T, 1000, consts, noise)
    np.testing.assert_allclose(x[0].numpy().T, g["ddpm1000"], rtol=0, atol=1e-4)


def test_kaiser_and_activation(golden):
    g = golden("bigvgan")
    taps = W.kaiser_sinc_filter1d(0.25, 0.3, 12).numpy().ravel()
    assert np.array_equal(taps, g["kaiser"])
    vsd = W.make_vocoder_state(C.load_config().vocoder, seed=0)
    y = OM.activation1d(torch.from_numpy(g["act_x"]), torch.from_numpy(vsd["activation_post.act.alpha"]),
                        torch.from_numpy(vsd["activation_post.act.beta"]), torch.from_numpy(taps))
    np.testing.assert_allclose(y.numpy(), g["act_y"], rtol=0, atol=1e-6)


def test_bigvgan_and_synthesis(golden):
    g = golden("bigvgan")
    vcfg = C.load_config().vocoder
    vsd = W.make_vocoder_state(vcfg, seed=0)
    wav = OM.bigvgan_forward(vsd, vcfg, torch.from_numpy(g["mel"]).unsqueeze(0))
    np.testing.assert_allclose(wav.numpy(), g["wav"], rtol=0, atol=2e-5)
    syn = OF.synthesis_fade(wav[0, 0], g["mel"].shape[-1])
    np.testing.assert_allclose(syn.numpy(), g["synth"], rtol=0, atol=2e-5)


@pytest.mark.parametrize("variant", ["amp2_snake_log", "amp2_snake_lin", "amp1_snake_log"])
def test_bigvgan_variants(golden, variant):
    """F4: AMPBlock2 and Snake (log and linear scale), pinned to the reference's own Generator
    (tools/make_goldens_amp2.py)."""
    g = golden("bigvgan_variants")
    vcfg = W.vocoder_variant_cfg(C.load_config().vocoder, variant)
    vsd = W.make_vocoder_state(vcfg, seed=0)
    wav = OM.bigvgan_forward(vsd, vcfg, torch.from_numpy(g["mel"]).unsqueeze(0))
    np.testing.assert_allclose(wav.numpy(), g[variant], rtol=0, atol=2e-5)


def test_format_golden(golden):
    """Config 1 format (gen/1100000814_svcc_CDF1.wav): 24 kHz, 1200 + 379*256 + 1200 samples,
    peak -29491 = round(-0.9*32768), silent padding (utils/util.py:20-37)."""
    g = golden("format_golden")
    T = OF.mel_frames(int(round(int(g["in_len"]) * 24000 / int(g["in_sr"]))))
    assert T == 379
    assert int(g["out_len"]) == 1200 + 256 * T + 1200
    assert int(g["out_min"]) == -29491
    assert np.all(g["out_head"][:1200] == 0) and np.all(g["out_tail"][-1200:] == 0)
    w = np.linspace(-0.5, 0.2, 5000).astype(np.float32)
    pcm = OF.save_audio_pcm16(w, 24000)
    assert len(pcm) == 5000 + 2400 and pcm.min() == -29491


# ---------------------------------------------------------------------------- A8: HuBERT / ContentVec variant
def test_hubert_map_reference(golden):
    """utils/hubert.py:83-134 restated; fixtures from the reference's own function."""
    g = golden("hubert_map")
    for s, t in g["cases"]:
        out = OF.map_hubert_features(g[f"raw_{s}_{t}"], int(t))
        ref = g[f"out_{s}_{t}"]
        assert out.shape == ref.shape == (t, 24)
        assert np.array_equal(out, ref), (s, t)
    for s, t, exited in g["exits"]:
        assert exited == 1
        with pytest.raises(OF.MappingError):
            OF.map_hubert_features(np.zeros((int(s), 4), np.float32), int(t))


def test_hubert_encoder_tiny(golden):
    """oracle.models.hubert_content vs transformers.HubertModel (independent implementation of fairseq's
    HuBERT; fairseq itself is absent and unpinned — SURVEY.md §8c)."""
    g = golden("hubert_encoder_tiny")
    dims = W.HUBERT_DIMS["tiny-test"]
    sd = W.make_hubert_state(dims, seed=0)
    with torch.no_grad():
        feats = OM.hubert_content(sd, torch.from_numpy(g["wav16"]), dims["output_layer"])
    assert feats.shape[1] == W.hubert_frames(g["wav16"].shape[1])
    np.testing.assert_allclose(feats.numpy(), g["feats"], rtol=0, atol=1e-5)


def test_conditioner_multi_content(golden):
    """EncoderFramework with content_feature ["whisper", "contentvec"] and ["contentvec"] (reference fixtures)."""
    g = golden("conditioner_multi_content")
    for tag, types_ in (("multi", ["whisper", "contentvec"]), ("cv", ["contentvec"])):
        mcfg = C.load_config().mapper
        mcfg.content_feature = types_
        mcfg.input_content_dim["whisper"] = 128
        mcfg.input_content_dim["contentvec"] = 32
        sd = W.make_mapper_state(mcfg, seed=0)
        content = {ct: torch.from_numpy(g[f"content_{ct}"]) for ct in types_}
        cond = OM.conditioner(sd, content, torch.from_numpy(g["f0"]), torch.from_numpy(g["energy"]),
                              torch.from_numpy(g["singer"]).long())
        np.testing.assert_allclose(cond.numpy(), g[f"cond_{tag}"], rtol=0, atol=2e-5)
