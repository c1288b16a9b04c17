"""GPU parity, op level: every HIP kernel family against a torch-CPU fp32 reference of the same op.

Tolerances: MFMA operands are fp16 (inputs and weights rounded to binary16, fp32 accumulation), so
GEMM-shaped ops are checked with a relative L2 error <= 2e-3 (fp16 unit roundoff 4.9e-4, a few
roundings per output); element-wise f32 ops with fp16 outputs <= 1e-3; frame counts and index maps
bit-exact.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from gpu_util import call, dev, ptr, rel_l2, stream  # noqa: E402
from oracle import models as OM  # noqa: E402


def _tm(x):  # [B, C, T] -> time-major [B*T, C]
    return x.permute(0, 2, 1).contiguous()


# (gemm_variant, gemm3_direct kernel switches): every conv_gemm3 tile and conv_gemm4 with conv_gemm3's register
# epilogues (15 = every form), and the LDS-staged epilogue (0) on the tiles pick3 chooses in production
_GEMM_MODES = ([(v, "15") for v in ("10", "11", "12", "13", "14", "15", "16", "20", "24")] +
               [(v, "0") for v in ("10", "13", "14", "16")])


@pytest.mark.parametrize("B,T,Cin,Cout,k,stride,dil,pad,act", [
    (2, 93, 384, 768, 3, 1, 1, 1, 0),        # DiffSVC dilated conv, d=1
    (2, 93, 384, 768, 3, 1, 8, 8, 0),        # d=8
    (1, 200, 100, 384, 1, 1, 1, 0, 2),       # mel_preprocess (Cin not a multiple of 8/64), relu
    (2, 60, 80, 128, 3, 1, 1, 1, 1),         # whisper conv1 (gelu)
    (2, 60, 128, 128, 3, 2, 1, 1, 1),        # whisper conv2 (stride 2)
    (1, 37, 100, 1536, 7, 1, 1, 3, 0),       # conv_pre
    (2, 301, 24, 24, 11, 1, 5, 25, 0),       # last BigVGAN stage
    (1, 130, 48, 48, 7, 1, 3, 9, 0),
    (1, 70, 96, 96, 3, 1, 1, 1, 0),
    (3, 17, 384, 100, 1, 1, 1, 0, 0),        # output projection (N=100)
    (3, 700, 384, 768, 3, 1, 2, 2, 0),       # several M tiles + M tail (gemm3 tile shapes)
    (2, 333, 256, 512, 3, 1, 4, 4, 2),
    (2, 300, 384, 384, 11, 1, 5, 25, 0),     # BigVGAN stage 2 k=11 d=5
    (1, 150, 768, 768, 7, 1, 3, 9, 0),       # BigVGAN stage 1 k=7 d=3
    (3, 129, 192, 192, 11, 1, 3, 15, 0),     # utterance boundaries inside tiles
    (1, 90, 128, 256, 7, 1, 7, 21, 0),       # |shift| 21, T < tile
])
@pytest.mark.parametrize("variant,direct", _GEMM_MODES)
def test_conv1d(B, T, Cin, Cout, k, stride, dil, pad, act, variant, direct, tune):
    # gemm_variant 10..14 / 16: conv_gemm3 tiles (16: 256 x 192 on 4 x 2 waves), 15: auto, 20/24: conv_gemm4;
    # gemm3_direct: conv_gemm3 register epilogues
    # (all forms) or the LDS-staged C tile
    tune(None, gemm_variant=variant, gemm3_direct=direct)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, Cin, T, generator=g)
    w = torch.randn(Cout, Cin, k, generator=g) / np.sqrt(Cin * k)
    b = torch.randn(Cout, generator=g) * 0.1
    ref = F.conv1d(x, w, b, stride=stride, padding=pad, dilation=dil)
    ref = [ref, F.gelu(ref), F.relu(ref)][act]
    To = ref.shape[-1]
    y = torch.empty(B * To, Cout, device="cuda")
    xd, wd, bd = dev(_tm(x)), dev(w), dev(b)  # keep device tensors alive across the call
    call("svc_op_conv1d", ptr(xd), B, T, Cin, ptr(wd), ptr(bd), Cout, k, stride, dil, pad, act, ptr(y), stream())
    out = y.cpu().view(B, To, Cout).permute(0, 2, 1).numpy()
    assert rel_l2(out, ref.numpy()) < 2e-3


@pytest.mark.parametrize("B,T,Cin,Cout,k,s", [(2, 25, 768, 384, 8, 4), (1, 40, 96, 48, 4, 2), (2, 33, 48, 24, 4, 2),
                                              (1, 9, 1536, 768, 8, 4)])
@pytest.mark.parametrize("variant", ["10", "14", "15", "16", "20", "24"])
def test_conv_transpose1d(B, T, Cin, Cout, k, s, variant, tune):
    tune(None, gemm_variant=variant)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, Cin, T, generator=g)
    w = torch.randn(Cin, Cout, k, generator=g) / np.sqrt(Cin * k / s)
    b = torch.randn(Cout, generator=g) * 0.1
    pad = (k - s) // 2
    ref = F.conv_transpose1d(x, w, b, stride=s, padding=pad)
    To = ref.shape[-1]
    assert To == T * s
    y = torch.empty(B * To, Cout, device="cuda")
    xd, wd, bd = dev(_tm(x)), dev(w), dev(b)
    call("svc_op_conv_transpose1d", ptr(xd), B, T, Cin, ptr(wd), ptr(bd), Cout, k, s, pad, ptr(y), stream())
    out = y.cpu().view(B, To, Cout).permute(0, 2, 1).numpy()
    assert rel_l2(out, ref.numpy()) < 2e-3


@pytest.mark.parametrize("x16", [False, True])
@pytest.mark.parametrize("B,L,C", [(2, 37, 24), (1, 1, 24), (1, 2, 48), (1, 3, 8), (2, 11, 12), (3, 129, 96),
                                   (1, 300, 768), (2, 64, 40), (2, 257, 48), (2, 700, 1536), (3, 1000, 192)])
def test_activation1d(B, L, C, x16):
    """f32 input (the generator's residual stream) and f16 input (an AMPBlock1 convs1 output): the reference runs on
    the same f16-rounded values. L = 700 / 1000 hold runs clear of both utterance ends (the clamp-free form)."""
    from svc_inference_pipeline_amd import weights as W
    g = torch.Generator().manual_seed(2)
    x = torch.randn(B, C, L, generator=g) * 2
    if x16:
        x = x.half().float()
    al = torch.randn(C, generator=g) * 0.3
    be = torch.randn(C, generator=g) * 0.3
    f = W.kaiser_sinc_filter1d(0.25, 0.3, 12).view(-1)
    ref = OM.activation1d(x, al, be, f)
    y = torch.empty(B * L, C, device="cuda")
    xd, ad, bd, fd = dev(_tm(x), torch.float16 if x16 else torch.float32), dev(al), dev(be), dev(f)
    call("svc_op_activation1d_x16" if x16 else "svc_op_activation1d", ptr(xd), B, L, C, ptr(ad), ptr(bd), ptr(fd),
         ptr(y), stream())
    out = y.cpu().view(B, L, C).permute(0, 2, 1).numpy()
    assert rel_l2(out, ref.numpy()) < 1e-3
    # fp16 output rounding bound, element-wise
    assert np.max(np.abs(out - ref.numpy()) / (np.abs(ref.numpy()) + 1e-2)) < 5e-3


@pytest.mark.parametrize("C", [24, 48, 96, 192])
@pytest.mark.parametrize("B,L,k,d", [(2, 37, 3, 1), (1, 1, 11, 5), (1, 5, 7, 3), (2, 130, 11, 5), (1, 300, 7, 3),
                                     (3, 257, 11, 1), (2, 600, 3, 5)])
def test_amp_conv(B, L, k, d, C):
    """Fused SnakeBeta Activation1d -> dilated conv -> bias + residual (BigVGAN C <= 96 stages; C <= 48 run the
    packed channel-pair activation; C = 96 on 256-row tiles of 2 x 2 waves, C = 192 of 2 x 4)."""
    from svc_inference_pipeline_amd import weights as W
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, C, L, generator=g) * 2
    al = torch.randn(C, generator=g) * 0.3
    be = torch.randn(C, generator=g) * 0.3
    f = W.kaiser_sinc_filter1d(0.25, 0.3, 12).view(-1)
    w = torch.randn(C, C, k, generator=g) / np.sqrt(C * k)
    b = torch.randn(C, generator=g) * 0.1
    res = torch.randn(B, C, L, generator=g)
    ref = F.conv1d(OM.activation1d(x, al, be, f), w, b, padding=(k - 1) // 2 * d, dilation=d) + res
    y = torch.empty(B * L, C, device="cuda")
    xd, ad, bd, fd, wd, bbd, rd = dev(_tm(x)), dev(al), dev(be), dev(f), dev(w), dev(b), dev(_tm(res))
    call("svc_op_amp_conv", ptr(xd), B, L, C, ptr(ad), ptr(bd), ptr(fd), ptr(wd), ptr(bbd), k, d, ptr(rd), ptr(y),
         stream())
    out = y.cpu().view(B, L, C).permute(0, 2, 1).numpy()
    assert rel_l2(out, ref.numpy()) < 2e-3


def test_bigvgan_activation_launch_chunks():
    """Batches whose activation input spans more than 2 GiB: activation1d and amp_conv address x through 32-bit buffer
    descriptors, so the host splits the batch into launches of < 2^31 bytes (98 + 2 utterances here). Each utterance
    of the big batch must equal the same utterance run alone, bit for bit, on both sides of the split."""
    from svc_inference_pipeline_amd import weights as W
    B, L, C, k, d = 100, 224000, 24, 3, 1
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(B * L, C, device="cuda", generator=g) * 2
    al = torch.randn(C, device="cuda", generator=g) * 0.3
    be = torch.randn(C, device="cuda", generator=g) * 0.3
    f = W.kaiser_sinc_filter1d(0.25, 0.3, 12).view(-1).cuda()
    w = torch.randn(C, C, k, device="cuda", generator=g) / np.sqrt(C * k)
    b = torch.randn(C, device="cuda", generator=g) * 0.1
    y = torch.empty(B * L, C, device="cuda")
    y1 = torch.empty(L, C, device="cuda")
    for op in ("act", "amp"):
        if op == "act":
            call("svc_op_activation1d", ptr(x), B, L, C, ptr(al), ptr(be), ptr(f), ptr(y), stream())
        else:
            call("svc_op_amp_conv", ptr(x), B, L, C, ptr(al), ptr(be), ptr(f), ptr(w), ptr(b), k, d, None, ptr(y),
                 stream())
        for u in (0, 97, 98, 99):
            xu = x[u * L:(u + 1) * L]
            if op == "act":
                call("svc_op_activation1d", ptr(xu), 1, L, C, ptr(al), ptr(be), ptr(f), ptr(y1), stream())
            else:
                call("svc_op_amp_conv", ptr(xu), 1, L, C, ptr(al), ptr(be), ptr(f), ptr(w), ptr(b), k, d, None,
                     ptr(y1), stream())
            torch.cuda.synchronize()
            assert torch.equal(y[u * L:(u + 1) * L], y1), (op, u)


@pytest.mark.parametrize("B,L,D", [(1, 1500, 1024), (2, 100, 128), (1, 64, 64), (2, 1, 64), (1, 129, 256)])
def test_attention(B, L, D):
    g = torch.Generator().manual_seed(3)
    q, k, v = (torch.randn(B, L, D, generator=g) for _ in range(3))
    H = D // 64
    sc = 64 ** -0.25
    qh = q.view(B, L, H, 64).permute(0, 2, 1, 3) * sc
    kh = k.view(B, L, H, 64).permute(0, 2, 3, 1) * sc
    vh = v.view(B, L, H, 64).permute(0, 2, 1, 3)
    ref = (F.softmax(qh @ kh, dim=-1) @ vh).permute(0, 2, 1, 3).reshape(B, L, D)
    out = torch.empty(B * L, D, device="cuda")
    qd, kd, vd = dev(q.reshape(B * L, D)), dev(k.reshape(B * L, D)), dev(v.reshape(B * L, D))
    call("svc_op_attention", ptr(qd), ptr(kd), ptr(vd), B, L, D, ptr(out), stream())
    assert rel_l2(out.cpu().view(B, L, D).numpy(), ref.numpy()) < 3e-3


@pytest.mark.parametrize("mode", ["ramp", "outlier"])
def test_attention_rescale(mode):
    """The deferred online-softmax rescale (attention.hip: the running max moves only when a tile's P column sum exceeds
    ATT_PSUM) on inputs that make it fire: key norms ramping up along the sequence (the max grows on many tiles), and
    one outlier key per head far past the first tile (P of a column jumps from <= 1 to ~2^40 in one tile). Against the
    fp32 torch reference at the Whisper-medium head layout (L = 1500, 4 heads)."""
    B, L, D = 2, 1500, 256
    g = torch.Generator().manual_seed(11)
    q, k, v = (torch.randn(B, L, D, generator=g) for _ in range(3))
    if mode == "ramp":
        k = k * torch.linspace(0.5, 4.0, L)[None, :, None]
    else:
        k[:, 1100] *= 12.0
        q = q + 0.5 * k[:, 1100:1101]
    H = D // 64
    sc = 64 ** -0.25
    qh = q.view(B, L, H, 64).permute(0, 2, 1, 3) * sc
    kh = k.view(B, L, H, 64).permute(0, 2, 3, 1) * sc
    vh = v.view(B, L, H, 64).permute(0, 2, 1, 3)
    ref = (F.softmax(qh @ kh, dim=-1) @ vh).permute(0, 2, 1, 3).reshape(B, L, D)
    out = torch.empty(B * L, D, device="cuda")
    qd, kd, vd = dev(q.reshape(B * L, D)), dev(k.reshape(B * L, D)), dev(v.reshape(B * L, D))
    call("svc_op_attention", ptr(qd), ptr(kd), ptr(vd), B, L, D, ptr(out), stream())
    o = out.cpu().view(B, L, D).numpy()
    assert np.isfinite(o).all()
    assert rel_l2(o, ref.numpy()) < 3e-3


def test_layernorm():
    g = torch.Generator().manual_seed(4)
    x = torch.randn(300, 1024, generator=g) * 3 + 1
    gm = torch.randn(1024, generator=g)
    bt = torch.randn(1024, generator=g)
    ref = F.layer_norm(x, (1024,), gm, bt)
    y = torch.empty(300, 1024, device="cuda")
    xd, gd, bd = dev(x), dev(gm), dev(bt)
    call("svc_op_layernorm", ptr(xd), ptr(gd), ptr(bd), 300, 1024, ptr(y), stream())
    np.testing.assert_allclose(y.cpu().numpy(), ref.numpy(), rtol=0, atol=2e-5)
