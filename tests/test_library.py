"""CPU: the C-ABI library builds, loads and exports every symbol include/svc_hip.h declares; the
native slaney filterbank matches the reference's mel_filters.npz known answer."""
import ctypes
import os
import re

import numpy as np

from svc_inference_pipeline_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(REPO, "include", "svc_hip.h")).read()
    return sorted(set(re.findall(r"^(?:svc_status|const char\*|int|int64_t)\s+(svc_[a-z0-9_]+)\s*\(", txt, re.M)))


def test_header_matches_binding():
    assert header_symbols() == sorted(_lib.PROTOTYPES)


def test_library_exports_all_symbols():
    lib = _lib.load()
    for name in header_symbols():
        assert hasattr(lib, name), name
    assert lib.svc_abi_version() == _lib.ABI_VERSION == 3  # 3: svc_ctx_get_config, config keys checked


def test_native_mel_filterbank_kat(golden):
    kat = golden("mel_filters_kat")["mel_80"]
    out = np.zeros((80, 201), dtype=np.float32)
    _lib.call("svc_mel_filterbank", 16000, 400, 80, 0.0, 8000.0, out.ctypes.data_as(ctypes.c_void_p))
    assert np.max(np.abs(out - kat)) <= 2e-7 * np.abs(kat).max()


def test_native_mel_filterbank_24k():
    from oracle.features import slaney_mel_filterbank
    ref = slaney_mel_filterbank(24000, 1024, 100, 0.0, 12000.0)
    out = np.zeros_like(ref)
    _lib.call("svc_mel_filterbank", 24000, 1024, 100, 0.0, 12000.0, out.ctypes.data_as(ctypes.c_void_p))
    assert np.max(np.abs(out - ref)) <= 2e-7 * np.abs(ref).max()


def test_no_gpu_error_is_loud():
    """Without a GPU, creating a context fails with a status + message (no silent fallback)."""
    import torch
    if torch.cuda.is_available():
        return
    ctx = ctypes.c_void_p()
    st = _lib.load().svc_ctx_create(0, ctypes.byref(ctx))
    assert st != 0 and _lib.load().svc_last_error()


def test_kernel_switches_are_per_context_config():
    """Kernel switches go through svc_ctx_set_config("tune.<name>") (here on the op-level context, ctx NULL; no GPU
    call is made): known names are accepted and read back by svc_ctx_get_config, unknown ones are rejected loudly,
    "tune.reset" restores the defaults."""
    import pytest
    default = _lib.get_config(None, "tune.sampler_streams")
    _lib.tune(None, gemm_variant=24, sampler_streams=1, amp_maxc=0)
    assert _lib.get_config(None, "tune.sampler_streams") == 1.0
    assert _lib.get_config(None, "tune.gemm_variant") == 24.0
    _lib.tune(None, reset=1)
    assert _lib.get_config(None, "tune.sampler_streams") == default
    with pytest.raises(_lib.SVCError, match="unknown kernel switch"):
        _lib.tune(None, no_such_switch=1)
    with pytest.raises(_lib.SVCError, match="unknown kernel switch"):
        _lib.get_config(None, "tune.no_such_switch")
    with pytest.raises(_lib.SVCError, match="null context"):
        _lib.call("svc_ctx_set_config", None, b"mapper.n_mel", 100.0)


def test_every_documented_kernel_switch_is_accepted():
    """Every "tune.<name>" key the header documents (include/svc_hip.h, svc_ctx_set_config) is a switch the library
    knows (op-level context, no GPU call), and there are at most 10 of them (measured-slower alternates are deleted,
    not kept behind switches); the context is reset afterwards."""
    text = open(os.path.join(REPO, "include", "svc_hip.h")).read()
    block = re.search(r"kernel switch of this context at any time \(([^;]*);", text).group(1)
    names = [n.strip() for n in block.split(",")]
    assert 5 <= len(names) <= 10 and "diff_head" in names and "sampler_streams" in names
    try:
        for n in names:
            _lib.tune(None, **{n: _lib.get_config(None, "tune." + n)})
    finally:
        _lib.tune(None, reset=1)


def test_config_keys_are_checked():
    """svc_ctx_set_config rejects a configuration key the context does not read (a misspelt precision key would
    otherwise leave its default silently in place), and accepts every key SVCEngine writes; checked on the key
    validator alone, without a GPU context, through the flattened reference config."""
    from svc_inference_pipeline_amd import config as C
    from svc_inference_pipeline_amd.runtime import engine_config_keys
    keys = engine_config_keys(C.load_config())
    assert "vocoder.resblock_dilation_sizes.0.n" in keys and "mapper.residual_channels" in keys
    lib = _lib.load()
    for k in list(keys) + ["content.split", "content.wsplit_mlp", "mapper.head_split", "hubert.output_layer"]:
        assert lib.svc_config_key_known(k.encode()) == 1, k
    for k in ["content.wsplit_linears", "mapper.residual_channel", "vocoder.upsample_rates.x", "fs2", ""]:
        assert lib.svc_config_key_known(k.encode()) == 0, k
