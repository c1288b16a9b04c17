"""ctypes binding of libsvc_hip.so (include/svc_hip.h). There is no fallback: if the library is
missing or fails to load, importing the runtime raises."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SVC_HIP_LIB", os.path.join(_HERE, "libsvc_hip.so"))

c_void_p, c_int, c_int64, c_uint64, c_double = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
c_float_p = ctypes.POINTER(ctypes.c_float)

# name -> (restype, argtypes); every symbol declared in include/svc_hip.h
PROTOTYPES = {
    "svc_last_error": (ctypes.c_char_p, []),
    "svc_abi_version": (c_int, []),
    "svc_ctx_create": (c_int, [c_int, ctypes.POINTER(c_void_p)]),
    "svc_ctx_destroy": (c_int, [c_void_p]),
    "svc_ctx_set_config": (c_int, [c_void_p, ctypes.c_char_p, c_double]),
    "svc_ctx_get_config": (c_int, [c_void_p, ctypes.c_char_p, ctypes.POINTER(c_double)]),
    "svc_config_key_known": (c_int, [ctypes.c_char_p]),
    "svc_ctx_add_param": (c_int, [c_void_p, ctypes.c_char_p, c_void_p, c_int, ctypes.POINTER(c_int64)]),
    "svc_ctx_finalize": (c_int, [c_void_p]),
    "svc_ctx_memory": (c_int, [c_void_p, ctypes.POINTER(c_int64), ctypes.POINTER(c_int64)]),
    "svc_ctx_stream": (c_int, [c_void_p, c_int, ctypes.POINTER(c_void_p)]),
    "svc_mel_energy": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "svc_f0_ac": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p, c_int, c_void_p, c_void_p]),
    "svc_f0_pyin": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p, c_double, c_int, c_int, c_double, c_double,
                            c_int, c_void_p, c_void_p]),
    "svc_pitch_shift": (c_int, [c_void_p, c_void_p, c_int, c_int, c_double, c_void_p]),
    "svc_whisper_encode": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p, c_void_p]),
    "svc_map_content": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "svc_map_content_ex": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "svc_hubert_encode": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p, c_void_p]),
    "svc_hubert_frames": (c_int64, [c_int64]),
    "svc_hubert_dims": (c_int, [c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "svc_condition": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "svc_condition_indices": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "svc_diffsvc_sample": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                   c_uint64, c_void_p, c_void_p, c_void_p]),
    "svc_diffsvc_eps": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p]),
    "svc_bigvgan": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "svc_op_conv1d": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                              c_int, c_void_p, c_void_p]),
    "svc_op_conv_transpose1d": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                        c_void_p, c_void_p]),
    "svc_resample_len": (ctypes.c_int64, [ctypes.c_int64, c_int, c_int]),
    "svc_resample": (c_int, [c_void_p, c_int, ctypes.c_int64, c_int, c_int, c_int, c_void_p, c_void_p]),
    "svc_resample_filter": (c_int, [c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "svc_op_amp_conv": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                c_int, c_void_p, c_void_p, c_void_p]),
    "svc_op_activation1d": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "svc_op_activation1d_x16": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p]),
    "svc_op_attention": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "svc_op_layernorm": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "svc_profile_enable": (c_int, [c_int]),
    "svc_profile_filter": (c_int, [ctypes.c_char_p]),
    "svc_profile_read": (c_int, [c_int, ctypes.c_char_p, c_int, ctypes.POINTER(c_double), ctypes.POINTER(c_int64),
                                 ctypes.POINTER(c_double), ctypes.POINTER(c_double), ctypes.POINTER(c_int)]),
    "svc_gemm_bench": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_double)]),
    "svc_mel_filterbank": (c_int, [c_int, c_int, c_int, c_double, c_double, c_void_p]),
}

ABI_VERSION = 3  # svc_abi_version() of the library these prototypes describe (2: ragged-batch length tables,
#                  3: svc_ctx_get_config, unknown configuration keys rejected)

_lib = None


class SVCError(RuntimeError):
    pass


def load():
    """Load libsvc_hip.so once; raise (no fallback) if it is absent or incomplete."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SVCError(f"libsvc_hip.so not found at {LIB_PATH}: build it with `make` (or __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in PROTOTYPES.items():
        fn = getattr(lib, name)  # AttributeError if an exported symbol is missing
        fn.restype = res
        fn.argtypes = args
    if lib.svc_abi_version() != ABI_VERSION:
        raise SVCError(f"{LIB_PATH}: ABI version {lib.svc_abi_version()}, these bindings need {ABI_VERSION} (rebuild)")
    _lib = lib
    return lib


def check(status):
    if status != 0:
        msg = load().svc_last_error().decode(errors="replace")
        raise SVCError(f"libsvc_hip status {status}: {msg}")
    return status


def call(name, *args):
    return check(getattr(load(), name)(*args))


def tune(ctx=None, **switches):
    """Kernel switches (include/svc_hip.h "tune.<name>", csrc/common.h Tuning) of a context, or with ctx None of the
    op-level entry points' context; tune(ctx, reset=1) restores the values the context was created with."""
    for k, v in switches.items():
        call("svc_ctx_set_config", ctx, f"tune.{k}".encode(), float(v))


def get_config(ctx, key):
    """svc_ctx_get_config: a configuration key's value, or a kernel switch's ("tune.<name>"; ctx None: op level)."""
    v = c_double()
    call("svc_ctx_get_config", ctx, key.encode(), ctypes.byref(v))
    return v.value


def profile_enable(on=True):
    call("svc_profile_enable", 1 if on else 0)


def profile_filter(prefix=""):
    call("svc_profile_filter", prefix.encode() if prefix else None)


def profile_read():
    """{kernel name: dict(ms, launches, flops, bytes)} for the launches recorded since profile_enable(True)."""
    n = ctypes.c_int()
    call("svc_profile_read", -1, None, 0, None, None, None, None, ctypes.byref(n))
    out = {}
    for i in range(n.value):
        name = ctypes.create_string_buffer(128)
        ms, la, fl, by = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
        call("svc_profile_read", i, name, 128, ctypes.byref(ms), ctypes.byref(la), ctypes.byref(fl), ctypes.byref(by),
             ctypes.byref(n))
        out[name.value.decode()] = dict(ms=ms.value, launches=la.value, flops=fl.value, bytes=by.value)
    return out
