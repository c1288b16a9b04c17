"""Helpers for the -m gpu parity tests (they call libsvc_hip.so through its C-ABI)."""
import ctypes

import numpy as np
import torch

from svc_inference_pipeline_amd import _lib


def dev(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a)).to(dtype).cuda().contiguous()


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def call(name, *args):
    _lib.call(name, *args)
    torch.cuda.synchronize()
