"""Inputs of tests/golden/plms100_headline.npz (written by tools/make_goldens_headline.py from the reference's own
svc_model_inference, PLMS speedup 10 at T = 937): the mapper weights (seed 0, the final eps head x OUT_GAIN), the
seeded conditioning and x_T of its two utterances. Shared by the generator and the CPU / GPU tests."""
import numpy as np

from oracle import noise as ON
from svc_inference_pipeline_amd import weights as W

T = 937
OUT_GAIN = 3.0
XT_SEEDS = (11, 12)
COND_SEEDS = (21, 22)


def headline_mapper_state(mcfg):
    """make_mapper_state(seed 0) with modules/diffsvc.py:282's output_projection (the eps head) x OUT_GAIN: the random
    denoiser's eps then spreads ~1.1 per element, the scale of the unit-variance noise a trained eps-predictor estimates,
    so the eps-induced part of the PLMS-100 output (x_0 - x_0|eps=0) is 80 % of its norm (~10 % with the plain random
    weights)."""
    sd = W.make_mapper_state(mcfg, 0)
    for k in ("1.output_projection.weight", "1.output_projection.bias"):
        sd[k] = (sd[k] * np.float32(OUT_GAIN)).astype(np.float32)
    return sd


def headline_cond(u):
    """utterance u's conditioning [1, T, 384] (the sampler's input; the conditioner is pinned separately)"""
    return np.random.default_rng(COND_SEEDS[u]).standard_normal((1, T, 384), dtype=np.float32)


def headline_x_T(u):
    return ON.x_T(XT_SEEDS[u], 1, T)
