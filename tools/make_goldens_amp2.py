"""Generate tests/golden/bigvgan_variants.npz: the REFERENCE's own BigVGAN Generator (modules/bigvgan.py:519-622)
in the configurations `infer.py` does not use but the config can select:
  * amp2_snake_log : resblock "2" (AMPBlock2, :442-516, dilations (1, 3)), activation "snake" (:42-92), log scale
  * amp2_snake_lin : the same with snake_logscale = false (alpha used as is)
  * amp1_snake_log : resblock "1" (AMPBlock1) with Snake instead of SnakeBeta
Weights are seeded (svc_inference_pipeline_amd.weights.make_vocoder_state on the modified vocoder config, seed 0);
the input is a de-normalised mel of 24 frames. Build container only; outputs are data only.
Usage:  python tools/make_goldens_amp2.py
"""
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_goldens import OUT, install_shims, load_into  # noqa: E402
from oracle import features as OF  # noqa: E402
from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd import weights as W  # noqa: E402

def main():
    install_shims()
    torch.set_num_threads(8)
    from modules.bigvgan import Generator  # noqa: E402

    cfg = C.load_config()
    stats = C.load_stats(cfg)
    Tv = 24  # synthesis_audios needs T >= 20 (modules/bigvgan_inference.py:33-44)
    mel = OF.denormalize_mel_channel(np.random.default_rng(21).uniform(-1, 1, (100, Tv)).astype(np.float32),
                                     stats["mel_min"], stats["mel_max"]).astype(np.float32)
    out = {"mel": mel}
    for name in W.VOCODER_VARIANTS:
        vcfg = W.vocoder_variant_cfg(cfg.vocoder, name)
        sd = W.make_vocoder_state(vcfg, seed=0)
        gen = Generator(vcfg)
        load_into(gen, sd)
        gen.eval()
        with torch.no_grad():
            out[name] = gen(torch.from_numpy(mel).unsqueeze(0)).numpy()
        print(name, out[name].shape, float(np.abs(out[name]).mean()))
    np.savez_compressed(os.path.join(OUT, "bigvgan_variants.npz"), **out)


if __name__ == "__main__":
    main()
