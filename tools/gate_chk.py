import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np, torch
from gpu_util import dev, rel_l2
from svc_inference_pipeline_amd import config as C, weights as W
from svc_inference_pipeline_amd.runtime import SVCEngine
from oracle import models as OM
cfg = C.load_config(); TINY = W.WHISPER_DIMS["tiny-test"]; cfg.mapper.input_content_dim["whisper"] = TINY["n_audio_state"]
ms = W.make_mapper_state(cfg.mapper, 0)
e = SVCEngine(cfg, 0, whisper_state=W.make_whisper_state(TINY, 0), mapper_state=ms, vocoder_state=W.make_vocoder_state(cfg.vocoder, 0))
G = lambda n: np.load(os.path.join("tests/golden", n + ".npz"))
g = G("conditioner_diffsvc"); s = G("samplers")
out = {}
for t in (0, 500, 999):
    eps = e.diffsvc_eps(dev(g["cond"]), dev(g["x_in"]), t).cpu().numpy()
    out[f"eps{t}"] = rel_l2(eps, g[f"eps_t{t}"])
cond = dev(g["cond"])
x4 = e.diffsvc_sample(cond, fast_inference=True, speedup=250, x_T=dev(s["x_T"]))
out["plms4"] = rel_l2(x4[0].cpu().numpy().T, s["plms4"])
x = e.diffsvc_sample(cond, fast_inference=True, speedup=10, x_T=dev(s["x_T"]))
out["plms100"] = rel_l2(x[0].cpu().numpy().T, s["plms100"])
np.save(f"gpurun_out/gate_{os.environ.get('TAGX','x')}.npy", x.cpu().numpy())
print(os.environ.get("TAGX"), {k: f"{v:.3e}" for k, v in out.items()}, flush=True)
