"""F3: ragged request lists through SVCPipeline.convert_many. Every output must be
bit-identical to converting that clip alone with the same utterance id (exact integer equality of the f32
waveform): bucketing by length never changes per-utterance arithmetic."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from gpu_util import dev  # noqa: E402
from oracle import noise as ON  # noqa: E402
from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd import weights as W  # noqa: E402
from svc_inference_pipeline_amd.pipeline import SVCPipeline  # noqa: E402
from svc_inference_pipeline_amd.runtime import SVCEngine  # noqa: E402


def test_convert_many_matches_single_clips():
    cfg = C.load_config()
    dims = W.WHISPER_DIMS["tiny-test"]
    cfg.mapper.input_content_dim["whisper"] = dims["n_audio_state"]
    e = SVCEngine(cfg, 0, whisper_state=W.make_whisper_state(dims, 0), mapper_state=W.make_mapper_state(cfg.mapper, 0),
                  vocoder_state=W.make_vocoder_state(cfg.vocoder, 0))
    try:
        pipe = SVCPipeline(e)
        secs = [0.6, 1.0, 0.6, 0.45]
        w24 = [dev(ON.synth_clip(40 + i, s, 24000)) for i, s in enumerate(secs)]
        w16 = [dev(ON.synth_clip_16k_quantised(40 + i, s)) for i, s in enumerate(secs)]
        singers = [1, 3, 0, 2]
        outs = pipe.convert_many(w24, w16, singers, speedup=250, seed=5)
        assert [o.shape[0] for o in outs] == [((len(w) + 768 - 1024) // 256 + 1) * 256 for w in w24]
        for i in range(len(secs)):
            one = pipe.convert(w24[i][None], w16[i][None], dev(np.array([singers[i]]), torch.int32), speedup=250,
                               seed=5, utt_ids=dev(np.array([i]), torch.int32)).wav[0]
            assert torch.equal(outs[i], one), i
    finally:
        e.close()


def test_feature_side_stream_and_residual_modes(monkeypatch):
    """The 24 kHz features on the context's sub-stream 2 (SVC_F0_SIDE, default on) give bit-identical conversions to
    running them on the caller's stream; the split-fp16 DiffSVC residual stream (default) stays within 2e-3 of the
    f32 one (SVC_DIFF_RES32=1) on the sampler output."""
    cfg = C.load_config()
    dims = W.WHISPER_DIMS["tiny-test"]
    cfg.mapper.input_content_dim["whisper"] = dims["n_audio_state"]
    e = SVCEngine(cfg, 0, whisper_state=W.make_whisper_state(dims, 0), mapper_state=W.make_mapper_state(cfg.mapper, 0),
                  vocoder_state=W.make_vocoder_state(cfg.vocoder, 0))
    try:
        pipe = SVCPipeline(e)
        w24 = dev(np.stack([ON.synth_clip(60 + i, 0.8, 24000) for i in range(3)]))
        w16 = dev(np.stack([ON.synth_clip_16k_quantised(60 + i, 0.8) for i in range(3)]))
        sing = dev(np.array([0, 2, 4]), torch.int32)
        res = {}
        for side in ("1", "0"):
            monkeypatch.setenv("SVC_F0_SIDE", side)
            r = pipe.convert(w24, w16, sing, speedup=250, seed=3)
            res[side] = (r.wav.clone(), r.f0.clone(), r.mel.clone(), r.x0.clone())
        for a, b in zip(res["1"], res["0"]):
            assert torch.equal(a, b)
        monkeypatch.setenv("SVC_DIFF_RES32", "1")
        x32 = pipe.convert(w24, w16, sing, speedup=250, seed=3).x0
        rel = float(torch.linalg.norm(res["1"][3] - x32) / torch.linalg.norm(x32))
        assert rel < 2e-3, rel
    finally:
        e.close()
