"""Configuration: a JSON5-subset reader + attribute-style hyper-parameter object.

Mirrors the reference's `load_config` / `JsonHParams` (utils/util.py:57-122). json5 is not
installed here, so `loads_json5` accepts exactly what the reference's config.json uses: `//` line
comments, `/* */` block comments and trailing commas. The `basic_config` inheritance through
`$WORD_DIR` (utils/util.py:68-77) is kept.

The package ships a condensed copy of the reference's config (svc_inference_pipeline_amd/config/):
the 1000-entry explicit `mapper.noise_schedule` list is omitted because DiffSVC overwrites it from
`noise_schedule_factors` (modules/diffsvc.py:248-252); `noise_schedule()` below derives it the same
way. Normalisation/F0 statistics come from config/stats.json (extracted from the reference pickles
without unpickling, tools/extract_config_stats.py).
"""
import json
import os
import re

import numpy as np

CONFIG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config")


def _strip_json5(text: str) -> str:
    out = []
    i, n = 0, len(text)
    in_str = None
    while i < n:
        c = text[i]
        if in_str:
            out.append(c)
            if c == "\\" and i + 1 < n:
                out.append(text[i + 1])
                i += 2
                continue
            if c == in_str:
                in_str = None
            i += 1
            continue
        if c in "\"'":
            in_str = c
            out.append('"')  # single-quoted JSON5 strings are normalised to double quotes
            i += 1
            continue
        if text.startswith("//", i):
            j = text.find("\n", i)
            i = n if j < 0 else j
            continue
        if text.startswith("/*", i):
            j = text.find("*/", i + 2)
            if j < 0:
                raise ValueError("unterminated block comment")
            i = j + 2
            continue
        out.append(c)
        i += 1
    s = "".join(out)
    return re.sub(r",(\s*[}\]])", r"\1", s)


def loads_json5(text: str):
    return json.loads(_strip_json5(text))


def override_config(basic_config, new_config):
    """utils/util.py:57-65."""
    for k, v in new_config.items():
        if isinstance(v, dict):
            basic_config[k] = override_config(basic_config.get(k, {}), v)
        else:
            basic_config[k] = v
    return basic_config


def _load_config(config_fn):
    """utils/util.py:68-78 (basic_config inheritance via $WORD_DIR)."""
    with open(config_fn, "r") as f:
        cfg = loads_json5(f.read())
    if "basic_config" in cfg:
        parent = os.path.join(os.getenv("WORD_DIR", ""), cfg["basic_config"])
        cfg = override_config(_load_config(parent), cfg)
    return cfg


class JsonHParams:
    """Attribute-style nested config (utils/util.py:92-122)."""

    def __init__(self, **kwargs):
        for k, v in kwargs.items():
            if isinstance(v, dict):
                v = JsonHParams(**v)
            self[k] = v

    def keys(self):
        return self.__dict__.keys()

    def items(self):
        return self.__dict__.items()

    def values(self):
        return self.__dict__.values()

    def __len__(self):
        return len(self.__dict__)

    def __getitem__(self, key):
        return getattr(self, key)

    def __setitem__(self, key, value):
        return setattr(self, key, value)

    def __contains__(self, key):
        return key in self.__dict__

    def __repr__(self):
        return self.__dict__.__repr__()

    def to_dict(self):
        return {k: (v.to_dict() if isinstance(v, JsonHParams) else v) for k, v in self.items()}


def load_config(config_fn=None):
    """utils/util.py:81-89. Defaults to the packaged config."""
    if config_fn is None:
        config_fn = os.path.join(CONFIG_DIR, "config.json")
    hps = JsonHParams(**_load_config(config_fn))
    hps.config_dir = os.path.dirname(os.path.abspath(config_fn))
    return hps


def noise_schedule(mapper_cfg):
    """modules/diffsvc.py:248-252: np.linspace(*noise_schedule_factors) (f64)."""
    a, b, n = mapper_cfg.noise_schedule_factors
    return np.linspace(a, b, int(n))


def load_stats(cfg):
    path = os.path.join(getattr(cfg, "config_dir", CONFIG_DIR), cfg.stats_file)
    with open(path) as f:
        s = json.load(f)
    return {
        "mel_min": np.asarray(s["mel_min"], dtype=np.float32),
        "mel_max": np.asarray(s["mel_max"], dtype=np.float32),
        "target_f0_median": float(s["target_f0_median"]),
    }


def load_singers(cfg):
    path = os.path.join(getattr(cfg, "config_dir", CONFIG_DIR), cfg.singer_file)
    with open(path) as f:
        return json.load(f)
