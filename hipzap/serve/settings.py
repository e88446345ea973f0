"""Zappa-compatible settings (``zappa_settings.json``) + typed hipzap serving config.

The reference reads ``zappa_settings.json[stage]['aws_environment_variables']`` into
``os.environ`` for local runs (/root/reference/main.py:115-126) and Zappa injects the same
variables on Lambda; the models bucket comes from ``models_bucket`` (main.py:88). The same
schema is accepted here (stage selectable, ``HIPZAP_STAGE``), plus an optional ``hipzap``
block for the runtime (models, devices, contexts, graph capture, port). Environment
variables override the file (``HIPZAP_*``).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field

DEFAULT_STAGE = "dev"


@dataclass
class ModelSpec:
    name: str                     # registry name: resnet50, resnet18, bert-base, vit-b16, awd-lstm
    key: str | None = None        # artifact key of the state_dict (models/<name>/<name>.model.pth)
    vocab_key: str | None = None  # AWD-LSTM vocabulary (models/<name>/<name>.itos.pkl)
    batch: int = 1
    contexts: int = 2
    dtype: str = "bf16"
    extra: dict = field(default_factory=dict)


@dataclass
class Settings:
    stage: str = DEFAULT_STAGE
    models_bucket: str | None = None
    artifact_root: str = os.environ.get("HIPZAP_ARTIFACT_ROOT", "/tmp")
    models: dict = field(default_factory=dict)       # route name -> ModelSpec
    default_model: str = "resnet50"
    lm_model: str = "rjokes"
    lm_words: int = 200
    devices: list = field(default_factory=lambda: [0])
    capture_graphs: bool = True
    host: str = "0.0.0.0"
    port: int = 8082
    raw: dict = field(default_factory=dict)

    @property
    def lm_model_key(self) -> str:
        return f"models/{self.lm_model}/{self.lm_model}.model.pth"

    @property
    def lm_vocab_key(self) -> str:
        return f"models/{self.lm_model}/{self.lm_model}.itos.pkl"


def read_zappa_settings(path: str = "zappa_settings.json") -> dict:
    with open(path) as f:
        return json.load(f)


def apply_environment(cfg: dict, stage: str = DEFAULT_STAGE, environ=None) -> dict:
    """main.py:121-125: copy ``aws_environment_variables`` of ``stage`` into the environment."""
    environ = os.environ if environ is None else environ
    env = cfg.get(stage, {}).get("aws_environment_variables", {}) or {}
    for k, v in env.items():
        environ[str(k)] = str(v)
    return env


def load_settings(path: str | None = None, stage: str | None = None, environ=None) -> Settings:
    environ = os.environ if environ is None else environ
    stage = stage or environ.get("HIPZAP_STAGE") or DEFAULT_STAGE
    path = path or environ.get("HIPZAP_SETTINGS") or "zappa_settings.json"
    raw = {}
    if path and os.path.exists(path):
        raw = read_zappa_settings(path)
        apply_environment(raw, stage, environ)
    st = Settings(stage=stage, raw=raw)
    st.models_bucket = environ.get("models_bucket") or environ.get("HIPZAP_MODELS_BUCKET")
    hz = raw.get(stage, {}).get("hipzap", {}) if raw else {}
    for k in ("default_model", "lm_model", "lm_words", "devices", "capture_graphs", "host", "port", "artifact_root"):
        if k in hz:
            setattr(st, k, hz[k])
    for name, spec in (hz.get("models") or {}).items():
        st.models[name] = ModelSpec(name=spec.get("model", name), key=spec.get("key"), vocab_key=spec.get("vocab_key"),
                                    batch=int(spec.get("batch", 1)), contexts=int(spec.get("contexts", 2)),
                                    dtype=spec.get("dtype", "bf16"), extra=spec.get("extra", {}))
    if "HIPZAP_PORT" in environ:
        st.port = int(environ["HIPZAP_PORT"])
    if "HIPZAP_DEVICES" in environ:
        st.devices = [int(x) for x in environ["HIPZAP_DEVICES"].split(",") if x.strip()]
    if "HIPZAP_LM_WORDS" in environ:
        st.lm_words = int(environ["HIPZAP_LM_WORDS"])
    if environ.get("HIPZAP_NO_GRAPH"):
        st.capture_graphs = False
    return st
