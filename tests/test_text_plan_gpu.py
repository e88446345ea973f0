"""Torch-free BERT serving from a text plan image (VERDICT r2 "next round" #8): ``hipzap plan
--model bert-base --batch 16`` writes a plan whose three host inputs (token ids, token types,
additive mask) ``PlanTextBackend`` fills from a JSON request; the server picks it for the
checkpoint, ``POST /predict {"input_ids": ...}`` is answered without torch on the request path,
and a fresh process cold-starts from the plan without importing torch."""
import json
import os

import numpy as np
import pytest
import torch

from hipzap.engine.engine import Engine
from hipzap.engine.plan import export_from_checkpoint
from hipzap.models import registry

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bert(tmp_path_factory):
    d = tmp_path_factory.mktemp("bucket")
    torch.manual_seed(3)
    m = registry.get("bert-base").make_model().eval()
    sd = m.state_dict()
    base = d / "models" / "bert"
    base.mkdir(parents=True)
    ckpt = str(base / "bert.model.pth")
    torch.save(sd, ckpt)
    plan = export_from_checkpoint("bert-base", ckpt, batch=16, contexts=1)
    return {"dir": d, "ckpt": ckpt, "plan": plan, "sd": sd, "model": m}


def _request(n=3, L=100, seed=0):
    g = np.random.default_rng(seed)
    ids = g.integers(1000, 30000, (n, L))
    ids[:, 0] = 101
    types = np.zeros_like(ids)
    types[:, L // 2:] = 1
    mask = np.ones_like(ids)
    mask[1, 60:] = 0  # one sequence padded inside the request
    return ids, types, mask


def test_text_plan_equals_engine_and_hf(bert):
    from hipzap.serve.server import PlanTextBackend
    from hipzap.serve.settings import ModelSpec
    be = PlanTextBackend("bert-base", bert["plan"], 0, ModelSpec(name="bert-base", contexts=2))
    ids, types, mask = _request()
    got = be.infer_np(ids, types, mask)
    assert got.shape == (3, 2) and np.isfinite(got).all()
    # the torch-built engine runs the same program from the same checkpoint (packed on the GPU)
    eng = Engine.from_state_dict("bert-base", bert["sd"], "cuda:0", batch=16, num_contexts=1)
    from hipzap.models.bert import encode_inputs
    Lc = 128
    pad = lambda a: np.pad(a, ((0, 16 - a.shape[0]), (0, Lc - a.shape[1])))  # noqa: E731
    ref = eng.infer(encode_inputs(*(torch.from_numpy(pad(a)) for a in (ids, types, mask))))[:3].float().numpy()
    assert np.abs(got - ref).max() <= 2e-2 * np.abs(ref).max() + 1e-3, (got, ref)
    # and the HF model in fp32 on the unpadded request
    with torch.no_grad():
        hf = bert["model"](input_ids=torch.from_numpy(ids), token_type_ids=torch.from_numpy(types),
                           attention_mask=torch.from_numpy(mask)).logits.numpy()
    assert np.abs(got - hf).max() <= 5e-2 * np.abs(hf).max() + 2e-2, (got, hf)
    # more sequences than the captured batch: chunked; the first 3 rows are unchanged
    ids2 = np.concatenate([ids] * 7)  # 21 > 16
    got2 = be.infer_np(ids2, np.concatenate([types] * 7), np.concatenate([mask] * 7))
    assert got2.shape == (21, 2) and np.array_equal(got2[:3], got) and np.array_equal(got2[18:21], got)
    # concurrent requests through the per-request executor once the contexts exist
    be.engine.ensure_contexts()
    assert np.array_equal(be.infer_np(ids, types, mask), got)
    with pytest.raises(ValueError):
        be.infer_np(np.full((1, 4), 30522))  # outside the vocabulary: rejected on the host
    with pytest.raises(ValueError):
        be.infer_np(np.zeros((1, 129), np.int64))  # longer than the captured sequence
    be.engine.close()


def test_text_plan_served_by_the_app(bert, monkeypatch):
    from hipzap.serve import app as app_mod
    from hipzap.serve.server import ModelServer, PlanTextBackend
    from hipzap.serve.settings import load_settings
    settings = bert["dir"] / "zappa_settings.json"
    settings.write_text(json.dumps({"dev": {"aws_environment_variables": {"models_bucket": f"file://{bert['dir']}"},
                                            "hipzap": {"models": {"bert-base": {"key": "models/bert/bert.model.pth",
                                                                                "contexts": 2}}}}}))
    monkeypatch.setenv("HIPZAP_ARTIFACT_ROOT", str(bert["dir"] / "cache"))
    st = load_settings(str(settings), "dev")
    srv = ModelServer(st, backend="gpu")
    app_mod.set_server(srv)
    try:
        c = app_mod.app.test_client()
        ids, types, mask = _request(n=2, L=40, seed=1)
        r = c.post("/predict", json={"model": "bert-base", "input_ids": ids.tolist(),
                                     "token_type_ids": types.tolist(), "attention_mask": mask.tolist()})
        assert r.status_code == 200, r.data
        assert isinstance(srv._models["bert-base"], PlanTextBackend)
        probs = np.asarray(r.json["probs"])
        assert probs.shape == (2, 2) and np.allclose(probs.sum(-1), 1, atol=1e-4)
        direct = srv._models["bert-base"].infer_np(ids, types, mask)
        assert r.json["label"] == [int(i) for i in direct.argmax(-1)]
        r = c.post("/predict", json={"model": "bert-base", "input_ids": [[5, 40000]]})
        assert r.status_code == 400 and r.json["error"] == "ValueError"
    finally:
        app_mod.set_server(None)
        be = srv._models.get("bert-base")
        if be is not None and hasattr(be.engine, "close"):
            be.engine.close()


def test_text_plan_fresh_process_cold_start(bert):
    from hipzap.coldstart import measure_fresh
    res = measure_fresh("plan", bert["plan"], trials=3)
    print("bert plan cold start", json.dumps(res))
    assert res["torch_imported"] is False
    assert res["p50_ms"] < 5000
