"""The Python-free plan server (csrc/tools/serve_plan.cpp, `hipzap-serve-plan`): its --once
cold-start probe and its HTTP front end agree with the PlanEngine on the same plan image."""
import base64
import http.client
import json
import os
import socket
import subprocess
import time

import numpy as np
import pytest
import torch

from hipzap.build import SERVE_PLAN
from hipzap.engine.plan import export_from_checkpoint
from hipzap.lite import PlanEngine
from hipzap.models import registry
from hipzap.models.resnet import randomize_bn

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def plan(tmp_path_factory):
    if not SERVE_PLAN.exists():
        pytest.fail(f"{SERVE_PLAN} not built (python -m hipzap.build)")
    torch.manual_seed(0)
    d = tmp_path_factory.mktemp("native")
    ckpt = str(d / "resnet18.model.pth")
    torch.save(randomize_bn(registry.get("resnet18").make_model()).eval().state_dict(), ckpt)
    return export_from_checkpoint("resnet18", ckpt, batch=1, contexts=1), d


def _img(seed):
    return np.random.default_rng(seed).integers(0, 256, (224, 224, 3), dtype=np.uint8)


def test_once_matches_plan_engine(plan):
    path, d = plan
    img = _img(0)
    raw = d / "img.raw"
    raw.write_bytes(img.tobytes())
    r = subprocess.run([str(SERVE_PLAN), path, "--once", str(raw)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    ref = np.frombuffer(PlanEngine(path, device=0).infer_raw(img), np.float32)
    assert out["argmax"] == int(ref.argmax())
    assert abs(out["logit0"] - float(ref[0])) <= 1e-5 * max(1.0, abs(float(ref[0])))
    assert out["main_to_logits_ms"] > 0


def test_http_predict_health_404(plan):
    path, _ = plan
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    srv = subprocess.Popen([str(SERVE_PLAN), path, "--port", str(port), "--contexts", "4"],
                           stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    try:
        t0 = time.time()
        while True:
            assert srv.poll() is None, srv.stderr.read()
            try:
                c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
                c.request("GET", "/health")
                r = c.getresponse()
                health = json.loads(r.read())
                break
            except OSError:
                assert time.time() - t0 < 60
                time.sleep(0.05)
        assert health["status"] == "ok" and health["contexts"] == 4
        pe = PlanEngine(path, device=0)
        for i in range(3):
            img = _img(10 + i)
            body = json.dumps({"image_b64": base64.b64encode(img.tobytes()).decode(), "shape": [224, 224, 3]})
            c.request("POST", "/predict", body=body, headers={"Content-Type": "application/json"})
            r = c.getresponse()
            got = json.loads(r.read())
            assert r.status == 200 and r.getheader("X-Hipzap-Path") == "native"
            ref = np.frombuffer(pe.infer_raw(img), np.float32)
            assert got["top5"][0][0][0] == int(ref.argmax())
        c.request("GET", "/inference")
        r = c.getresponse()
        r.read()
        assert r.status == 404
    finally:
        srv.terminate()
        srv.wait(timeout=30)
