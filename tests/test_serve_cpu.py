"""Flask app, CORS, routes and the Zappa-style Lambda adapter on the CPU backend."""
import base64
import io
import json

import numpy as np
import pytest
import torch

from hipzap.serve import app as app_mod
from hipzap.serve.lambda_handler import event_to_environ, is_keep_warm, make_handler
from hipzap.serve.server import ModelServer
from hipzap.serve.settings import Settings


@pytest.fixture(scope="module")
def client(tmp_path_factory, monkeypatch_module):
    monkeypatch_module.setenv("HIPZAP_RANDOM_WEIGHTS", "1")
    monkeypatch_module.setenv("HIPZAP_LM_VOCAB", "300")
    st = Settings(default_model="resnet18", lm_words=12)
    app_mod.set_server(ModelServer(st, backend="cpu"))
    with app_mod.app.test_client() as c:
        yield c
    app_mod.set_server(None)


@pytest.fixture(scope="module")
def monkeypatch_module():
    mp = pytest.MonkeyPatch()
    yield mp
    mp.undo()


def test_index_and_health(client):
    r = client.get("/")
    assert r.status_code == 200 and r.json["service"] == "hipzap"
    assert r.headers["Access-Control-Allow-Origin"] == "*"
    assert client.get("/health").json["status"] == "ok"


def test_cors_preflight(client):
    r = client.open("/predict", method="OPTIONS", headers={"Origin": "http://x", "Access-Control-Request-Method": "POST",
                                                           "Access-Control-Request-Headers": "Content-Type"})
    assert r.status_code == 200
    assert r.headers["Access-Control-Allow-Origin"] == "*"
    assert "POST" in r.headers["Access-Control-Allow-Methods"]


def test_inference_schema(client):
    r = client.get("/inference?seed=1")
    assert r.status_code == 200 and r.mimetype == "application/json"
    body = r.json
    assert set(body) == {"response"} and set(body["response"]) == {"text"}
    assert isinstance(body["response"]["text"], str) and body["response"]["text"].startswith(" ")
    # deterministic with a seed
    assert client.get("/inference?seed=1").json == body


def test_predict_json_tensor(client):
    x = torch.randn(1, 3, 64, 64)
    r = client.post("/predict", json={"model": "resnet18", "inputs": x.tolist()})
    assert r.status_code == 200, r.data
    top = r.json["top5"][0]
    assert len(top) == 5 and all(0 <= i < 1000 for i, _ in top)
    probs = [p for _, p in top]
    assert probs == sorted(probs, reverse=True)


def test_x_timing_header(client):
    """Per-request phase timers (SURVEY.md §5 tracing): decode/load/infer/total in X-Timing."""
    r = client.post("/predict", json={"model": "resnet18", "inputs": torch.randn(1, 3, 32, 32).tolist()})
    phases = dict(kv.split("=") for kv in r.headers["X-Timing"].split(";"))
    assert {"decode", "load", "infer", "total"} <= set(phases)
    assert all(float(v) >= 0 for v in phases.values())
    assert float(phases["total"]) >= float(phases["infer"])
    assert "X-Timing" in r.headers["Access-Control-Expose-Headers"]
    gen = dict(kv.split("=") for kv in client.get("/inference?seed=3").headers["X-Timing"].split(";"))
    assert {"load", "generate", "total"} <= set(gen)


def test_predict_npy_and_image(client):
    buf = io.BytesIO()
    np.save(buf, np.random.randn(2, 3, 32, 32).astype(np.float32))
    r = client.post("/predict?model=resnet18", data=buf.getvalue(), content_type="application/octet-stream")
    assert r.status_code == 200 and r.json["batch"] == 2
    img = np.random.randint(0, 255, (32, 32, 3), dtype=np.uint8)
    r = client.post("/predict", json={"model": "resnet18", "image_b64": base64.b64encode(img.tobytes()).decode(),
                                      "shape": [32, 32, 3]})
    assert r.status_code == 200 and r.json["batch"] == 1


def test_predict_bad_request_is_json_error(client):
    r = client.post("/predict", json={"nothing": 1})
    assert r.status_code == 400 and r.json["error"] == "ValueError"


def test_metrics(client):
    client.get("/health")
    text = client.get("/metrics").data.decode()
    assert "hipzap_requests_total" in text


def test_lambda_v1_event_roundtrip(client):
    handler = make_handler(app_mod.app)
    ev = {"httpMethod": "GET", "path": "/inference", "headers": {"Host": "abc.execute-api"},
          "queryStringParameters": {"seed": "3"}, "body": None, "isBase64Encoded": False,
          "requestContext": {"identity": {"sourceIp": "1.2.3.4"}}}
    resp = handler(ev, None)
    assert resp["statusCode"] == 200 and not resp["isBase64Encoded"]
    assert "text" in json.loads(resp["body"])["response"]
    assert resp["headers"]["Access-Control-Allow-Origin"] == "*"


def test_lambda_v2_post_base64(client):
    handler = make_handler(app_mod.app)
    x = torch.randn(1, 3, 32, 32)
    body = json.dumps({"model": "resnet18", "tensor_b64": base64.b64encode(x.numpy().tobytes()).decode(),
                       "shape": [1, 3, 32, 32]})
    ev = {"version": "2.0", "rawPath": "/predict", "rawQueryString": "",
          "headers": {"content-type": "application/json"},
          "requestContext": {"http": {"method": "POST", "sourceIp": "5.6.7.8"}},
          "body": base64.b64encode(body.encode()).decode(), "isBase64Encoded": True}
    resp = handler(ev, None)
    assert resp["statusCode"] == 200, resp["body"]
    assert json.loads(resp["body"])["model"] == "resnet18"


def test_keep_warm_event():
    ev = {"source": "aws.events", "detail-type": "Scheduled Event"}
    assert is_keep_warm(ev)
    resp = make_handler(lambda e, s: None)(ev, None)
    assert resp["statusCode"] == 200


def test_environ_multivalue_query():
    env = event_to_environ({"httpMethod": "GET", "path": "/x",
                            "multiValueQueryStringParameters": {"a": ["1", "2"]}, "headers": {}})
    assert env["QUERY_STRING"] == "a=1&a=2"


def test_predict_text_bert(client):
    r = client.post("/predict", json={"model": "bert-base", "input_ids": [[101, 2023, 2003, 102]],
                                      "attention_mask": [[1, 1, 1, 1]]})
    assert r.status_code == 200, r.data
    body = r.json
    assert body["model"] == "bert-base" and len(body["probs"][0]) == 2
    assert abs(sum(body["probs"][0]) - 1.0) < 1e-4
