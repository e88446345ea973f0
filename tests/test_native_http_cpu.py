"""Native HTTP/1.1 front end (csrc/http.cpp) on the CPU: every request takes the WSGI fallback
(no plan executor here), so this pins the protocol side -- request parsing, keep-alive and
pipelining, bodies split across reads, Connection: close, rejected framings -- and that the
Flask app behind it answers exactly as it does under werkzeug."""
import base64
import http.client
import json
import socket

import numpy as np
import pytest

from hipzap.serve import app as app_mod
from hipzap.serve.native_http import NativeHTTPServer, listening_socket
from hipzap.serve.server import ModelServer
from hipzap.serve.settings import Settings


@pytest.fixture(scope="module")
def server():
    mp = pytest.MonkeyPatch()
    mp.setenv("HIPZAP_RANDOM_WEIGHTS", "1")
    mp.setenv("HIPZAP_LM_VOCAB", "300")
    app_mod.set_server(ModelServer(Settings(default_model="resnet18", lm_words=8), backend="cpu"))
    sock = listening_socket("127.0.0.1", 0)
    srv = NativeHTTPServer(app_mod.app, sock)
    yield srv, sock.getsockname()[1]
    srv.stop()
    sock.close()
    app_mod.set_server(None)
    mp.undo()


def test_routes_and_keep_alive(server):
    srv, port = server
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
    for _ in range(3):  # one connection, several requests
        c.request("GET", "/health")
        r = c.getresponse()
        body = json.loads(r.read())
        assert r.status == 200 and body["status"] == "ok"
        assert r.getheader("Access-Control-Allow-Origin") == "*"
    c.request("GET", "/inference?words=5&seed=1")
    r = c.getresponse()
    assert r.status == 200 and "text" in json.loads(r.read())["response"]
    img = np.random.default_rng(0).integers(0, 256, (224, 224, 3), dtype=np.uint8)
    c.request("POST", "/predict", body=json.dumps({"image_b64": base64.b64encode(img.tobytes()).decode(),
                                                   "shape": [224, 224, 3]}),
              headers={"Content-Type": "application/json"})
    r = c.getresponse()
    out = json.loads(r.read())
    assert r.status == 200 and len(out["top5"][0]) == 5 and r.getheader("X-Timing")
    c.request("GET", "/nope")
    r = c.getresponse()
    r.read()
    assert r.status == 404
    st = srv.stats()
    assert st["wsgi"] >= 6 and st["native"] == 0


def _raw(port, data: bytes, chunks=1) -> bytes:
    s = socket.create_connection(("127.0.0.1", port), timeout=30)
    step = max(1, len(data) // chunks)
    for i in range(0, len(data), step):
        s.sendall(data[i: i + step])
    s.shutdown(socket.SHUT_WR)
    out = b""
    while True:
        k = s.recv(65536)
        if not k:
            break
        out += k
    s.close()
    return out


def test_pipelined_requests_and_split_body(server):
    _, port = server
    body = b'{"words": 1}'
    req = (b"GET /health HTTP/1.1\r\nHost: x\r\n\r\n"
           b"POST /nope HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\nContent-Length: "
           + str(len(body)).encode() + b"\r\n\r\n" + body +
           b"GET /health HTTP/1.1\r\nConnection: close\r\n\r\n")
    out = _raw(port, req, chunks=7)
    assert out.count(b"HTTP/1.1 200") == 2 and out.count(b"HTTP/1.1 404") == 1
    assert out.rstrip().endswith(b"}")


def test_rejected_framing_and_bad_request(server):
    _, port = server
    out = _raw(port, b"POST /predict HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n0\r\n\r\n")
    assert out.startswith(b"HTTP/1.1 411")
    out = _raw(port, b"garbage\r\n\r\n")
    assert out.startswith(b"HTTP/1.1 400")
