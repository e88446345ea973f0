"""The native GET /inference route (csrc/http.cpp try_lm) against the Flask route it shadows:
for the same seed and word count the bodies are byte-identical (the detokenizer table -- JSON
fragments, capitalised forms, NO_SPACE / CAPITALIZE_AFTER flags -- comes from the backend's own
vocabulary and the Flask route's encoder); requests the native route does not take (a prompt, a
bad word count) still reach the Flask route."""
import http.client
import json

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def served(tmp_path_factory):
    # the environment is restored after the module: later tests read HIPZAP_RANDOM_WEIGHTS etc.
    mp = pytest.MonkeyPatch()
    for k, v in dict(HIPZAP_RANDOM_WEIGHTS="1", HIPZAP_LM_VOCAB="2000", HIPZAP_BACKEND="gpu",
                     HIPZAP_SETTINGS=str(tmp_path_factory.mktemp("s") / "none.json")).items():
        mp.setenv(k, v)
    from hipzap.serve import app as app_mod
    from hipzap.serve.native_http import NativeHTTPServer, listening_socket
    from hipzap.serve.server import ModelServer
    from hipzap.serve.settings import load_settings
    srv = ModelServer(load_settings(), backend="gpu")
    app_mod.set_server(srv)
    sock = listening_socket("127.0.0.1", 0)
    http_srv = NativeHTTPServer(app_mod.app, sock, server=srv)
    yield app_mod, srv, http_srv, sock.getsockname()[1]
    http_srv.stop()
    app_mod.set_server(None)
    mp.undo()


def _get(port, path):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=120)
    c.request("GET", path)
    r = c.getresponse()
    body = r.read()
    c.close()
    return r.status, dict(r.getheaders()), body


def test_native_route_is_byte_identical_to_the_flask_route(served):
    app_mod, srv, http_srv, port = served
    st, h, body = _get(port, "/inference?seed=7")  # first request: Flask loads the LM, the route turns native
    assert st == 200 and h.get("X-Hipzap-Path") != "native"
    assert http_srv.lm_native
    cl = app_mod.app.test_client()
    for q in ("seed=7", "seed=12345&words=37", "words=200&seed=3", "seed=-5", "seed=999999999999999999"):
        st, h, nb = _get(port, f"/inference?{q}")
        assert st == 200 and h.get("X-Hipzap-Path") == "native", q
        fb = cl.get(f"/inference?{q}").get_data()  # the WSGI route, same engine
        assert nb == fb, (q, nb[:200], fb[:200])
        text = json.loads(nb)["response"]["text"]
        assert text.startswith(" ")
    assert json.loads(_get(port, "/inference?seed=7")[2]) == json.loads(body)  # same seed, same text


def test_requests_the_native_route_does_not_take_reach_flask(served):
    app_mod, srv, http_srv, port = served
    _get(port, "/inference?seed=1")
    st, h, body = _get(port, "/inference?prompt=the%20cat&seed=1")
    assert st == 200 and h.get("X-Hipzap-Path") != "native"
    assert json.loads(body)["response"]["text"].startswith(" the cat")
    st, h, _ = _get(port, "/inference?words=0")
    assert st >= 400 and h.get("X-Hipzap-Path") != "native"
    st, h, _ = _get(port, "/inference?seed=18446744073709551621")  # past 2^63: the Flask route's answer
    assert h.get("X-Hipzap-Path") != "native"
    st, h, body = _get(port, "/inference")  # no seed: a random one, natively
    assert st == 200 and h.get("X-Hipzap-Path") == "native" and json.loads(body)["response"]["text"]
