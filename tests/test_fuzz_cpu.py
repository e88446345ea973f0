"""Property tests (hypothesis) of host-side invariants: the static arena planner never aliases
two simultaneously live tensors; the Lambda adapter round-trips any query string / body /
header set through a WSGI echo app; the detokenizer never emits a leading space before
no-space tokens."""
import base64
import json

import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from hipzap.engine.graph import Graph, lifetimes, plan_memory
from hipzap.serve.lambda_handler import make_handler

FUZZ = settings(max_examples=60, deadline=None, derandomize=True)


@st.composite
def graphs(draw):
    g = Graph("fuzz")
    live = [g.tensor((draw(st.integers(1, 64)),), torch.bfloat16, "in", external=True)]
    for i in range(draw(st.integers(1, 25))):
        ins = draw(st.lists(st.sampled_from(live), min_size=1, max_size=3))
        out = g.tensor((draw(st.integers(1, 4096)),), draw(st.sampled_from([torch.bfloat16, torch.float32])), f"t{i}")
        kind = draw(st.sampled_from(["conv", "gemm", "fork", "join"]))
        g.add(kind, ins, [out], slot=draw(st.integers(0, 1)))
        live.append(out)
    return g


@FUZZ
@given(graphs())
def test_arena_planner_never_aliases_live_tensors(g):
    offs, total = plan_memory(g)
    life = lifetimes(g)
    items = [(t, offs[t], offs[t] + g.tensors[t].nbytes, *life[t]) for t in life]
    for i, (ta, oa, ea, sa, xa) in enumerate(items):
        assert oa % 256 == 0 and ea <= total
        for (tb, ob, eb, sb, xb) in items[i + 1:]:
            if sa <= xb and sb <= xa:  # lifetimes overlap -> byte ranges must not
                assert ea <= ob or eb <= oa, (ta, tb)
    noreuse, total_nr = plan_memory(g, reuse=False)
    assert total_nr >= total


def _echo(environ, start_response):
    n = int(environ.get("CONTENT_LENGTH") or 0)
    body = environ["wsgi.input"].read(n)
    out = json.dumps({"method": environ["REQUEST_METHOD"], "path": environ["PATH_INFO"],
                      "query": environ.get("QUERY_STRING", ""), "body": base64.b64encode(body).decode(),
                      "hdr": environ.get("HTTP_X_FUZZ", "")}).encode()
    start_response("200 OK", [("Content-Type", "application/json"), ("Content-Length", str(len(out)))])
    return [out]


SAFE = st.text(alphabet=st.characters(min_codepoint=48, max_codepoint=122, blacklist_characters="\\`^[]"),
               min_size=1, max_size=12)


@FUZZ
@given(method=st.sampled_from(["GET", "POST", "PUT"]), path=SAFE.map(lambda s: "/" + s),
       query=st.dictionaries(SAFE, SAFE, max_size=4), body=st.binary(max_size=300), b64=st.booleans(),
       hdr=SAFE, v2=st.booleans())
def test_lambda_adapter_roundtrip(method, path, query, body, b64, hdr, v2):
    handler = make_handler(_echo)
    raw = base64.b64encode(body).decode() if b64 else body.decode("latin-1")
    if v2:
        from urllib.parse import urlencode
        ev = {"version": "2.0", "rawPath": path, "rawQueryString": urlencode(query), "headers": {"x-fuzz": hdr},
              "requestContext": {"http": {"method": method, "sourceIp": "1.1.1.1"}}, "body": raw,
              "isBase64Encoded": b64}
    else:
        ev = {"httpMethod": method, "path": path, "headers": {"X-Fuzz": hdr}, "queryStringParameters": query or None,
              "body": raw, "isBase64Encoded": b64}
    resp = handler(ev, None)
    assert resp["statusCode"] == 200
    got = json.loads(resp["body"])
    assert got["method"] == method and got["path"] == path and got["hdr"] == hdr
    from urllib.parse import parse_qsl
    assert dict(parse_qsl(got["query"])) == query
    sent = body if b64 else body.decode("latin-1").encode("utf-8")
    assert base64.b64decode(got["body"]) == sent


@FUZZ
@given(st.lists(st.sampled_from(["hello", "world", ".", ",", "!", "'s", "n't", "\n", "xxmaj", "it", "?"]),
                min_size=1, max_size=30))
def test_detokenizer_spacing(words):
    from hipzap.serve.text import NO_SPACE, Detokenizer
    det = Detokenizer()
    for w in words:
        det.add(w)
    text = det.text
    for tok in NO_SPACE:  # main.py:75-78: no leading space before these tokens
        assert " " + tok not in text, (words, text)
    assert text.startswith(" ") or words[0] in NO_SPACE
