"""Zappa-compatible Lambda entry point: ``handler(event, context)`` -> any WSGI app.

The reference relied on Zappa's handler (pinned ``zappa==0.47.0``) to turn
API Gateway events into WSGI calls of ``main.app``. This is an in-house equivalent:
  * API Gateway REST (v1 proxy) events: ``httpMethod``, ``path``, ``headers`` /
    ``multiValueHeaders``, ``queryStringParameters`` / ``multiValueQueryStringParameters``,
    ``body``, ``isBase64Encoded``, ``requestContext``;
  * API Gateway HTTP API (v2 payload) events: ``rawPath``, ``rawQueryString``,
    ``requestContext.http.method``, ``cookies``;
  * keep-warm / scheduled events (``source: aws.events`` / ``detail-type: Scheduled Event``)
    — Zappa's keep_warm ping: answered without touching the app (optionally pre-loading
    models, ``HIPZAP_WARM_MODELS``);
  * responses become ``{statusCode, headers, multiValueHeaders, body, isBase64Encoded}``;
    non-text bodies are base64-encoded;
  * one Apache common-log-format access line per request (wsgi-request-logger parity).
"""
from __future__ import annotations

import base64
import io
import logging
import os
import sys
import time
from urllib.parse import urlencode

log = logging.getLogger("hipzap.access")

TEXT_TYPES = ("text/", "application/json", "application/javascript", "application/xml")


def is_keep_warm(event: dict) -> bool:
    return event.get("source") == "aws.events" or event.get("detail-type") == "Scheduled Event"


def _query_string(event: dict) -> str:
    if "rawQueryString" in event:
        return event.get("rawQueryString") or ""
    mv = event.get("multiValueQueryStringParameters")
    if mv:
        return urlencode([(k, v) for k, vs in mv.items() for v in (vs or [])])
    qs = event.get("queryStringParameters") or {}
    return urlencode(qs)


def event_to_environ(event: dict, context=None) -> dict:
    v2 = event.get("version") == "2.0" or "rawPath" in event
    if v2:
        http = event.get("requestContext", {}).get("http", {})
        method = http.get("method", "GET")
        path = event.get("rawPath", "/")
        source_ip = http.get("sourceIp", "127.0.0.1")
    else:
        method = event.get("httpMethod", "GET")
        path = event.get("path", "/")
        source_ip = event.get("requestContext", {}).get("identity", {}).get("sourceIp", "127.0.0.1")
    headers = {}
    for k, vs in (event.get("multiValueHeaders") or {}).items():
        headers[k.lower()] = ",".join(vs or [])
    for k, v in (event.get("headers") or {}).items():
        headers[k.lower()] = v
    if v2 and event.get("cookies"):
        headers["cookie"] = "; ".join(event["cookies"])
    body = event.get("body") or ""
    if event.get("isBase64Encoded"):
        raw = base64.b64decode(body)
    else:
        raw = body.encode("utf-8") if isinstance(body, str) else bytes(body)
    environ = {
        "REQUEST_METHOD": method,
        "SCRIPT_NAME": "",
        "PATH_INFO": path,
        "QUERY_STRING": _query_string(event),
        "SERVER_NAME": headers.get("host", "lambda"),
        "SERVER_PORT": headers.get("x-forwarded-port", "443"),
        "SERVER_PROTOCOL": "HTTP/1.1",
        "REMOTE_ADDR": source_ip,
        "CONTENT_LENGTH": str(len(raw)),
        "CONTENT_TYPE": headers.get("content-type", ""),
        "wsgi.version": (1, 0),
        "wsgi.url_scheme": headers.get("x-forwarded-proto", "https"),
        "wsgi.input": io.BytesIO(raw),
        "wsgi.errors": sys.stderr,
        "wsgi.multithread": False,
        "wsgi.multiprocess": False,
        "wsgi.run_once": False,
        "lambda.event": event,
        "lambda.context": context,
    }
    for k, v in headers.items():
        if k in ("content-type", "content-length"):
            continue
        environ["HTTP_" + k.upper().replace("-", "_")] = v
    return environ


def call_wsgi(app, environ: dict) -> tuple[int, list, bytes]:
    status_headers = {}

    def start_response(status, headers, exc_info=None):
        status_headers["status"] = status
        status_headers["headers"] = headers
        return lambda data: None

    chunks = app(environ, start_response)
    try:
        body = b"".join(chunks)
    finally:
        if hasattr(chunks, "close"):
            chunks.close()
    code = int(status_headers["status"].split()[0])
    return code, status_headers["headers"], body


def wsgi_to_response(code: int, headers: list, body: bytes) -> dict:
    single, multi = {}, {}
    for k, v in headers:
        single[k] = v
        multi.setdefault(k, []).append(v)
    ctype = single.get("Content-Type", "")
    is_text = any(ctype.startswith(t) for t in TEXT_TYPES)
    if is_text:
        payload, b64 = body.decode("utf-8"), False
    else:
        payload, b64 = base64.b64encode(body).decode("ascii"), True
    return {"statusCode": code, "headers": single, "multiValueHeaders": multi, "body": payload,
            "isBase64Encoded": b64}


def make_handler(app):
    def handler(event, context=None):
        if is_keep_warm(event):
            warm = os.environ.get("HIPZAP_WARM_MODELS")
            if warm:
                from .app import get_server
                for name in warm.split(","):
                    get_server().vision(name.strip())
            return {"statusCode": 200, "body": "warm", "headers": {}, "isBase64Encoded": False}
        t0 = time.perf_counter()
        environ = event_to_environ(event, context)
        code, headers, body = call_wsgi(app, environ)
        resp = wsgi_to_response(code, headers, body)
        log.info('%s - - [%s] "%s %s%s %s" %d %d %.1fms', environ["REMOTE_ADDR"],
                 time.strftime("%d/%b/%Y:%H:%M:%S %z"), environ["REQUEST_METHOD"], environ["PATH_INFO"],
                 ("?" + environ["QUERY_STRING"]) if environ["QUERY_STRING"] else "", environ["SERVER_PROTOCOL"],
                 code, len(body), (time.perf_counter() - t0) * 1e3)
        return resp
    return handler


def lambda_handler(event, context=None):
    """Default handler bound to ``hipzap.serve.app.app`` (Zappa ``app_function: main.app``)."""
    from .app import app
    return make_handler(app)(event, context)


handler = lambda_handler
