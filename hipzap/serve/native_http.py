"""Serve the WSGI app through the native HTTP/1.1 front end (csrc/http.cpp).

The hot route -- ``POST /predict`` with one uint8 image of a plan-backed model's shape (JSON
``image_b64``/``shape`` or an ``.npy`` body) -- is answered in C++ straight through the request
executor, without the GIL. Every other request is handed to the Flask app through a ctypes
callback that builds a WSGI environ (the same adapter the Lambda handler uses), so behaviour
and the Zappa contract are unchanged; only the throughput of the hot route is.
"""
from __future__ import annotations

import ctypes as C
import io
import logging
import socket
import sys
import threading
from urllib.parse import unquote

from .. import _native as N

log = logging.getLogger("hipzap.http")

_LEAKED: list = []  # executors a stopped server may still reference (never freed)
_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_uint64, C.c_void_p, C.c_uint64)


def listening_socket(host: str, port: int, backlog: int = 1024) -> socket.socket:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.bind((host, port))
    s.listen(backlog)
    return s


def _environ(method: str, target: str, headers: str, body: bytes, server_port: str) -> dict:
    path, _, query = target.partition("?")
    env = {
        "REQUEST_METHOD": method, "SCRIPT_NAME": "", "PATH_INFO": unquote(path), "QUERY_STRING": query,
        "SERVER_NAME": "hipzap", "SERVER_PORT": server_port, "SERVER_PROTOCOL": "HTTP/1.1",
        "REMOTE_ADDR": "127.0.0.1", "CONTENT_LENGTH": str(len(body)), "CONTENT_TYPE": "",
        "wsgi.version": (1, 0), "wsgi.url_scheme": "http", "wsgi.input": io.BytesIO(body),
        "wsgi.errors": sys.stderr, "wsgi.multithread": True, "wsgi.multiprocess": False, "wsgi.run_once": False,
    }
    for line in headers.split("\r\n"):
        k, sep, v = line.partition(":")
        if not sep:
            continue
        k, v = k.strip().lower(), v.strip()
        if k == "content-type":
            env["CONTENT_TYPE"] = v
        elif k != "content-length":
            env["HTTP_" + k.upper().replace("-", "_")] = v
    return env


def lm_route_table(itos) -> tuple[bytes, bytes]:
    """The native GET /inference detokenizer table (csrc/http.cpp ``Lm``): per word its JSON-escaped
    form and that of its ``str.capitalize()`` (the Flask route's encoder, ``json.dumps``), NUL
    separated, and a flag byte: bit0 word in NO_SPACE, bit1 capitalised form in NO_SPACE, bit2 word
    in CAPITALIZE_AFTER, bit3 capitalised form in CAPITALIZE_AFTER (serve/text.py Detokenizer)."""
    import json
    from .text import CAPITALIZE_AFTER, NO_SPACE
    ns, ca = set(NO_SPACE), set(CAPITALIZE_AFTER)
    parts, flags = [], bytearray(len(itos))
    for i, w in enumerate(itos):
        c = w.capitalize()
        parts.append(json.dumps(w)[1:-1].encode() + b"\0" + json.dumps(c)[1:-1].encode() + b"\0")
        flags[i] = (w in ns) | ((c in ns) << 1) | ((w in ca) << 2) | ((c in ca) << 3)
    return b"".join(parts), bytes(flags)


def render_with_table(blob: bytes, flags: bytes, ids) -> str:
    """What csrc/http.cpp try_lm writes inside ``"text": "..."`` for the empty prompt (a Python
    mirror of its loop, for the CPU test against the Detokenizer)."""
    ents = blob.split(b"\0")[:-1]
    w, wc = ents[0::2], ents[1::2]
    out, cap = [b" "], False
    for t in ids:
        f = flags[t]
        if not f & (2 if cap else 1):
            out.append(b" ")
        out.append(wc[t] if cap else w[t])
        cap = bool(f & (8 if cap else 4))
    return b"".join(out).decode()


class NativeHTTPServer:
    """``app``: any WSGI app (the Flask app). ``sock``: a listening socket (shared by cluster
    workers). ``fast``: a :class:`~hipzap.serve.server.PlanVisionBackend` whose model gets the
    native ``POST /predict`` route (its contexts are built first so the executor covers them)."""

    def __init__(self, app, sock: socket.socket, fast=None, server=None):
        from .lambda_handler import call_wsgi
        self.app, self.sock = app, sock
        self._call_wsgi = call_wsgi
        self._port = str(sock.getsockname()[1])
        self._cb = _CB(self._handle)  # keep a reference: the C side calls it from its threads
        self.fast_model = None
        self._stopped = threading.Event()
        # the fast route's executor is built BEFORE the port accepts anything: a /predict that
        # reached the WSGI fallback first could otherwise build the other executor kind over the
        # same contexts
        ex = self._prepare_fast(fast) if fast is not None else None
        self._h = N.lib().hz_http_start(sock.fileno(), self._cb)
        if not self._h:
            raise RuntimeError("hz_http_start failed")
        if fast is not None:
            self._route_fast(fast, ex)
        self.lm_native = False
        if server is not None:  # GET /inference goes native once the LM backend exists
            server.lm_listeners.append(self.set_lm)
            loaded = server._models.get("__lm__")
            if loaded is not None:
                self.set_lm(loaded)

    @staticmethod
    def _prepare_fast(backend):
        eng = backend.engine
        eng.ensure_contexts()
        b = backend.in_shape[0]
        # a batch-B plan is served with dynamic batching: each POST is one row of a shared replay
        ex = eng.executor() if b == 1 else eng.batched_executor(getattr(backend, "max_wait_us", 200.0))
        if ex is None:
            raise RuntimeError("plan engine has no executor (capture disabled?)")
        return ex

    def set_fast(self, backend) -> None:
        self._route_fast(backend, self._prepare_fast(backend))

    def _route_fast(self, backend, ex) -> None:
        eng = backend.engine
        b, h, w, c = backend.in_shape
        self._exec = ex  # keep alive
        self._fast_engine = eng
        out = eng.out_spec
        rc = N.lib().hz_http_set_fast(self._h, ex._h, h, w, c, out["bytes"] // b // 4, int(backend.num_labels),
                                      int(backend.probs), backend.name.encode())
        if rc:
            raise RuntimeError(f"native /predict route rejected (rc={rc}, plan batch {b})")
        self.fast_model = backend.name

    def set_lm(self, backend) -> bool:
        """Route ``GET /inference`` natively (csrc/http.cpp try_lm) over ``backend``'s batched
        decode scheduler. The detokenizer's table is computed here from the backend's own
        vocabulary with the Flask route's rules and its JSON encoder, so the native body is
        byte-for-byte the WSGI one for the same seed: per word its JSON-escaped form and that of
        its ``str.capitalize()`` (serve/text.py Detokenizer), and whether each form is in
        ``NO_SPACE`` / ``CAPITALIZE_AFTER``. Backends without a batched scheduler (the CPU model,
        the context pool) stay on the WSGI route. Returns whether the route is native."""
        core = getattr(getattr(backend, "engine", None), "core", None)
        sched = getattr(core, "_sched", None)
        if not sched or not getattr(self, "_h", None):
            return False
        itos, stoi = backend.itos, backend.stoi
        V = int(core.V)
        if len(itos) < V:
            return False
        blob, flags = lm_route_table(itos[:V])
        from .app import get_server
        dflt = int(get_server().settings.lm_words)
        rc = N.lib().hz_http_set_lm(self._h, sched, V, int(core.max_words), dflt, int(stoi.get("", 0)), blob,
                                    len(blob), bytes(flags))
        if rc:
            log.warning("native GET /inference route rejected (rc=%d)", rc)
            return False
        self._lm_backend = backend  # keep its scheduler alive while the route points at it
        self.lm_native = True
        return True

    def _handle(self, req, method, target, headers, hlen, body_ptr, blen):
        try:
            body = C.string_at(body_ptr, blen) if blen else b""
            env = _environ(method.decode(), target.decode(), C.string_at(headers, hlen).decode("latin-1"), body,
                           self._port)
            code, hdrs, out = self._call_wsgi(self.app, env)
            lines = "".join(f"{k}: {v}\r\n" for k, v in hdrs if k.lower() not in ("content-length", "connection"))
            lines += f"Content-Length: {len(out)}\r\n"
            raw = lines.encode("latin-1")
            N.lib().hz_http_respond(req, code, raw, len(raw), out, len(out))
        except Exception as e:  # noqa: BLE001 - must answer; the C side waits for the response
            log.exception("native http callback failed")
            msg = ('{"error": "%s"}' % type(e).__name__).encode()
            hdr = f"Content-Type: application/json\r\nContent-Length: {len(msg)}\r\n".encode()
            N.lib().hz_http_respond(req, 500, hdr, len(hdr), msg, len(msg))

    def stats(self) -> dict:
        a = (C.c_uint64 * 4)()
        N.lib().hz_http_stats(self._h, a)
        return {"native": a[0], "wsgi": a[1], "rejected": a[2], "open_connections": a[3]}

    def serve_forever(self) -> None:
        try:
            while not self._stopped.wait(0.5):
                pass
        except KeyboardInterrupt:
            pass
        finally:
            self.stop()

    def stop(self) -> None:
        h, self._h = getattr(self, "_h", None), None
        self._stopped.set()
        if h and not N.lib().hz_http_stop(h):
            # a connection thread is still live and may be inside the executor: never free it, nor
            # the plan whose contexts and pinned slots it submits to. Disarm both handles so a later
            # engine close() (PlanEngine.close -> ex.close, hz_plan_close) cannot destroy them.
            ex, eng = getattr(self, "_exec", None), getattr(self, "_fast_engine", None)
            if ex is not None:
                ex._h = None
            if eng is not None and hasattr(eng, "_h"):
                eng._h = None
            _LEAKED.append((ex, eng))
            log.warning("native http: connections still open at stop; executor and plan kept alive")
