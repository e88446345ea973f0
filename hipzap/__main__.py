"""hipzap command line: serve | pack | tune | upload | info | bench.

    python -m hipzap serve --port 8082            # local dev server (reference: main.py:115-127)
    python -m hipzap pack --model resnet50 --ckpt m.pth --out m.hzpack
    python -m hipzap plan --model resnet50 --ckpt m.pth [--contexts 24]  # torch-free cold-start image
    python -m hipzap tune --model resnet50 --batch 1 --concurrent 1 8
    python -m hipzap upload --models-dir ./models  # scripts/upload_models.py parity
    python -m hipzap info
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys


def cmd_serve(a):
    from .serve.settings import load_settings
    st = load_settings(a.settings, a.stage)
    host, port = a.host or st.host, a.port or st.port
    if a.gpus and a.gpus > 1:  # one worker process per GPU sharing the listening socket (serve/cluster.py)
        from .serve.cluster import launch
        sys.exit(launch(a.gpus, host, port, settings=a.settings, stage=a.stage))
    from .serve.app import app, serve_threaded, set_server
    from .serve.server import ModelServer, PlanVisionBackend
    srv = ModelServer(st)  # the settings named on the command line, not the default file
    set_server(srv)
    if srv.backend == "gpu" and os.environ.get("HIPZAP_NATIVE_HTTP", "1") != "0":
        # native HTTP/1.1 front end: POST /predict for the plan-backed default model in C++,
        # everything else through the Flask app (serve/native_http.py)
        from .serve.native_http import NativeHTTPServer, listening_socket
        be = srv.vision(st.default_model)  # cold start before the port opens
        fast = be if isinstance(be, PlanVisionBackend) else None
        if os.environ.get("HIPZAP_LM_PRELOAD", "0") == "1":
            srv.lm()  # GET /inference backend before the port opens (else on its first request)
        http = NativeHTTPServer(app, listening_socket(host, port), fast=fast, server=srv)
        print(f"hipzap serving stage {st.stage} on {host}:{port} (native http, fast route: "
              f"{fast.name if fast else None}, native GET /inference: {http.lm_native})", flush=True)
        http.serve_forever()
        return
    from werkzeug.serving import WSGIRequestHandler
    WSGIRequestHandler.protocol_version = "HTTP/1.1"  # keep-alive: no TCP handshake per request
    print(f"hipzap serving stage {st.stage} on {host}:{port} (models bucket {st.models_bucket!r})", flush=True)
    app.run(host=host, port=port, debug=False, threaded=serve_threaded())


def cmd_pack(a):
    import hashlib

    import torch

    from .engine.packfile import save_packed
    from .models import registry
    ad = registry.get(a.model)
    sd = torch.load(a.ckpt, map_location="cpu", weights_only=True)
    params, cfg = ad.pack(sd, "cpu")
    h = hashlib.sha256(open(a.ckpt, "rb").read()).hexdigest()
    save_packed(params, cfg, a.out, h)
    print(json.dumps({"out": a.out, "entries": len(params), "source_sha256": h}))


def cmd_plan(a):
    from .engine.plan import export_from_checkpoint
    from .lite import read_meta
    out = export_from_checkpoint(a.model, a.ckpt, a.out, batch=a.batch, contexts=a.contexts, probs=a.probs,
                                 dp_shard=a.dp_shard)
    m = read_meta(out)
    print(json.dumps({"out": out, "ops": m["n_ops"], "blob_bytes": m["blob_bytes"], "source": m["source"]}))


def cmd_tune(a):
    sys.argv = ["tune", "--model", a.model, "--batch", *map(str, a.batch), "--concurrent", *map(str, a.concurrent)]
    from .engine import tune
    tune.main()


def cmd_upload(a):
    from .serve.artifacts import ArtifactStore
    from .serve.settings import load_settings
    st = load_settings(a.settings, a.stage)
    bucket = a.bucket or st.models_bucket
    if not bucket:
        sys.exit("no models bucket: set aws_environment_variables.models_bucket in zappa_settings.json or --bucket")
    copied = ArtifactStore(bucket).upload_dir(a.models_dir)
    print(json.dumps({"bucket": bucket, "copied": copied}))


def cmd_info(a):
    import torch

    from . import __version__, _native
    from .models import registry
    info = {"version": __version__, "models": registry.names(), "native_library": str(_native._LIB_PATH),
            "native_built": _native.available(), "gpu": torch.cuda.is_available()}
    if torch.cuda.is_available():
        info["devices"] = [torch.cuda.get_device_name(i) for i in range(torch.cuda.device_count())]
    print(json.dumps(info, indent=1))


def cmd_bench(a, rest):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.exit(subprocess.call([sys.executable, os.path.join(root, "bench.py"), *rest]))


def main(argv=None):
    ap = argparse.ArgumentParser(prog="hipzap")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("serve")
    s.add_argument("--host", default=None)
    s.add_argument("--port", type=int, default=None)
    s.add_argument("--stage", default=None)
    s.add_argument("--settings", default=None)
    s.add_argument("--gpus", type=int, default=0, help="> 1: data-parallel cluster, one worker process per GPU")
    p = sub.add_parser("pack")
    p.add_argument("--model", required=True)
    p.add_argument("--ckpt", required=True)
    p.add_argument("--out", required=True)
    pl = sub.add_parser("plan")
    pl.add_argument("--model", required=True)
    pl.add_argument("--ckpt", required=True)
    pl.add_argument("--out", default=None, help="default: <ckpt>.hzplan")
    pl.add_argument("--batch", type=int, default=1)
    pl.add_argument("--contexts", type=int, default=1, help="request concurrency the launch configs are tuned for")
    pl.add_argument("--probs", action="store_true", help="softmax head on device")
    pl.add_argument("--dp-shard", type=int, default=None,
                    help="also write <ckpt>.dp<S>.hzplan: the per-GPU shard program of batched DP requests")
    t = sub.add_parser("tune")
    t.add_argument("--model", default="resnet50")
    t.add_argument("--batch", type=int, nargs="+", default=[1])
    t.add_argument("--concurrent", type=int, nargs="+", default=[1])
    u = sub.add_parser("upload")
    u.add_argument("--models-dir", default="./models")
    u.add_argument("--bucket", default=None)
    u.add_argument("--stage", default=None)
    u.add_argument("--settings", default=None)
    sub.add_parser("info")
    sub.add_parser("bench", add_help=False)
    args, rest = ap.parse_known_args(argv)
    if args.cmd == "bench":
        return cmd_bench(args, rest)
    {"serve": cmd_serve, "pack": cmd_pack, "plan": cmd_plan, "tune": cmd_tune, "upload": cmd_upload, "info": cmd_info}[args.cmd](args)


if __name__ == "__main__":
    main()
