"""Zappa ``app_function`` target (``main.app``) and local dev server (``python main.py``).

Parity with the reference entry point (/root/reference/main.py:17, 115-127): exposes the
WSGI ``app``; when run directly it copies ``zappa_settings.json[stage]`` environment
variables into ``os.environ`` and serves on 0.0.0.0:8082.
"""
import os

from hipzap.serve.app import app, serve_threaded  # noqa: F401  (WSGI callable for Zappa / gunicorn / Werkzeug)
from hipzap.serve.lambda_handler import lambda_handler  # noqa: F401

if __name__ == "__main__":
    from hipzap.serve.settings import load_settings
    st = load_settings(stage=os.environ.get("HIPZAP_STAGE", "dev"))
    print(f"hipzap: stage {st.stage}, models bucket {st.models_bucket!r}; serving on {st.host}:{st.port}")
    app.run(host=st.host, port=st.port, debug=False, threaded=serve_threaded())
