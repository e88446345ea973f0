"""End-to-end: boot the dev server as a subprocess, hit it over HTTP (CPU backend)."""
import json
import os
import socket
import subprocess
import sys
import time
import urllib.request

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
def test_dev_server_subprocess():
    port = _port()
    env = dict(os.environ, HIPZAP_RANDOM_WEIGHTS="1", HIPZAP_LM_VOCAB="300", HIPZAP_LM_WORDS="8",
               HIPZAP_PORT=str(port), HIPZAP_BACKEND="cpu", HIPZAP_SETTINGS="/nonexistent")
    proc = subprocess.Popen([sys.executable, "main.py"], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                            stderr=subprocess.STDOUT)
    try:
        base = f"http://127.0.0.1:{port}"
        for _ in range(300):
            try:
                urllib.request.urlopen(base + "/health", timeout=1)
                break
            except Exception:
                time.sleep(0.2)
        else:
            raise AssertionError("server did not come up")
        body = json.loads(urllib.request.urlopen(base + "/inference?seed=2", timeout=60).read())
        assert "text" in body["response"]
        req = urllib.request.Request(base + "/predict", data=json.dumps(
            {"model": "resnet18", "inputs": [[[[0.0] * 32] * 32] * 3]}).encode(),
            headers={"Content-Type": "application/json"})
        out = json.loads(urllib.request.urlopen(req, timeout=120).read())
        assert len(out["top5"][0]) == 5
    finally:
        proc.terminate()
        proc.wait(timeout=30)
