"""Torch-free cold start from a ``.pth`` on the GPU (hipzap/lite.py PlanEngine.from_checkpoint):
the weights-only reader + weightless plan template + device-side packing (csrc/pack.hip) must
produce the plan image's weight blob byte for byte and the same logits; a fresh process does it
without importing torch (or numpy)."""
import ctypes as C
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import logits_match

from hipzap import hip
from hipzap.engine.plan import export_from_checkpoint
from hipzap.lite import PlanEngine
from hipzap.models.resnet import randomize_bn, resnet18, resnet50

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _blob(eng) -> bytes:
    addr, nb = eng.blob()
    buf = (C.c_char * nb)()
    hip.memcpy(C.addressof(buf), addr, nb, hip.D2H)
    return bytes(buf)


@pytest.mark.parametrize("mk,model", [(resnet50, "resnet50"), (resnet18, "resnet18")])
def test_device_pack_equals_plan_image(tmp_path, mk, model):
    torch.manual_seed(1)
    m = randomize_bn(mk()).eval()
    ckpt = str(tmp_path / f"{model}.pth")
    torch.save(m.state_dict(), ckpt)
    plan = export_from_checkpoint(model, ckpt, str(tmp_path / f"{model}.hzplan"))
    ref = PlanEngine(plan, device=0, contexts=1)
    lite = PlanEngine.from_checkpoint(ckpt, device=0, contexts=1)
    assert lite.timings["raw_MB"] > 10 and "pack_ms" in lite.timings
    assert _blob(lite) == _blob(ref)
    img = os.urandom(224 * 224 * 3)
    assert logits_match(lite.infer_raw(img), ref.infer_raw(img))
    lite.close()
    ref.close()


def test_fresh_process_cold_start_without_torch(tmp_path):
    torch.manual_seed(2)
    ckpt = str(tmp_path / "r50.pth")
    torch.save(randomize_bn(resnet50()).eval().state_dict(), ckpt)
    r = subprocess.run([sys.executable, "-m", "hipzap.coldstart", "pth-lite", ckpt], capture_output=True, text=True,
                       timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["ok"] and not out["torch_imported"] and not out["numpy_imported"], out
    assert out["phases_ms"]["pack_ms"] < 50, out
