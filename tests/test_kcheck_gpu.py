"""DEBUG kernel variant (csrc/common.h HZ_DCHECK, hipzap/utils/kcheck.py): on MI355X the checked
library runs whole models with no contract failure, gives the same logits as the release
library, and reports (not faults on) a deliberately inconsistent launch.

Runs in a child process because HIPZAP_DEBUG selects the library at import time (this test
process already holds the release one). libhipzap_debug.so is built in-tree beforehand
(`python -m hipzap.build --debug`, also done by __graft_entry__.build()).
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent

CHILD = r"""
import json, torch
from hipzap import _native as N
from hipzap.engine.engine import Engine
from hipzap.models import registry
from hipzap.models.resnet import randomize_bn
from hipzap.ops import conv as cv
from hipzap.utils import kcheck

import os
assert N.DEBUG and os.path.basename(N._LIB_PATH) == "libhipzap_debug.so", N._LIB_PATH
res = {}
torch.manual_seed(0)
dev = "cuda:0"
# 1) a correct conv launch: no failure recorded
w = torch.randn(64, 64, 3, 3) * 0.05
pc = cv.pack_conv(w.to(dev), torch.zeros(64, device=dev), stride=1, pad=1)
x = torch.randn(2, 14, 14, 64, device=dev).bfloat16()
cv.conv2d_nhwc(x, pc)
res["clean_conv"] = kcheck.poll()
# 2) an inconsistent launch: the params claim 1 image while M covers 2 -> the contract check
#    records it and the tile returns before touching memory (no fault)
cfg, kw = cv.choose_config(2 * 14 * 14, pc.cout, pc.K)
xb = cv.to_blocked(x)
out = torch.zeros(2 * 14 * 14 * 64, device=dev, dtype=torch.bfloat16)
prm, _, _ = cv.make_params(xb.data_ptr(), pc, 2, 14, 14, out.data_ptr(), 0, "relu", False, cfg, kw)
prm.N = 1
N.check(N.lib().hz_conv_launch(prm, cfg, N.stream_ptr()), "hz_conv_launch")
res["bad_conv"] = kcheck.poll()
res["bad_conv_untouched"] = bool((out == 0).all().item())
# 3) whole models under the checked kernels (Engine.infer raises KernelCheckError on a failure)
for name in ("resnet50", "bert-base", "vit-b16"):
    a = registry.get(name)
    m = a.make_model()
    if name == "resnet50":
        m = randomize_bn(m)
    sd = m.eval().state_dict()
    eng = Engine.from_state_dict(name, sd, dev, batch=2, num_contexts=1)
    y = eng.infer(a.example_input(2))
    res[name] = {"finite": bool(torch.isfinite(y).all().item()), "fails": kcheck.poll()}
print("RESULT " + json.dumps(res))
"""


def test_debug_variant_checks_and_reports():
    lib = ROOT / "hipzap" / "_lib" / "libhipzap_debug.so"
    assert lib.exists(), "build it first: python -m hipzap.build --debug"
    env = dict(os.environ, HIPZAP_DEBUG="1", HIPZAP_NO_AUTOBUILD="1")
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    assert res["clean_conv"] == []
    assert len(res["bad_conv"]) == 1 and res["bad_conv"][0]["unit"] == "conv", res["bad_conv"]
    assert res["bad_conv"][0]["count"] >= 1
    assert res["bad_conv_untouched"]
    for name in ("resnet50", "bert-base", "vit-b16"):
        assert res[name]["finite"] and res[name]["fails"] == [], (name, res[name])
