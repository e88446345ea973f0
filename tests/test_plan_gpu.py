"""Plan images on MI355X: the torch-free runtime (hipzap/lite.py -> csrc/plan.cpp) runs the
SAME launches as the torch-built Engine (bitwise-equal logits), contexts are independent and
thread-safe, and a fresh process cold-starts from a plan without importing torch."""
import json
import os
import subprocess
import sys
import threading
import time

import pytest
import torch

from conftest import logits_match

from hipzap.engine.engine import Engine
from hipzap.engine.plan import export_plan
from hipzap.lite import PlanEngine, PlanError
from hipzap.models import registry
from hipzap.models.resnet import randomize_bn

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def r50(tmp_path_factory):
    torch.manual_seed(0)
    a = registry.get("resnet50")
    sd = randomize_bn(a.make_model()).eval().state_dict()
    params, kw = a.pack(sd, "cpu")
    kw = dict(kw, input_uint8=True)
    path = str(tmp_path_factory.mktemp("plan") / "r50.hzplan")
    export_plan("resnet50", params, kw, path, batch=1, contexts=1)
    return sd, kw, path, params


def test_plan_equals_engine_bitwise(r50):
    """Same packed weights (CPU packing, as exported), same launches -> identical logits; the
    engine that packs on the GPU agrees to bf16 rounding of the BN fold."""
    from hipzap.parallel.comm import _rebuild, _tensor_fields
    sd, kw, path, params = r50
    dev = torch.device("cuda:0")
    p_dev = {k: _rebuild(v, {n: t.to(dev) for n, t in _tensor_fields(v)}) for k, v in params.items()}
    eng = Engine("resnet50", p_dev, dev, batch=1, num_contexts=1, arch_kw=kw, host_io=True, zero_copy="all")
    eng_gpu_pack = Engine.from_state_dict("resnet50", sd, dev, batch=1, num_contexts=1,
                                          arch_kw={"input_uint8": True}, host_io=True, zero_copy="all")
    pe = PlanEngine(path, device=0, contexts=1)
    for seed in range(3):
        x = torch.randint(0, 256, (1, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(seed))
        ye = eng.infer(x)
        yp = torch.from_numpy(pe.infer(x.numpy()).copy())
        assert yp.shape == ye.shape == (1, 1000)
        assert logits_match(yp, ye), (yp - ye).abs().max()  # bitwise unless the program has seams
        yg = eng_gpu_pack.infer(x)
        assert (yp - yg).abs().max() / yg.abs().max() < 1e-2
    assert pe.timings["upload_ms"] > 0 and pe.timings["capture_ms"] > 0


def test_plan_contexts_concurrent(r50):
    _, _, path, _ = r50
    pe = PlanEngine(path, device=0, contexts=4, eager_contexts=1)
    assert pe.contexts == 1
    assert pe.ensure_contexts() > 0 and pe.contexts == 4
    xs = [os.urandom(224 * 224 * 3) for _ in range(8)]
    ref = [pe.infer_raw(x, ctx=0) for x in xs]
    got = [None] * len(xs)

    def work(i):
        got[i] = pe.infer_raw(xs[i])

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(xs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert all(logits_match(g, r) for g, r in zip(got, ref))
    assert pe.bench(5) > 0
    with pytest.raises(PlanError):
        pe.infer_raw(b"\0" * 10)


def test_plan_broadcast_fill_hook(r50):
    """read_blob=False + fill_blob: the DP receive path fills the weight blob itself (here by a
    device copy from a plan that did read the file) before the contexts are bound."""
    _, _, path, _ = r50
    src = PlanEngine(path, device=0, contexts=1)
    import ctypes as C
    from hipzap import lite
    nb = C.c_uint64()
    saddr = lite.lib().hz_plan_blob(src._h, C.byref(nb))

    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]

    def fill(addr, n):
        assert n == nb.value
        assert hip.hipMemcpy(addr, saddr, n, 3) == 0  # hipMemcpyDeviceToDevice

    dst = PlanEngine(path, device=0, contexts=1, read_blob=False, fill_blob=fill)
    x = os.urandom(224 * 224 * 3)
    assert logits_match(dst.infer_raw(x), src.infer_raw(x))


def test_fresh_process_cold_start_without_torch(r50):
    _, _, path, _ = r50
    t0 = time.time()
    r = subprocess.run([sys.executable, "-m", "hipzap.coldstart", "plan", path], cwd=ROOT, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["ok"] and not res["torch_imported"]
    ms = (res["t_first"] - t0) * 1e3
    print(f"fresh-process plan cold start {ms:.1f} ms: {res['phases_ms']}")
    assert ms < 20000


def test_engine_executor_concurrent_requests(r50):
    """Engine.infer from many threads goes through the native executor: every caller gets the
    logits of ITS image (same as a 1-context engine), with more callers than contexts."""
    sd, kw, path, params = r50
    dev = torch.device("cuda:0")
    one = Engine.from_state_dict("resnet50", sd, dev, batch=1, num_contexts=1, arch_kw={"input_uint8": True},
                                 host_io=True, zero_copy="all")
    eng = Engine("resnet50", one.params, dev, batch=1, num_contexts=4, arch_kw=dict(one.arch_kw), host_io=True,
                 zero_copy="all")
    xs = [torch.randint(0, 256, (1, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(i))
          for i in range(12)]
    ref = [one.infer(x) for x in xs]
    got = [None] * len(xs)

    def work(i):
        got[i] = eng.infer(xs[i])

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(xs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert eng.executor() is not None and eng.executor().stats()["served"] >= len(xs)
    for g, r in zip(got, ref):
        assert logits_match(g, r)
    wall, lat = eng.serve_bench(5)
    assert wall > 0 and len(lat) == 4 * 5 and min(lat) > 0


def test_plan_shared_context_streams(r50, monkeypatch):
    """HIPZAP_CTX_STREAMS=2 in the native loader: contexts 3.. borrow the first two streams (and
    are captured on the plan's private capture stream); concurrent requests still return the
    single-context logits."""
    _, _, path, _ = r50
    ref_pe = PlanEngine(path, device=0, contexts=1)
    xs = [os.urandom(224 * 224 * 3) for _ in range(8)]
    ref = [ref_pe.infer_raw(x) for x in xs]
    ref_pe.close()
    monkeypatch.setenv("HIPZAP_CTX_STREAMS", "2")
    pe = PlanEngine(path, device=0, contexts=5, eager_contexts=2)
    assert pe.ensure_contexts() > 0 and pe.contexts == 5
    got = [None] * len(xs)

    def work(i):
        got[i] = pe.infer_raw(xs[i])

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(xs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert all(logits_match(g, r) for g, r in zip(got, ref))
    pe.close()
