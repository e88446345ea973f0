"""Persistent conv chain (csrc/conv.hip conv_chain_kernel, HIPZAP_CONV_CHAIN): ResNet-50 layer3 +
layer4 (or layer2..4) as ONE launch with in-launch stage hand-offs must give the per-conv program's
logits (same tiles; only the waves-per-tile K split, hence the fp32 summation order, differs), keep
doing so over many graph replays (the last workgroup resets the stage counters) and under
concurrent contexts, and never hit its bounded-wait timeout."""
import threading

import pytest
import torch

from hipzap.engine.program import ExecContext
from hipzap.models import registry
from hipzap.models.resnet import randomize_bn

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _experiments_lib():
    """The chain kernel is a measured negative (profiles/r3_chain): HZ_EXPERIMENTS library only."""
    from hipzap import _native as N
    if not N.experiments():
        pytest.skip("conv chain: build with python -m hipzap.build --experiments, run with HIPZAP_LIB")
DEV = "cuda:0"


@pytest.fixture(scope="module")
def r50():
    torch.manual_seed(0)
    a = registry.get("resnet50")
    sd = randomize_bn(a.make_model()).eval().state_dict()
    params, kw = a.pack({k: v.to(DEV) for k, v in sd.items()}, torch.device(DEV))
    return a, params, kw


def _ctx(r50, monkeypatch, chain, grid=128):
    a, params, kw = r50
    g = a.build_graph(batch=1, **kw)
    with monkeypatch.context() as m:
        if chain:
            m.setenv("HIPZAP_CONV_CHAIN", chain)
            m.setenv("HIPZAP_CHAIN_GRID", str(grid))
        else:
            m.delenv("HIPZAP_CONV_CHAIN", raising=False)
        return ExecContext(g, params, torch.device(DEV))


def _run(ctx, x, stream=None):
    ctx.input.copy_(x)
    if ctx.captured:
        ctx.replay(stream)
    else:
        ctx.run(stream)
    torch.cuda.synchronize()
    return ctx.output.reshape(-1).clone()


@pytest.mark.parametrize("chain,grid", [("layer3", 128), ("layer3", 64), ("layer2", 256)])
def test_chain_matches_per_conv_program(r50, monkeypatch, chain, grid):
    base = _ctx(r50, monkeypatch, None)
    ch = _ctx(r50, monkeypatch, chain, grid)
    assert ch.chain_info["layers"] >= 26 and ch.chain_info["stages"] >= 17, ch.chain_info
    s = torch.cuda.Stream()
    ch.capture(s)
    for seed in range(12):  # replays: the stage counters must come back to zero every time
        x = torch.randn(1, 3, 224, 224, generator=torch.Generator().manual_seed(seed)).to(DEV)
        y0 = _run(base, x)
        with torch.cuda.stream(s):
            y1 = _run(ch, x, s)
        rel = (y1 - y0).abs().max().item() / y0.abs().max().item()
        assert rel < 2e-2, (seed, rel)
        assert int(y1.argmax()) == int(y0.argmax()) or y0.topk(2).values.diff().abs().item() < 1e-2
    assert ch.chain_error() == 0
    assert int(ch.chain_sync[: ch.chain_stages * 32].abs().sum().item()) == 0  # counters reset


def test_chain_concurrent_contexts(r50, monkeypatch):
    """8 contexts replaying at once on 8 streams (8 chain launches in flight, 128 workgroups each)."""
    base = _ctx(r50, monkeypatch, None)
    ctxs = [_ctx(r50, monkeypatch, "layer3") for _ in range(8)]
    streams = [torch.cuda.Stream() for _ in ctxs]
    for c, s in zip(ctxs, streams):
        c.capture(s)
    xs = [torch.randn(1, 3, 224, 224, generator=torch.Generator().manual_seed(100 + i)).to(DEV) for i in range(8)]
    refs = [_run(base, x) for x in xs]
    for c, x in zip(ctxs, xs):
        c.input.copy_(x)
    torch.cuda.synchronize()
    for _ in range(20):
        for c, s in zip(ctxs, streams):
            c.replay(s)
    torch.cuda.synchronize()
    for c, r in zip(ctxs, refs):
        y = c.output.reshape(-1)
        assert (y - r).abs().max().item() / r.abs().max().item() < 2e-2
        assert c.chain_error() == 0
