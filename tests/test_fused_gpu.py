"""Fused ResNet stages (csrc/block.hip, engine/fusion.py) on MI355X: the stem kernel (image ->
normalise -> 7x7/2 conv -> max-pool), the layer1 bottleneck kernel and the weight-streaming
layer2 bottleneck kernel against (a) the per-conv
program of the same packed weights and (b) the fp32 graph oracle, tensor by tensor; graph replay,
batch > 1 and the dispatch count."""
import pytest
import torch

from hipzap.engine import fusion
from hipzap.engine.program import ExecContext
from hipzap.engine.reference import run_graph_reference
from hipzap.models import registry
from hipzap.models.resnet import randomize_bn
from hipzap.ops.conv import from_blocked

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def r50():
    torch.manual_seed(0)
    a = registry.get("resnet50")
    sd = randomize_bn(a.make_model()).eval().state_dict()
    params, kw = a.pack({k: v.to(DEV) for k, v in sd.items()}, torch.device(DEV))
    params_cpu, _ = a.pack(sd, "cpu")
    return a, params, params_cpu, kw


def _read(ctx, tid):
    return from_blocked(ctx.view(tid).reshape(-1), ctx.graph.shape(tid)).float().cpu()


def _run(ctx, x):
    ctx.input.copy_(x.to(ctx.input.device))
    ctx.run()
    torch.cuda.synchronize()


def _rel(a, b):
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-6)


def _fused_tensors(ctx):
    """(tensor id, label) of every tensor a fused kernel writes."""
    return [(f.nodes[-1].outputs[0], f.kind + ":" + str(f.nodes[-1].attrs.get("name", f.nodes[-1].kind)))
            for f in ctx.fused.values()]


@pytest.mark.parametrize("uint8,batch,th,fuse", [(True, 1, 8, "all"), (False, 1, 8, "all"), (True, 3, 8, "all"),
                                                (True, 1, 4, "all"), (True, 2, 4, "all"),
                                                (True, 1, 8, "convpool,bneck"), (False, 2, 8, "convpool,bneck"),
                                                (True, 1, 8, "convpool,bneck,bneck2"), (True, 2, 8, "bneck2")])
def test_fused_matches_per_conv_program_and_oracle(r50, uint8, batch, th, fuse, monkeypatch):
    monkeypatch.setenv("HIPZAP_ARENA_NOREUSE", "1")  # every intermediate stays readable after the run
    monkeypatch.setenv("HIPZAP_BNECK_TH", str(th))  # 8x8 or 4x8 bottleneck output tiles
    a, params, params_cpu, kw = r50
    g = a.build_graph(batch=batch, **dict(kw, input_uint8=uint8))
    fused = ExecContext(g, params, torch.device(DEV), fuse=fuse)
    plain = ExecContext(g, params, torch.device(DEV), fuse="none")
    kinds = [f.kind for f in fused.fused.values()]
    want = fusion.enabled_kinds(fuse)
    expect = (["stem"] if "stem" in want else ["convpool"] if "convpool" in want else []) + \
        ["bneck"] * 3 * ("bneck" in want) + ["bneck2"] * 4 * ("bneck2" in want)
    assert kinds == expect, kinds
    assert plain.fused == {}
    gen = torch.Generator().manual_seed(batch)
    if uint8:
        x = torch.randint(0, 256, (batch, 224, 224, 3), dtype=torch.uint8, generator=gen)
    else:
        x = torch.randn(batch, 3, 224, 224, generator=gen)
    _run(fused, x)
    _run(plain, x)
    ref = run_graph_reference(g, params_cpu, [x])
    for tid, label in _fused_tensors(fused):
        yf, yp, yr = _read(fused, tid), _read(plain, tid), ref[tid].float()
        # same bf16 operands, fp32 accumulation in a different order: within a few bf16 ulps
        assert _rel(yf, yp) < 2e-2, (label, _rel(yf, yp))
        assert _rel(yf, yr) < 2e-2, (label, _rel(yf, yr))
        if label.startswith(("stem", "convpool")):  # same K order as the per-conv kernel: at most 1 ulp apart
            d = (yf - yp).abs() / yp.abs().clamp_min(1e-3)
            assert d.max().item() <= 2 ** -7, label
    lf, lp = fused.output.float().cpu().reshape(batch, -1), plain.output.float().cpu().reshape(batch, -1)
    lr = ref[g.outputs[0]].reshape(batch, -1)
    assert _rel(lf, lr) < 3e-2 and _rel(lf, lp) < 3e-2
    assert torch.equal(lf.argmax(1), lp.argmax(1))


def test_fused_dispatch_count_and_replay(r50):
    a, params, _, kw = r50
    g = a.build_graph(batch=1, **dict(kw, input_uint8=True))
    plain = ExecContext(g, params, torch.device(DEV), fuse="none")
    ctx = ExecContext(g, params, torch.device(DEV), fuse="all")
    # stem 3 -> 1, layer1 and layer2 blocks 3 (first block: 4) -> 1 each
    assert plain.num_ops() - ctx.num_ops() == 16  # (the first blocks' downsample + conv1 were one paired launch)
    assert ctx.num_ops() <= 36
    # default: convpool (-15 with the blocks), the seven layer3/layer4 seams (-7) and the layer3 ->
    # layer4 cross-stage seam (-1; tests/test_seam_gpu.py)
    assert plain.num_ops() - ExecContext(g, params, torch.device(DEV)).num_ops() == 23
    s = torch.cuda.Stream()
    ctx.capture(s)
    eager = ExecContext(g, params, torch.device(DEV), fuse="all")
    for seed in range(3):
        x = torch.randint(0, 256, (1, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(seed))
        _run(eager, x)
        with torch.cuda.stream(s):
            ctx.input.copy_(x.to(DEV))
            ctx.replay(s)
        torch.cuda.synchronize()
        assert torch.equal(eager.output, ctx.output)  # no cross-workgroup state: bitwise across replays


def test_fused_zero_copy_request(r50):
    """The stem reads the uint8 request straight from pinned host memory (zero-copy) and gives the
    bytes the device-copy program gives."""
    a, params, _, kw = r50
    g = a.build_graph(batch=1, **dict(kw, input_uint8=True))
    zc = ExecContext(g, params, torch.device(DEV), host_io=True, zero_copy="all", fuse="all")
    cp = ExecContext(g, params, torch.device(DEV), host_io=True, zero_copy="", fuse="all")
    x = torch.randint(0, 256, (1, 224, 224, 3), dtype=torch.uint8)
    for c in (zc, cp):
        c.host_input.copy_(x)
        c.run()
    torch.cuda.synchronize()
    assert torch.equal(zc.host_output, cp.host_output)


@pytest.mark.parametrize("batch", [2, 8])
def test_layer2_two_images_per_workgroup_is_bitwise_one_image(r50, batch, monkeypatch):
    """Batched programs run the layer2 kernels with two images per workgroup (HzBneckParams.imgs:
    each weight fragment streamed once for both images); per image the arithmetic and its order are
    the one-image kernel's, so every layer2 output and the logits are bitwise equal, and half the
    workgroups are launched."""
    monkeypatch.setenv("HIPZAP_ARENA_NOREUSE", "1")
    a, params, params_cpu, kw = r50
    g = a.build_graph(batch=batch, **dict(kw, input_uint8=True))
    monkeypatch.setenv("HIPZAP_B2_IMG", "2")  # two per workgroup (auto picks two from batch 8)
    two = ExecContext(g, params, torch.device(DEV))
    monkeypatch.setenv("HIPZAP_B2_IMG", "1")
    one = ExecContext(g, params, torch.device(DEV))
    x = torch.randint(0, 256, (batch, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(11))
    _run(two, x)
    _run(one, x)
    b2 = [f for f in two.fused.values() if f.kind == "bneck2"]
    assert len(b2) == 4
    for f in b2:
        tid = f.nodes[-1].outputs[0]
        assert torch.equal(two.view(tid), one.view(tid)), f.nodes[-1].attrs.get("name")
    assert torch.equal(two.output, one.output)
    ref = run_graph_reference(g, params_cpu, [x])[g.outputs[0]].reshape(batch, -1)
    assert _rel(two.output.float().cpu().reshape(batch, -1), ref) < 3e-2
