"""End-to-end ResNet engine on MI355X: native program vs the graph oracle, hipGraph replay
discipline (replay == eager, new input picked up), concurrent contexts."""
import pytest
import torch

from conftest import logits_match

from hipzap.engine.engine import Engine
from hipzap.engine.program import ExecContext
from hipzap.engine.reference import run_graph_reference
from hipzap.models import registry
from hipzap.models.resnet import randomize_bn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", params=["resnet18", "resnet50"])
def model_sd(request):
    torch.manual_seed(0)
    a = registry.get(request.param)
    m = randomize_bn(a.make_model()).eval()
    return request.param, m, m.state_dict()


@pytest.mark.parametrize("batch", [1, 3])
def test_engine_matches_oracle(model_sd, batch):
    name, m, sd = model_sd
    a = registry.get(name)
    eng = Engine.from_state_dict(name, sd, DEV, batch=batch, num_contexts=1)
    x = torch.randn(batch, 3, 224, 224)
    y = eng.infer(x)
    params_cpu, _ = a.pack(sd, "cpu")
    ref = run_graph_reference(eng.graph, params_cpu, [x])[eng.graph.outputs[0]].reshape(batch, -1)
    rel = (y - ref).abs().max().item() / ref.abs().max().item()
    assert rel < 3e-2, rel
    with torch.no_grad():
        eager = m(x)  # the unfolded fp32 torch model (BN in eval mode)
    rel_e = (y - eager).abs().max().item() / eager.abs().max().item()
    assert rel_e < 3e-2, rel_e
    top3 = eager.topk(3, dim=1).indices
    assert all(int(y[i].argmax()) in top3[i].tolist() for i in range(batch))


def test_graph_replay_equals_eager_and_tracks_input(model_sd):
    name, m, sd = model_sd
    a = registry.get(name)
    params, kw = a.pack({k: v.to(DEV) for k, v in sd.items()}, torch.device(DEV))
    g = a.build_graph(batch=1, **kw)
    ctx_e = ExecContext(g, params, torch.device(DEV))
    ctx_g = ExecContext(g, params, torch.device(DEV))
    s = torch.cuda.Stream()
    ctx_g.capture(s)
    assert ctx_g.captured
    for seed in range(3):
        x = torch.randn(1, 3, 224, 224, generator=torch.Generator().manual_seed(seed)).to(DEV)
        ctx_e.input.copy_(x)
        ctx_e.run()
        with torch.cuda.stream(s):
            ctx_g.input.copy_(x)
            ctx_g.replay(s)
        torch.cuda.synchronize()
        assert logits_match(ctx_g.output, ctx_e.output)  # bitwise unless the program has seams


def test_concurrent_contexts(model_sd):
    name, m, sd = model_sd
    eng = Engine.from_state_dict(name, sd, DEV, batch=1, num_contexts=4)
    xs = [torch.randn(1, 3, 224, 224) for _ in range(4)]
    singles = [eng.infer(x) for x in xs] + [eng.infer(x) for x in xs]
    for i in range(4):
        assert logits_match(singles[i + 4], singles[i])
    secs = eng.bench(20)
    assert secs > 0


def test_deferred_contexts(model_sd):
    """eager_contexts=1: one context serves the first request; ensure_contexts (and bench) build
    the rest, which produce the same logits."""
    name, m, sd = model_sd
    eng = Engine.from_state_dict(name, sd, DEV, batch=1, num_contexts=3, eager_contexts=1)
    assert len(eng.contexts) == 1
    x = torch.randn(1, 3, 224, 224)
    y0 = eng.infer(x)
    assert eng.ensure_contexts() > 0 and len(eng.contexts) == len(eng.streams) == len(eng._locks) == 3
    assert eng.ensure_contexts() == 0.0
    for _ in range(3):
        assert logits_match(eng.infer(x), y0)
    assert eng.bench(5) > 0


def test_probs_head(model_sd):
    """Engine(probs=True): on-device softmax over the logits (csrc/transformer.hip softmax_kernel)."""
    name, m, sd = model_sd
    x = torch.randn(1, 3, 224, 224)
    logits = Engine.from_state_dict(name, sd, DEV, batch=1).infer(x)
    probs = Engine.from_state_dict(name, sd, DEV, batch=1, probs=True).infer(x)
    assert probs.shape == logits.shape
    assert torch.allclose(probs.sum(1), torch.ones(1), atol=1e-4)
    assert (probs - torch.softmax(logits.float(), 1)).abs().max().item() < 1e-5


def test_uint8_image_requests(model_sd):
    """bench.py's default payload: uint8 HWC images normalised on device (preprocess kernel)."""
    name, m, sd = model_sd
    a = registry.get(name)
    params, kw = a.pack({k: v.to(DEV) for k, v in sd.items()}, torch.device(DEV))
    eng = Engine(name, params, DEV, batch=1, arch_kw=dict(kw, input_uint8=True))
    img = torch.randint(0, 256, (1, 224, 224, 3), dtype=torch.uint8)
    y = eng.infer(img)
    params_cpu, _ = a.pack(sd, "cpu")
    ref = run_graph_reference(eng.graph, params_cpu, [img])[eng.graph.outputs[0]].reshape(1, -1)
    assert (y - ref).abs().max().item() / ref.abs().max().item() < 3e-2
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    with torch.no_grad():
        eager = m((img.permute(0, 3, 1, 2).float() / 255 - mean) / std)
    assert y.argmax(1).item() == eager.argmax(1).item()


@pytest.mark.parametrize("zc", ["in", "out", "all"])
def test_zero_copy_host_io(model_sd, zc):
    """Kernels reading the request from / writing logits to pinned host memory (no copy nodes)
    give the same result as the copy-node program, across several replays."""
    name, m, sd = model_sd
    base = Engine.from_state_dict(name, sd, DEV, batch=1, zero_copy="")
    eng = Engine.from_state_dict(name, sd, DEV, batch=1, zero_copy=zc)
    for seed in range(3):
        x = torch.randn(1, 3, 224, 224, generator=torch.Generator().manual_seed(seed))
        assert logits_match(eng.infer(x), base.infer(x))


def test_dynamic_batching_backend(model_sd):
    """serve/batcher.py on the GPU: concurrent bs=1 requests coalesced into one batch-4
    replay return the same logits as the same engine run on each request alone."""
    import threading
    from hipzap.serve.server import VisionBackend
    from hipzap.serve.settings import ModelSpec
    name, m, sd = model_sd
    be = VisionBackend(name, sd, "gpu", DEV, ModelSpec(name, batch=4, contexts=1,
                                                         extra={"batching": {"max_wait_ms": 50}}), True)
    assert be.batcher is not None
    xs = [torch.randn(1, 3, 224, 224, generator=torch.Generator().manual_seed(s)) for s in range(4)]
    solo = [be._run_padded(x) for x in xs]  # batch-4 replay with three zero rows
    out = [None] * 4
    bar = threading.Barrier(4)

    def run(i):
        bar.wait()
        out[i] = be(xs[i])
    th = [threading.Thread(target=run, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    for a, b in zip(out, solo):
        assert logits_match(a, b)  # rows are independent: same kernels, same result per row
    assert be.batcher.batches < 4  # at least two requests shared a replay
    be.batcher.close()


def test_checkpoint_packed_fast_path(model_sd, tmp_path):
    """Engine.from_checkpoint: first cold start packs from the .pth and writes <ckpt>.hzpack; the
    next one streams the packed file straight to the GPU and gives identical logits."""
    from hipzap.engine.packfile import packed_path
    name, m, sd = model_sd
    ck = str(tmp_path / f"{name}.pth")
    torch.save(sd, ck)
    first = Engine.from_checkpoint(name, ck, DEV, batch=1, write_packed=True)
    assert "pack_ms" in first.timings
    import os
    assert os.path.exists(packed_path(ck))
    fast = Engine.from_checkpoint(name, ck, DEV, batch=1)
    assert "load_packed_ms" in fast.timings and "pack_ms" not in fast.timings
    x = torch.randn(1, 3, 224, 224)
    assert logits_match(first.infer(x), fast.infer(x))


def test_shared_context_streams_bitwise(monkeypatch):
    """HIPZAP_CTX_STREAMS=2: 6 request contexts share 2 streams (captured on a private stream,
    replayed on the shared one) and return the same logits as one stream per context."""
    from hipzap.models.resnet import randomize_bn
    torch.manual_seed(0)
    sd = randomize_bn(registry.get("resnet18").make_model()).eval().state_dict()
    x = torch.randn(1, 3, 224, 224)
    monkeypatch.setenv("HIPZAP_CTX_STREAMS", "0")
    ref = Engine.from_state_dict("resnet18", sd, "cuda:0", batch=1, num_contexts=2).infer(x)
    monkeypatch.setenv("HIPZAP_CTX_STREAMS", "2")
    eng = Engine.from_state_dict("resnet18", sd, "cuda:0", batch=1, num_contexts=6)
    eng.ensure_contexts()
    assert len({s.cuda_stream for s in eng.streams}) == 2
    outs = [eng.infer(x) for _ in range(12)]
    assert all(logits_match(o, ref) for o in outs)


@pytest.mark.parametrize("arch,dtype", [("resnet50", torch.float32), ("resnet18", torch.float32),
                                        ("resnet50", torch.bfloat16)])
def test_native_resnet_pack_is_bitwise_the_torch_pack(arch, dtype):
    """pack_resnet's GPU default (csrc/pack.hip: BN fold in IEEE fp32 with the float64-rounded
    scale, OIHW -> [cout][R*S*Cin_pad], RNE bf16, fragment-major) writes the torch-op packer's
    bytes for every conv and the FC (also from a bf16 checkpoint)."""
    from hipzap.models.resnet import pack_resnet, randomize_bn, resnet18, resnet50
    torch.manual_seed(3)
    m = randomize_bn((resnet50 if arch == "resnet50" else resnet18)()).eval()
    sd = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in m.state_dict().items()}
    a = pack_resnet(sd, "cuda:0", native=False)
    b = pack_resnet(sd, "cuda:0", native=True)
    assert list(a) == list(b)
    for k in a:
        pa, pb = a[k], b[k]
        assert (pa.cin, pa.cout, pa.r, pa.s, pa.stride, pa.pad) == (pb.cin, pb.cout, pb.r, pb.s, pb.stride, pb.pad), k
        assert pa.wf.shape == pb.wf.shape and torch.equal(pa.wf.view(torch.int16), pb.wf.view(torch.int16)), k
        assert torch.equal(pa.bias, pb.bias), k
