"""CPU checks of the vision lowering: packing, layouts, memory planning, graph oracle vs eager."""
import pytest
import torch

from hipzap.engine.graph import Graph, lifetimes, plan_memory
from hipzap.engine.reference import run_graph_reference
from hipzap.models import registry
from hipzap.models.resnet import ResNet, build_graph, infer_arch, pack_resnet, randomize_bn
from hipzap.ops import conv as C


def test_fragment_major_roundtrip():
    w = torch.randn(70, 3, 7, 7)
    pc = C.pack_conv(w, None, None, 2, 3, cin_pad=8)
    assert pc.wf.shape == (128 // 16, 13, 64, 8)  # rows padded to 128 (ROW_PAD 64), K 392 -> 13 steps
    d = pc.dense().reshape(70, 7, 7, 8)
    assert torch.allclose(d[..., :3].permute(0, 3, 1, 2), w.to(torch.bfloat16).float())
    assert torch.count_nonzero(d[..., 3:]) == 0
    # lane mapping: lane = kc*16 + row, element e -> k = s*32 + kc*8 + e
    wf = pc.wf.float()
    dense_full = torch.zeros(wf.shape[0] * 16, wf.shape[1] * 32)
    dense_full[:70, :pc.K] = pc.dense()
    g, s, lane, e = 1, 2, 37, 5
    kc, row = divmod(lane, 16)
    assert wf[g, s, lane, e] == dense_full[g * 16 + row, s * 32 + kc * 8 + e]


def test_bn_folding_matches_eager():
    g = torch.Generator().manual_seed(0)
    conv = torch.nn.Conv2d(16, 32, 3, 1, 1, bias=False)
    bn = torch.nn.BatchNorm2d(32).eval()
    bn.running_mean.data = torch.randn(32, generator=g)
    bn.running_var.data = torch.rand(32, generator=g) + 0.5
    bn.weight.data = torch.randn(32, generator=g)
    x = torch.randn(1, 16, 8, 8, generator=g)
    ref = bn(conv(x))
    w, b = C.fold_bn(conv.weight, None, {k: getattr(bn, k) for k in ("weight", "bias", "running_mean", "running_var")})
    assert torch.allclose(torch.nn.functional.conv2d(x, w, b, padding=1), ref, atol=1e-4)


def test_blocked_layout_roundtrip():
    x = torch.randn(2, 5, 7, 96)
    b = C.to_blocked(x)
    assert b.shape == (2, 3, 5, 7, 32)
    assert torch.equal(C.from_blocked(b, x.shape), x)
    y = torch.randn(1, 4, 4, 8)
    assert C.to_blocked(y).data_ptr() == y.data_ptr() or torch.equal(C.to_blocked(y), y)


def test_choose_config_legal():
    for M, N, K in [(12544, 64, 392), (49, 512, 4608), (1, 1000, 2048), (3136, 256, 64), (196, 1024, 256)]:
        cfg, kw = C.choose_config(M, N, K)
        assert C.legal(cfg, kw)
        for c, k in C.candidates(M, N, K):
            assert C.legal(c, k)


def test_memory_plan_no_overlap_of_live_tensors():
    g = build_graph("resnet50", 1)
    off, total = plan_memory(g)
    life = lifetimes(g)
    items = [(t, off[t], off[t] + g.tensors[t].nbytes, life[t]) for t in off]
    for i in range(len(items)):
        for j in range(i + 1, len(items)):
            a, b = items[i], items[j]
            live = a[3][0] <= b[3][1] and b[3][0] <= a[3][1]
            mem = a[1] < b[2] and b[1] < a[2]
            assert not (live and mem), (g.tensors[a[0]].name, g.tensors[b[0]].name)
    assert total < 8 * 2**20  # bs=1 ResNet-50 activations fit in a few MB with reuse


def test_side_stream_windows_extend_lifetimes():
    g = build_graph("resnet50", 1, side_stream=True)
    life = lifetimes(g)
    forks = [i for i, n in enumerate(g.nodes) if n.kind == "fork"]
    joins = [i for i, n in enumerate(g.nodes) if n.kind == "join"]
    assert len(forks) == len(joins) == 4
    ds = [n for n in g.nodes if n.kind == "conv" and "downsample" in n.attrs["w"]]
    assert all(n.slot == 1 for n in ds)
    for t in (n.outputs[0] for n in ds):
        s, e = life[t]
        assert any(s <= f and e >= j for f, j in zip(forks, joins))


@pytest.mark.parametrize("arch", ["resnet18", "resnet50"])
def test_graph_oracle_matches_eager(arch):
    torch.manual_seed(0)
    m = randomize_bn(ResNet(arch)).eval()
    sd = m.state_dict()
    assert infer_arch(sd) == (arch, 1000)
    P = pack_resnet(sd)
    g = build_graph(arch, 2)
    x = torch.randn(2, 3, 224, 224)
    with torch.no_grad():
        ref = m(x)
    out = run_graph_reference(g, P, [x], bf16_acts=False)[g.outputs[0]].reshape(2, -1)
    # only weight rounding to bf16 differs
    assert (out - ref).abs().max() / ref.abs().max() < 2e-2
    assert (out.argmax(1) == ref.argmax(1)).all()


def test_meta_params_match_real_packing():
    a = registry.get("resnet18")
    meta, kw = a.meta_params()
    real = pack_resnet(randomize_bn(a.make_model()).state_dict())
    assert set(meta) == set(real)
    for k in meta:
        assert meta[k].wf.shape == real[k].wf.shape and meta[k].bias.shape == real[k].bias.shape


def test_softmax_head_oracle():
    """Engine(probs=True) appends a row-softmax node over the logical classes."""
    from hipzap.engine.engine import add_softmax_head
    torch.manual_seed(0)
    m = randomize_bn(ResNet("resnet18")).eval()
    P = pack_resnet(m.state_dict())
    g = build_graph("resnet18", 2)
    logits_t = g.outputs[0]
    add_softmax_head(g)
    assert g.nodes[-1].kind == "softmax" and g.outputs[0] != logits_t
    x = torch.randn(2, 3, 224, 224)
    vals = run_graph_reference(g, P, [x], bf16_acts=False)
    probs = vals[g.outputs[0]].reshape(2, -1)
    assert probs.shape == (2, 1000)
    assert torch.allclose(probs.sum(1), torch.ones(2), atol=1e-5)
    assert torch.allclose(probs, torch.softmax(vals[logits_t].reshape(2, -1).float(), 1), atol=1e-6)
