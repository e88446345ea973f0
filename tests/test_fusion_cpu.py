"""Bind-time fusion planning (engine/fusion.py) on the CPU: which node runs of the ResNet graphs
become one fused launch for each HIPZAP_FUSE spec, and which do not (the kernels themselves are
checked on the GPU, tests/test_fused_gpu.py)."""
import pytest
import torch

from hipzap.engine import fusion
from hipzap.models import registry
from hipzap.models.resnet import randomize_bn


@pytest.fixture(scope="module")
def r50():
    torch.manual_seed(0)
    a = registry.get("resnet50")
    params, kw = a.pack(randomize_bn(a.make_model()).eval().state_dict(), "cpu")
    return a, params, kw


def _plan(a, params, kw, spec, **gkw):
    g = a.build_graph(**dict(kw, **gkw))
    return g, fusion.plan(g, params, fusion.enabled_kinds(spec))


@pytest.mark.parametrize("spec,expect", [
    ("none", []),
    ("convpool,bneck", ["convpool"] + ["bneck"] * 3),
    ("all", ["stem"] + ["bneck"] * 3 + ["bneck2"] * 4),
    ("bneck2", ["bneck2"] * 4),
    ("convpool,bneck,bneck2", ["convpool"] + ["bneck"] * 3 + ["bneck2"] * 4),
])
def test_resnet50_runs(r50, spec, expect):
    a, params, kw = r50
    g, fz = _plan(a, params, kw, spec, batch=1, input_uint8=True)
    assert [f.kind for f in fz.values()] == expect
    for i, f in fz.items():
        assert f.start == i and g.nodes[f.start:f.end] == f.nodes
    # fused runs never overlap and keep graph order
    spans = sorted((f.start, f.end) for f in fz.values())
    assert all(e <= s2 for (_, e), (s2, _) in zip(spans, spans[1:]))


def test_resnet50_block_shapes(r50):
    a, params, kw = r50
    g, fz = _plan(a, params, kw, "all", batch=2, input_uint8=False)
    b1 = [f for f in fz.values() if f.kind == "bneck"]
    b2 = [f for f in fz.values() if f.kind == "bneck2"]
    assert [len(f.nodes) for f in b1] == [4, 3, 3]  # the first layer1 block carries its downsample
    assert [len(f.nodes) for f in b2] == [4, 3, 3, 3]  # layer2: the first block with its downsample
    assert g.shape(b2[0].nodes[1].inputs[0]) == (2, 56, 56, 256)
    for f in b2:
        assert g.shape(f.nodes[-1].outputs[0]) == (2, 28, 28, 512)
    assert fz[min(fz)].kind == "stem"


def test_unknown_kinds_are_ignored_and_resnet18_has_no_bottleneck():
    assert fusion.enabled_kinds("bneck,foo") == {"bneck"}
    assert fusion.enabled_kinds("off") == set()
    a = registry.get("resnet18")
    params, kw = a.pack(randomize_bn(a.make_model()).eval().state_dict(), "cpu")
    g, fz = _plan(a, params, kw, "all", batch=1, input_uint8=True)
    assert [f.kind for f in fz.values()] == ["stem"]
