"""Implicit-GEMM convolution on the LDS-tiled MFMA GEMM (csrc/gemm.hip CV mode: channel-blocked
activations staged by buffer_load ... lds, zero padding from the descriptor's range check) against
fp32 PyTorch conv2d on bf16-rounded operands (MI355X only)."""
import pytest
import torch

from hipzap import _native as N
from hipzap.ops import conv as C

from test_vision_gpu import _case

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

# n, cin, h, cout, k, stride, pad, residual
SHAPES = [
    (2, 64, 20, 128, 3, 1, 1, True),     # 3x3, padding on every border, M = 800
    (2, 128, 15, 128, 3, 2, 1, False),   # strided 3x3, odd input -> P = 8
    (3, 256, 9, 256, 1, 1, 0, True),     # 1x1, M = 243: partial last row tile
    (2, 256, 14, 512, 1, 2, 0, False),   # strided 1x1 (ResNet downsample)
    (1, 512, 7, 512, 3, 1, 1, True),     # layer4 3x3, M = 49 < one tile
]


@pytest.mark.parametrize("cfg", C.LDS_CONV_CFGS)
def test_lds_conv_every_tile(cfg):
    for n, cin, h, cout, k, stride, pad, res in SHAPES:
        if not C.lds_conv_fits(cfg, cout):
            continue
        err = _case(n, cin, h, cout, k, stride, pad, residual=res, cfg=cfg, kw=1)
        assert err < 2e-2, (cfg, n, cin, h, cout, k, stride, pad, err)


def test_lds_conv_heuristic_large_m():
    """Batched ResNet layer1 shapes: the heuristic routes M >= LDS_CONV_MIN_M to the LDS tile."""
    for n, cin, h, cout, k, stride, pad in [(4, 64, 56, 64, 3, 1, 1), (2, 256, 56, 128, 1, 1, 0),
                                            (8, 512, 28, 256, 1, 1, 0)]:
        pc = C.pack_conv(torch.randn(cout, cin, k, k), None, None, stride, pad)
        M = n * h * h
        assert C.choose_config(M, cout, pc.K, pc=pc)[0] in C.LDS_CONV_CFGS
        assert _case(n, cin, h, cout, k, stride, pad, residual=True) < 2e-2


def test_lds_conv_bs1_unchanged():
    """bs=1 ResNet shapes keep the register-ring kernel (the headline path)."""
    for M, cin, cout, k in [(3136, 64, 64, 3), (784, 128, 512, 1), (49, 512, 2048, 1)]:
        pc = C.pack_conv(torch.randn(cout, cin, k, k), None, None, 1, k // 2)
        assert C.choose_config(M, cout, pc.K, pc=pc)[0] < 16


def test_resnet50_bs8_engine_lds_convs():
    """Whole ResNet-50 at batch 8 through the engine (LDS convs for the large-M layers) against
    the fp32 graph oracle."""
    from hipzap.engine.engine import Engine
    from hipzap.engine.reference import run_graph_reference
    from hipzap.models import registry
    from hipzap.models.resnet import randomize_bn
    torch.manual_seed(0)
    adapter = registry.get("resnet50")
    m = randomize_bn(adapter.make_model()).eval()
    sd = m.state_dict()
    eng = Engine.from_state_dict("resnet50", sd, DEV, batch=8, num_contexts=1, tuned={})
    cfgs = [c[2] for c in eng.contexts[0].configs]
    assert any(c in C.LDS_CONV_CFGS for c in cfgs), cfgs
    x = torch.randn(8, 3, 224, 224)
    y = eng.infer(x)
    ref = run_graph_reference(eng.graph, adapter.pack(sd, "cpu")[0], [x])[eng.graph.outputs[0]].reshape(8, -1)
    err = (y.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 5e-2, err
    assert torch.equal(y.float().argmax(1), ref.argmax(1))
