"""Native vision kernels vs fp32 PyTorch oracles (MI355X only)."""
import pytest
import torch

from hipzap.ops import conv as C
from hipzap.ops import vision as V

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rand_bn(c, g):
    return {"weight": 0.5 + torch.rand(c, generator=g), "bias": 0.1 * torch.randn(c, generator=g),
            "running_mean": 0.1 * torch.randn(c, generator=g), "running_var": 0.5 + torch.rand(c, generator=g)}


def _case(n, cin, h, cout, k, stride, pad, act="relu", residual=False, cfg=None, kw=None, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, cin, h, h, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    bn = _rand_bn(cout, g)
    pc = C.pack_conv(w, None, bn, stride, pad)
    p = (h + 2 * pad - k) // stride + 1
    res = torch.randn(n, cout, p, p, generator=g) if residual else None
    # bf16-rounded inputs for the oracle so only accumulation/epilogue error remains
    xb = x.to(torch.bfloat16).float()
    wref = pc.dense().reshape(cout, k, k, pc.cin)[..., :cin].permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(xb, wref, pc.bias, stride=stride, padding=pad)
    if res is not None:
        ref = ref + res.to(torch.bfloat16).float()
    if act == "relu":
        ref = torch.relu(ref)
    x_nhwc = torch.nn.functional.pad(xb.permute(0, 2, 3, 1), (0, pc.cin - cin)).to(torch.bfloat16)
    r_nhwc = None if res is None else res.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(DEV)
    out = C.conv2d_nhwc(x_nhwc.contiguous().to(DEV), pc.to(DEV), r_nhwc, act=act, cfg=cfg, kw=kw)
    torch.cuda.synchronize()
    got = out.float().cpu().permute(0, 3, 1, 2)
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    return err / scale


SHAPES = [
    # n, cin, h, cout, k, stride, pad
    (1, 64, 56, 64, 1, 1, 0),
    (1, 64, 56, 64, 3, 1, 1),
    (1, 128, 56, 128, 3, 2, 1),
    (1, 256, 14, 1024, 1, 1, 0),
    (1, 512, 7, 512, 3, 1, 1),
    (1, 1024, 14, 2048, 1, 2, 0),
    (2, 3, 32, 64, 7, 2, 3),     # stem-like, generic K path (cin padded to 8)
    (2, 64, 9, 96, 3, 1, 1),     # batch 2, odd spatial
    (1, 64, 5, 40, 1, 1, 0),     # Cout not a multiple of 32 -> row-major output
]


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_heuristic(shape):
    assert _case(*shape) < 2e-2


@pytest.mark.parametrize("cfg", range(len(C.TILES)))
@pytest.mark.parametrize("kw", [1, 2, 4, 16])
def test_conv_every_tile(cfg, kw):
    if not C.legal(cfg, kw):
        pytest.skip("illegal combo")
    assert _case(1, 64, 14, 96, 3, 1, 1, residual=True, cfg=cfg, kw=kw) < 2e-2
    assert _case(2, 3, 20, 64, 7, 2, 3, cfg=cfg, kw=kw) < 2e-2  # generic-K path
    assert _case(1, 64, 9, 128, 1, 1, 0, residual=True, cfg=cfg, kw=kw) < 2e-2  # 1x1 path
    assert _case(2, 128, 8, 64, 1, 2, 0, cfg=cfg, kw=kw) < 2e-2  # strided 1x1 (downsample)


def test_conv_candidates_all_launch():
    for cfg, kw in C.candidates(49, 512, 4608):
        assert _case(1, 512, 7, 512, 3, 1, 1, residual=True, cfg=cfg, kw=kw) < 2e-2, (cfg, kw)


def test_linear_rowmajor_fp32():
    g = torch.Generator().manual_seed(3)
    w = torch.randn(1000, 2048, generator=g) * 0.02
    b = torch.randn(1000, generator=g)
    pc = C.pack_linear(w, b).to(DEV)
    x = torch.randn(3, 2048, generator=g).to(torch.bfloat16)
    out = C.conv2d_nhwc(x.reshape(3, 1, 1, 2048).to(DEV), pc, act="none", out_f32=True).reshape(3, 1000).cpu()
    ref = x.float() @ w.to(torch.bfloat16).float().T + b
    assert (out - ref).abs().max() / ref.abs().max() < 1e-2


def test_maxpool_avgpool_preprocess():
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 9, 11, 64, generator=g).to(torch.bfloat16)
    y = V.maxpool_nhwc(x.to(DEV)).cpu().float()
    ref = torch.nn.functional.max_pool2d(x.float().permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.equal(y, ref)
    for blocked in (False, True):
        a = V.avgpool_nhwc(x.to(DEV), blocked=blocked).cpu().float()
        assert (a - x.float().mean(dim=(1, 2))).abs().max() < 1e-2
    img = torch.randn(2, 3, 20, 24, generator=g)
    p = V.preprocess(img.to(DEV)).cpu().float()
    assert (p - V.preprocess_reference(img)).abs().max() < 1e-2
    u8 = torch.randint(0, 256, (2, 20, 24, 3), dtype=torch.uint8, generator=g)
    p = V.preprocess(u8.to(DEV), mean=V.IMAGENET_MEAN, std=V.IMAGENET_STD).cpu().float()
    assert (p - V.preprocess_reference(u8, mean=V.IMAGENET_MEAN, std=V.IMAGENET_STD)).abs().max() < 2e-2


@pytest.mark.parametrize("shape,cpad", [((2, 30, 34), 8), ((1, 224, 224), 8), ((3, 16, 16), 16), ((1, 5, 7), 8)])
def test_preprocess_uint8_coalesced(shape, cpad):
    """uint8 3-channel payloads: 1024-pixel workgroups with a partial last one, Cpad > 8, and a pixel
    count that is not a multiple of 4 (generic per-pixel kernel) -- every element within one bf16
    ulp of the fp32 math (the output is bf16; fma ordering may move the rounding by one ulp)."""
    g = torch.Generator().manual_seed(2)
    u8 = torch.randint(0, 256, (*shape, 3), dtype=torch.uint8, generator=g)
    for mean, std in ((None, None), (V.IMAGENET_MEAN, V.IMAGENET_STD)):
        p = V.preprocess(u8.to(DEV), cpad=cpad, mean=mean, std=std).cpu().float()
        ref = V.preprocess_reference(u8, cpad=cpad, mean=mean, std=std)
        assert p.shape == ref.shape
        assert bool(((p - ref).abs() <= ref.abs() * 2.0 ** -7 + 1e-6).all()), (p - ref).abs().max()
        assert torch.equal(p[..., 3:], torch.zeros_like(p[..., 3:]))


@pytest.mark.parametrize("B,H,C,N", [(1, 7, 2048, 1000), (3, 7, 512, 10), (2, 4, 64, 33)])
def test_pool_fc(B, H, C, N):
    """Fused global-average-pool + FC (ResNet head) vs fp32."""
    from hipzap.ops import conv as Cv
    from hipzap.ops import vision as V
    g = torch.Generator().manual_seed(11)
    x = torch.randn(B, H, H, C, generator=g).to(torch.bfloat16)
    pc = Cv.pack_linear(torch.randn(N, C, generator=g) * 0.05, torch.randn(N, generator=g))
    y = V.pool_fc(x.to(DEV), pc.to(DEV))
    ref = V.pool_fc_ref(x, pc)
    assert y.shape == (B, N)
    assert ((y.cpu() - ref).abs().max() / ref.abs().max()).item() < 1e-2


@pytest.mark.parametrize("B,C,N", [(1, 2048, 1000), (3, 512, 10)])
def test_pool_fc_pooled_input(B, C, N):
    """HzPoolFcParams.pooled: x is already the fp32 channel means (a tail seam's output) -> FC only."""
    import ctypes
    from hipzap import _native as NN
    from hipzap.ops import conv as Cv
    from hipzap.ops import vision as V
    g = torch.Generator().manual_seed(12)
    m = torch.randn(B, C, generator=g)
    pc = Cv.pack_linear(torch.randn(N, C, generator=g) * 0.05, torch.randn(N, generator=g))
    pcd, md = pc.to(DEV), m.to(DEV)
    out = torch.empty(B, N, device=DEV)
    prm = V.PoolFcParams(md.data_ptr(), pcd.wf.data_ptr(), pcd.bias.data_ptr(), out.data_ptr(), B, C, 49, N, N, 1)
    NN.check(NN.lib().hz_launch_kernel(V.K_POOL_FC, ctypes.byref(prm), NN.stream_ptr()), "pool_fc")
    torch.cuda.synchronize()
    ref = m.to(torch.bfloat16).float() @ pc.dense().float().t() + pc.bias.float()  # the kernel's bf16 MFMA operands
    assert ((out.cpu() - ref).abs().max() / ref.abs().max()).item() < 1e-2


@pytest.mark.parametrize("cfg,kw", [(3, 2), (0, 4), (4, 1)])
@pytest.mark.parametrize("stride2", [False, True])
def test_conv_pair_grouped_launch(cfg, kw, stride2):
    """conv2_kernel (downsample + conv1 in one launch) == the two single launches, bitwise."""
    import ctypes
    from hipzap import _native as N
    g = torch.Generator().manual_seed(12)
    x = torch.randn(1, 14, 14, 256, generator=g).to(torch.bfloat16).to(DEV)
    pa = C.pack_conv(torch.randn(512, 256, 1, 1, generator=g) * 0.05, None, None, 2 if stride2 else 1, 0).to(DEV)
    pb = C.pack_conv(torch.randn(128, 256, 3 if stride2 else 1, 3 if stride2 else 1, generator=g) * 0.05, None,
                     None, 2 if stride2 else 1, 1 if stride2 else 0).to(DEV)
    ya = C.conv2d_nhwc(x, pa, act="none", cfg=cfg, kw=kw)
    yb = C.conv2d_nhwc(x, pb, act="relu", cfg=cfg, kw=kw)
    xb = C.to_blocked(x)
    outs, prms = [], []
    for pc, act in ((pa, "none"), (pb, "relu")):
        p = (14 + 2 * pc.pad - pc.r) // pc.stride + 1
        o = torch.empty(p * p * pc.cout, device=DEV, dtype=torch.bfloat16)
        prm, _, _ = C.make_params(xb.data_ptr(), pc, 1, 14, 14, o.data_ptr(), 0, act, False, cfg, kw)
        outs.append((o, (1, p, p, pc.cout)))
        prms.append(prm)
    N.check(N.lib().hz_conv2_launch(ctypes.byref(prms[0]), ctypes.byref(prms[1]), cfg, N.stream_ptr()), "conv2")
    torch.cuda.synchronize()
    assert torch.equal(C.from_blocked(outs[0][0], outs[0][1]), ya)
    assert torch.equal(C.from_blocked(outs[1][0], outs[1][1]), yb)
