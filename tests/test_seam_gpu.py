"""ResNet 1x1 -> 1x1 seams (csrc/block.hip seam_kernel, engine/fusion.py ``seam``) on MI355X.

* the kernel alone against an fp32 PyTorch oracle of the same op: y = relu(W3 t2 + b3 + res) and
  z = b1 + W1 y (layer3 and layer4 geometry, both slice widths, N > 1, a pixel count that is not a
  multiple of the 32-pixel tile);
* the consumer side: a 3x3 conv reading z (fp32, ReLU at the load) and presetting the next
  accumulator (HzConvParams.zinit) against the same conv on relu(z) in bf16;
* ResNet-50 with seams against the per-conv program and the fp32 graph oracle: every block output
  a seam writes, the logits, with the arena's default reuse and without, eager and graph replay;
  7 dispatches fewer;
* the tail (the last block's conv3 + global average pool, the classifier reading the means).
Atomic accumulation order varies run to run, so comparisons are within fp32/bf16 rounding, not
bitwise."""
import ctypes as C

import pytest
import torch

from hipzap import _native as N
from hipzap.engine import fusion
from hipzap.engine.program import ExecContext
from hipzap.engine.reference import run_graph_reference
from hipzap.models import registry
from hipzap.models.resnet import randomize_bn
from hipzap.ops import conv as CV

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SEAMS = "convpool,bneck,bneck2,seam"


def _rel(a, b):
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-6)


def _fixq(t):  # csrc/common.h hz_fixq: the 2^-10 grid every accumulator term (and preset) is rounded to
    return torch.round(t * 1024.0) / 1024.0


def _blk(x_nhwc):  # logical NHWC -> channel-blocked device layout
    return CV.to_blocked(x_nhwc).to(DEV)


@pytest.mark.parametrize("cm,cs,n,h", [(256, 128, 1, 14), (256, 64, 1, 14), (512, 64, 1, 7), (512, 128, 1, 7),
                                       (256, 128, 2, 10), (512, 64, 3, 7)])
def test_seam_kernel_vs_fp32(cm, cs, n, h):
    g = torch.Generator().manual_seed(cm + cs + n)
    co = 4 * cm
    w3 = torch.randn(co, cm, 1, 1, generator=g) * (2.0 / cm) ** 0.5
    w1 = torch.randn(cm, co, 1, 1, generator=g) * (2.0 / co) ** 0.5
    p3 = CV.pack_conv(w3, 0.1 * torch.randn(co, generator=g))
    p1 = CV.pack_conv(w1, 0.1 * torch.randn(cm, generator=g))
    t2 = torch.relu(torch.randn(n, h, h, cm, generator=g)).to(torch.bfloat16)
    res = torch.randn(n, h, h, co, generator=g).to(torch.bfloat16)
    # oracle: fp32 on the bf16 operands; y rounded to bf16 before conv1 (as the kernel feeds it)
    W3, W1 = p3.dense(), p1.dense()
    y_ref = torch.relu(t2.float() @ W3.t() + p3.bias + res.float())
    z_ref = p1.bias + y_ref.to(torch.bfloat16).float() @ W1.t()
    p3d, p1d = p3.to(DEV), p1.to(DEV)
    t2d, resd = _blk(t2), _blk(res)
    y = torch.zeros(n, co // 32, h, h, 32, dtype=torch.bfloat16, device=DEV)
    z = p1d.bias.view(1, cm // 32, 1, 1, 32).expand(n, cm // 32, h, h, 32).contiguous()  # the preset
    prm = fusion.SeamParams()
    prm.t2, prm.w3, prm.b3, prm.res, prm.y = t2d.data_ptr(), p3d.wf.data_ptr(), p3d.bias.data_ptr(), resd.data_ptr(), \
        y.data_ptr()
    prm.w1, prm.z, prm.N, prm.HW, prm.CM, prm.cs = p1d.wf.data_ptr(), z.data_ptr(), n, h * h, cm, cs
    fusion.launch("seam", prm)
    torch.cuda.synchronize()
    y_got = CV.from_blocked(y.cpu(), (n, h, h, co)).float()
    z_got = CV.from_blocked(z.cpu(), (n, h, h, cm))
    assert _rel(y_got, y_ref) < 1e-2, _rel(y_got, y_ref)
    assert _rel(z_got, z_ref) < 2e-3, _rel(z_got, z_ref)


@pytest.mark.parametrize("cs,n,h,t2f32", [(128, 1, 7, False), (128, 1, 7, True), (64, 1, 7, True), (64, 3, 7, False),
                                          (128, 2, 5, True), (128, 1, 8, False)])
def test_tail_kernel_vs_fp32(cs, n, h, t2f32):
    """Tail mode (the last block): pooled[n][c] = mean_hw relu(W3 t2 + b3 + res), fp32 into y's buffer;
    t2 bf16, or fp32 with the ReLU at the load (a K-split conv's accumulator)."""
    g = torch.Generator().manual_seed(cs + n + h + int(t2f32))
    cm, co = 512, 2048
    w3 = torch.randn(co, cm, 1, 1, generator=g) * (2.0 / cm) ** 0.5
    p3 = CV.pack_conv(w3, 0.1 * torch.randn(co, generator=g))
    t2 = torch.randn(n, h, h, cm, generator=g)
    t2in = torch.relu(t2).to(torch.bfloat16)  # what the kernel multiplies either way
    res = torch.randn(n, h, h, co, generator=g).to(torch.bfloat16)
    ref = torch.relu(t2in.float() @ p3.dense().t() + p3.bias + res.float()).mean(dim=(1, 2))
    p3d = p3.to(DEV)
    t2d = _blk(t2) if t2f32 else _blk(t2in)
    resd = _blk(res)
    y = torch.full((n * co * h * h // 2,), float("nan"), device=DEV)  # y's bf16 buffer, as fp32 words
    prm = fusion.SeamParams()
    prm.t2, prm.w3, prm.b3, prm.res, prm.y = t2d.data_ptr(), p3d.wf.data_ptr(), p3d.bias.data_ptr(), resd.data_ptr(), \
        y.data_ptr()
    prm.N, prm.HW, prm.CM, prm.cs, prm.t2_f32, prm.tail = n, h * h, cm, cs, int(t2f32), 1
    fusion.launch("tail", prm)
    torch.cuda.synchronize()
    got = y[: n * co].view(n, co).cpu()
    assert _rel(got, ref) < 1e-2, _rel(got, ref)
    prm.HW = 81  # > one 64-pixel tile
    assert N.lib().hz_launch_kernel(fusion.HZ_K_SEAM, C.byref(prm), None) != 0


@pytest.mark.parametrize("cs,n", [(128, 1), (64, 2)])
def test_cross_stage_seam_kernel_vs_fp32(cs, n):
    """The layer3 -> layer4 seam (HzSeamParams.cn): conv3 256 -> 1024 (+ residual) and the next
    stage's conv1 1024 -> 512 into its fp32 accumulator, t2 the fp32 sum of a K-split conv."""
    g = torch.Generator().manual_seed(cs + n)
    cm, cn, co, h = 256, 512, 1024, 14
    p3 = CV.pack_conv(torch.randn(co, cm, 1, 1, generator=g) * (2.0 / cm) ** 0.5, 0.1 * torch.randn(co, generator=g))
    p1 = CV.pack_conv(torch.randn(cn, co, 1, 1, generator=g) * (2.0 / co) ** 0.5, 0.1 * torch.randn(cn, generator=g))
    t2 = torch.randn(n, h, h, cm, generator=g)
    res = torch.randn(n, h, h, co, generator=g).to(torch.bfloat16)
    y_ref = torch.relu(torch.relu(t2).to(torch.bfloat16).float() @ p3.dense().t() + p3.bias + res.float())
    z_ref = p1.bias + y_ref.to(torch.bfloat16).float() @ p1.dense().t()
    p3d, p1d = p3.to(DEV), p1.to(DEV)
    t2d, resd = _blk(t2), _blk(res)
    y = torch.zeros(n, co // 32, h, h, 32, dtype=torch.bfloat16, device=DEV)
    z = p1d.bias.view(1, cn // 32, 1, 1, 32).expand(n, cn // 32, h, h, 32).contiguous()
    prm = fusion.SeamParams()
    prm.t2, prm.w3, prm.b3, prm.res, prm.y = t2d.data_ptr(), p3d.wf.data_ptr(), p3d.bias.data_ptr(), resd.data_ptr(), \
        y.data_ptr()
    prm.w1, prm.z, prm.N, prm.HW, prm.CM, prm.cs, prm.t2_f32, prm.cn = p1d.wf.data_ptr(), z.data_ptr(), n, h * h, cm, \
        cs, 1, cn
    fusion.launch("seam", prm)
    torch.cuda.synchronize()
    assert _rel(CV.from_blocked(y.cpu(), (n, h, h, co)).float(), y_ref) < 1e-2
    assert _rel(CV.from_blocked(z.cpu(), (n, h, h, cn)), z_ref) < 2e-3
    prm.cn = 384
    assert N.lib().hz_launch_kernel(fusion.HZ_K_SEAM, C.byref(prm), None) != 0


@pytest.mark.parametrize("cs,n", [(64, 1), (128, 2)])
def test_downsample_seam_kernel_vs_fp32(cs, n):
    """HzSeamParams.ds: layer4's first conv3 with its stride-2 1x1 downsample as more K (the residual
    computed from the stage input), then conv1 of the next block into its accumulator."""
    g = torch.Generator().manual_seed(7 * cs + n)
    cm, co, h = 512, 2048, 7
    p3 = CV.pack_conv(torch.randn(co, cm, 1, 1, generator=g) * (2.0 / cm) ** 0.5, 0.1 * torch.randn(co, generator=g))
    pd = CV.pack_conv(torch.randn(co, 2 * cm, 1, 1, generator=g) * (1.0 / cm) ** 0.5, 0.1 * torch.randn(co, generator=g),
                      None, 2, 0)
    p1 = CV.pack_conv(torch.randn(cm, co, 1, 1, generator=g) * (2.0 / co) ** 0.5, 0.1 * torch.randn(cm, generator=g))
    t2 = torch.randn(n, h, h, cm, generator=g)
    xd = torch.relu(torch.randn(n, 2 * h, 2 * h, 2 * cm, generator=g)).to(torch.bfloat16)
    ds_ref = xd[:, ::2, ::2, :].float() @ pd.dense().t() + pd.bias
    y_ref = torch.relu(torch.relu(t2).to(torch.bfloat16).float() @ p3.dense().t() + p3.bias + ds_ref)
    z_ref = p1.bias + y_ref.to(torch.bfloat16).float() @ p1.dense().t()
    p3d, pdd, p1d = p3.to(DEV), pd.to(DEV), p1.to(DEV)
    t2d, xdd = _blk(t2), _blk(xd)
    y = torch.zeros(n, co // 32, h, h, 32, dtype=torch.bfloat16, device=DEV)
    z = p1d.bias.view(1, cm // 32, 1, 1, 32).expand(n, cm // 32, h, h, 32).contiguous()
    prm = fusion.SeamParams()
    prm.t2, prm.w3, prm.b3, prm.res, prm.y = t2d.data_ptr(), p3d.wf.data_ptr(), p3d.bias.data_ptr(), y.data_ptr(), \
        y.data_ptr()
    prm.w1, prm.z, prm.N, prm.HW, prm.CM, prm.cs, prm.t2_f32 = p1d.wf.data_ptr(), z.data_ptr(), n, h * h, cm, cs, 1
    prm.ds, prm.xd, prm.wd, prm.bd, prm.xd_H, prm.xd_W = 1, xdd.data_ptr(), pdd.wf.data_ptr(), pdd.bias.data_ptr(), \
        2 * h, 2 * h
    fusion.launch("seam", prm)
    torch.cuda.synchronize()
    assert _rel(CV.from_blocked(y.cpu(), (n, h, h, co)).float(), y_ref) < 1e-2
    assert _rel(CV.from_blocked(z.cpu(), (n, h, h, cm)), z_ref) < 2e-3
    prm.xd_W = 13  # odd: not a stride-2 source of the 7 x 7 output
    assert N.lib().hz_launch_kernel(fusion.HZ_K_SEAM, C.byref(prm), None) != 0


def test_seam_launch_refuses_bad_geometry():
    prm = fusion.SeamParams()
    buf = torch.zeros(1 << 20, device=DEV)
    for f in ("t2", "w3", "b3", "res", "y", "w1", "z"):
        setattr(prm, f, buf.data_ptr())
    prm.N, prm.HW, prm.CM, prm.cs = 1, 196, 384, 128
    assert N.lib().hz_launch_kernel(fusion.HZ_K_SEAM, C.byref(prm), None) != 0
    prm.CM, prm.cs = 256, 96
    assert N.lib().hz_launch_kernel(fusion.HZ_K_SEAM, C.byref(prm), None) != 0


@pytest.mark.parametrize("cfg,kw", [(3, 16), (3, 8), (0, 4), (4, 8)])
def test_conv_fp32_relu_input_and_zinit(cfg, kw):
    """3x3 conv on fp32 z with ReLU at the load == the same conv on relu(z) in bf16, and the
    launch presets the next accumulator to its bias."""
    g = torch.Generator().manual_seed(cfg * 16 + kw)
    n, h, cm = 1, 14, 256
    z = torch.randn(n, h, h, cm, generator=g)
    pc = CV.pack_conv(torch.randn(cm, cm, 3, 3, generator=g) * (2.0 / (9 * cm)) ** 0.5, 0.1 * torch.randn(cm), None,
                      1, 1).to(DEV)
    want = CV.conv2d_nhwc(torch.relu(z).to(torch.bfloat16).contiguous().to(DEV), pc, act="relu", cfg=cfg, kw=kw)
    zd = _blk(z)
    out = torch.zeros(n, cm // 32, h, h, 32, dtype=torch.bfloat16, device=DEV)
    nxt = torch.full((n, cm // 32, h, h, 32), float("nan"), device=DEV)
    zb = torch.randn(cm, generator=g).to(DEV)
    prm, _, _ = CV.make_params(zd.data_ptr(), pc, n, h, h, out.data_ptr(), 0, "relu", False, cfg, kw)
    prm.x_f32, prm.zinit, prm.zbias, prm.z_C, prm.z_HW = 1, nxt.data_ptr(), zb.data_ptr(), cm, h * h
    N.check(N.lib().hz_conv_launch(prm, cfg, N.stream_ptr()), "hz_conv_launch")
    torch.cuda.synchronize()
    got = CV.from_blocked(out.cpu(), (n, h, h, cm))
    assert torch.equal(got, want.cpu())  # same bf16 operands, same kernel, same K order
    assert torch.equal(CV.from_blocked(nxt.cpu(), (n, h, h, cm)), _fixq(zb.cpu()).expand(n, h, h, cm))


@pytest.fixture(scope="module")
def r50():
    torch.manual_seed(0)
    a = registry.get("resnet50")
    sd = randomize_bn(a.make_model()).eval().state_dict()
    params, kw = a.pack({k: v.to(DEV) for k, v in sd.items()}, torch.device(DEV))
    params_cpu, _ = a.pack(sd, "cpu")
    return a, params, params_cpu, kw


def _run(ctx, x):
    ctx.input.copy_(x.to(ctx.input.device))
    ctx.run()
    torch.cuda.synchronize()


KCONV = SEAMS + ",kconv"
TAIL = KCONV + ",tail"
XSEAM = TAIL + ",xseam"


@pytest.mark.parametrize("batch,noreuse,spec", [(1, True, SEAMS), (1, False, SEAMS), (2, True, SEAMS),
                                                (1, True, KCONV), (1, False, KCONV), (2, False, KCONV),
                                                (1, False, TAIL), (2, True, TAIL), (1, False, XSEAM),
                                                (1, True, XSEAM), (2, False, XSEAM), (1, False, XSEAM + ":kconv"),
                                                (2, True, XSEAM + ":kconv"), (1, False, XSEAM + ",dsseam"),
                                                (1, True, XSEAM + ",dsseam"), (2, False, XSEAM + ",dsseam")])
def test_resnet50_seams_match_per_conv_and_oracle(r50, batch, noreuse, spec, monkeypatch):
    spec, _, ds_at = spec.partition(":")  # where layer4's downsample runs (HIPZAP_XSEAM_DS)
    monkeypatch.setenv("HIPZAP_XSEAM_DS", ds_at or "seam")
    if noreuse:
        monkeypatch.setenv("HIPZAP_ARENA_NOREUSE", "1")
    else:
        monkeypatch.delenv("HIPZAP_ARENA_NOREUSE", raising=False)
    a, params, params_cpu, kw = r50
    g = a.build_graph(batch=batch, **dict(kw, input_uint8=True))
    seam = ExecContext(g, params, torch.device(DEV), fuse=spec)
    plain = ExecContext(g, params, torch.device(DEV), fuse="none")
    assert sum(f.kind == "seam" for f in seam.fused.values()) == (8 if "xseam" in spec else 7)
    assert sum(f.kind == "skip" for f in seam.fused.values()) == (1 if "dsseam" in spec else 0)
    assert sum(f.kind == "kconv" for f in seam.fused.values()) == (9 if "kconv" in spec else 0)
    assert sum(f.kind == "tail" for f in seam.fused.values()) == (1 if "tail" in spec else 0)
    x = torch.randint(0, 256, (batch, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(5))
    _run(seam, x)
    _run(plain, x)
    ref = run_graph_reference(g, params_cpu, [x])
    if noreuse:  # every block output a seam writes
        for f in seam.fused.values():
            if f.kind != "seam":
                continue
            tid = f.nodes[0].outputs[0]
            ys = CV.from_blocked(seam.view(tid).reshape(-1), g.shape(tid)).float().cpu()
            yp = CV.from_blocked(plain.view(tid).reshape(-1), g.shape(tid)).float().cpu()
            assert _rel(ys, yp) < 2e-2 and _rel(ys, ref[tid].float()) < 3e-2, f.nodes[0].attrs["name"]
    ls, lp = seam.output.float().cpu().reshape(batch, -1), plain.output.float().cpu().reshape(batch, -1)
    lr = ref[g.outputs[0]].reshape(batch, -1)
    assert _rel(ls, lr) < 3e-2 and _rel(ls, lp) < 3e-2, (_rel(ls, lr), _rel(ls, lp))
    assert torch.equal(ls.argmax(1), lp.argmax(1))


@pytest.mark.parametrize("spec", [SEAMS, KCONV, TAIL, XSEAM, XSEAM + ",dsseam"])
def test_resnet50_seam_dispatches_and_replay(r50, spec):
    a, params, _, kw = r50
    g = a.build_graph(batch=1, **dict(kw, input_uint8=True))
    base = ExecContext(g, params, torch.device(DEV), fuse="convpool,bneck,bneck2")
    ctx = ExecContext(g, params, torch.device(DEV), fuse=spec)
    assert base.num_ops() - ctx.num_ops() == (8 if "xseam" in spec else 7)  # (dsseam: the pair becomes one conv)
    assert ctx.num_ops() <= 31
    s = torch.cuda.Stream()
    ctx.capture(s)
    for seed in range(4):  # the replayed accumulators are preset again on every replay
        x = torch.randint(0, 256, (1, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(seed))
        _run(base, x)
        with torch.cuda.stream(s):
            ctx.input.copy_(x.to(DEV))
            ctx.replay(s)
        torch.cuda.synchronize()
        lb, lc = base.output.float().cpu(), ctx.output.float().cpu()
        assert _rel(lc, lb) < 2e-2 and torch.equal(lc.argmax(-1), lb.argmax(-1))


KconvParams = fusion.KconvParams
HZ_K_KCONV = fusion.HZ_K_KCONV


@pytest.mark.parametrize("c,h,ck,xf32,n,st", [(256, 14, 64, True, 1, 1), (256, 14, 32, True, 1, 1),
                                              (256, 14, 64, False, 2, 1), (512, 7, 128, True, 1, 1),
                                              (512, 7, 64, True, 2, 1), (512, 7, 128, False, 1, 1),
                                              (256, 28, 32, False, 1, 2), (256, 28, 64, False, 2, 2),
                                              (512, 14, 64, False, 1, 2), (512, 14, 128, True, 1, 2)])
def test_kconv_vs_fp32(c, h, ck, xf32, n, st):
    """K-split 3x3 conv (stride 1 or 2, pad 1): out = preset bias + conv3x3(x, or relu(z) in bf16)
    by atomics; also presets the next accumulator."""
    g = torch.Generator().manual_seed(c + ck + n + st)
    x = torch.randn(n, h, h, c, generator=g)
    pc = CV.pack_conv(torch.randn(c, c, 3, 3, generator=g) * (2.0 / (9 * c)) ** 0.5, 0.1 * torch.randn(c, generator=g),
                      None, st, 1)
    xin = (torch.relu(x) if xf32 else x).to(torch.bfloat16).float()
    wref = pc.dense().reshape(c, 3, 3, c).permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(xin.permute(0, 3, 1, 2), wref, pc.bias, stride=st, padding=1).permute(0, 2, 3, 1)
    ho = h // st
    pcd = pc.to(DEV)
    xd = _blk(x) if xf32 else _blk(x.to(torch.bfloat16))
    out = pcd.bias.view(1, c // 32, 1, 1, 32).expand(n, c // 32, ho, ho, 32).contiguous()
    nxt = torch.full((n, 8, ho, ho, 32), float("nan"), device=DEV)
    zb = torch.randn(256, generator=g).to(DEV)
    prm = KconvParams()
    prm.x, prm.w, prm.out, prm.zinit, prm.zbias = xd.data_ptr(), pcd.wf.data_ptr(), out.data_ptr(), nxt.data_ptr(), \
        zb.data_ptr()
    prm.z_C, prm.z_HW, prm.N, prm.H, prm.W, prm.C, prm.Cout, prm.x_f32, prm.ck, prm.stride = \
        256, ho * ho, n, h, h, c, c, int(xf32), ck, st
    N.check(N.lib().hz_launch_kernel(HZ_K_KCONV, C.byref(prm), N.stream_ptr()), "kconv")
    torch.cuda.synchronize()
    got = CV.from_blocked(out.cpu(), (n, ho, ho, c))
    assert _rel(got, ref) < 1e-3, _rel(got, ref)
    assert torch.equal(CV.from_blocked(nxt.cpu(), (n, ho, ho, 256)), _fixq(zb.cpu()).expand(n, ho, ho, 256))


@pytest.mark.parametrize("n", [1, 2])
def test_kconv_with_downsample_job(n):
    """HzKconvParams.dso: layer4's stride-2 3x3 (fp32 input, ReLU at the load) and, in extra
    workgroups of the same launch, the block's stride-2 1x1 downsample 1024 -> 2048 (bf16 out)."""
    g = torch.Generator().manual_seed(40 + n)
    c, h, cd, cdo = 512, 14, 1024, 2048
    x = torch.randn(n, h, h, c, generator=g)
    pc = CV.pack_conv(torch.randn(c, c, 3, 3, generator=g) * (2.0 / (9 * c)) ** 0.5, 0.1 * torch.randn(c, generator=g),
                      None, 2, 1)
    pd = CV.pack_conv(torch.randn(cdo, cd, 1, 1, generator=g) * cd ** -0.5, 0.1 * torch.randn(cdo, generator=g),
                      None, 2, 0)
    xd = torch.relu(torch.randn(n, h, h, cd, generator=g)).to(torch.bfloat16)
    wref = pc.dense().reshape(c, 3, 3, c).permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(torch.relu(x).to(torch.bfloat16).float().permute(0, 3, 1, 2), wref, pc.bias,
                                     stride=2, padding=1).permute(0, 2, 3, 1)
    ds_ref = xd[:, ::2, ::2, :].float() @ pd.dense().t() + pd.bias
    ho = h // 2
    pcd, pdd = pc.to(DEV), pd.to(DEV)
    xdev, xdd = _blk(x), _blk(xd)
    out = pcd.bias.view(1, c // 32, 1, 1, 32).expand(n, c // 32, ho, ho, 32).contiguous()
    dso = torch.full((n, cdo // 32, ho, ho, 32), float("nan"), dtype=torch.bfloat16, device=DEV)
    prm = KconvParams()
    prm.x, prm.w, prm.out = xdev.data_ptr(), pcd.wf.data_ptr(), out.data_ptr()
    prm.N, prm.H, prm.W, prm.C, prm.Cout, prm.x_f32, prm.ck, prm.stride = n, h, h, c, c, 1, 64, 2
    prm.dsx, prm.dsw, prm.dsb, prm.dso = xdd.data_ptr(), pdd.wf.data_ptr(), pdd.bias.data_ptr(), dso.data_ptr()
    prm.ds_C, prm.ds_Cout, prm.ds_H, prm.ds_W = cd, cdo, h, h
    N.check(N.lib().hz_launch_kernel(HZ_K_KCONV, C.byref(prm), N.stream_ptr()), "kconv+ds")
    torch.cuda.synchronize()
    assert _rel(CV.from_blocked(out.cpu(), (n, ho, ho, c)), ref) < 1e-3
    assert _rel(CV.from_blocked(dso.cpu(), (n, ho, ho, cdo)).float(), ds_ref) < 1e-2
    prm.ds_H = 13  # odd: not a stride-2 source
    assert N.lib().hz_launch_kernel(HZ_K_KCONV, C.byref(prm), None) != 0


def test_kconv_refuses_bad_geometry():
    prm = KconvParams()
    buf = torch.zeros(1 << 20, device=DEV)
    prm.x, prm.w, prm.out = buf.data_ptr(), buf.data_ptr(), buf.data_ptr()
    prm.N, prm.H, prm.W, prm.C, prm.Cout, prm.ck = 1, 28, 28, 256, 256, 64  # 784 pixels at stride 1: none
    assert N.lib().hz_launch_kernel(HZ_K_KCONV, C.byref(prm), None) != 0
    prm.stride = 3
    assert N.lib().hz_launch_kernel(HZ_K_KCONV, C.byref(prm), None) != 0
    prm.stride = 1
    prm.H = prm.W = 14
    prm.ck = 96
    assert N.lib().hz_launch_kernel(HZ_K_KCONV, C.byref(prm), None) != 0
