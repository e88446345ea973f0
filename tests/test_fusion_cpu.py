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


def test_arena_never_aliases_a_fused_runs_tensors(r50):
    """A fused kernel reads its input's halo from other workgroups' tiles while it writes its
    output: the arena plan must keep the run's input and output apart (per-node lifetimes let the
    output of a downsample block reuse the block input, whose last reader is the run's 2nd node)."""
    from hipzap.engine.graph import plan_memory
    a, params, kw = r50
    g, fz = _plan(a, params, kw, "all", batch=1, input_uint8=True)
    offsets, _ = plan_memory(g, groups=[(f.start, f.end) for f in fz.values()])
    naive, _ = plan_memory(g)

    def overlap(off, t, u):
        a0, a1 = off[t], off[t] + g.tensors[t].nbytes
        b0, b1 = off[u], off[u] + g.tensors[u].nbytes
        return a0 < b1 and b0 < a1

    hit_naive = False
    for f in fz.values():
        ins = {t for n in f.nodes for t in n.inputs if t in offsets}
        outs = {t for n in f.nodes for t in n.outputs if t in offsets}
        ext_in = ins - outs
        last = f.nodes[-1].outputs[0]
        if last not in offsets:
            continue
        for t in ext_in:
            assert not overlap(offsets, t, last), (f.kind, g.tensors[t].name)
            hit_naive |= overlap(naive, t, last)
    assert hit_naive  # the hazard is real without the groups


def test_launchers_refuse_malformed_params_before_any_hip_call():
    """The fused launchers validate geometry and pointers on the host (returning -1 before any
    HIP call, so this runs without a GPU): a kernel launched on a shape its tiles do not assume
    would read out of bounds."""
    import ctypes as C
    from hipzap import _native as N
    lib = N.lib()
    fake = 1 << 20  # never dereferenced: every case below is refused first

    def bneck(**kw):
        p = fusion.BneckParams(x=fake, w1=fake, b1=fake, w2=fake, b2=fake, w3=fake, b3=fake, out=fake,
                               N=1, H=28, W=28, Cin=512, Cmid=128, Cout=512)
        for k, v in kw.items():
            setattr(p, k, v)
        return lib.hz_bneck_launch(C.byref(p), None)

    assert bneck(x=None) == -1
    assert bneck(out=None) == -1
    assert bneck(wd=fake) == -1                     # downsample weights without its bias
    assert bneck(H=0) == -1 and bneck(N=0) == -1
    assert bneck(H=30) == -1                        # layer2 tiles are 4x4
    assert bneck(Cin=256) == -1                     # layer2 first block needs its downsample
    assert bneck(Cout=256) == -1
    assert bneck(Cmid=64, Cin=256, Cout=256, H=56, W=56, tile_h=6) == -1
    assert bneck(Cmid=64, Cin=64, Cout=256, H=56, W=56) == -1  # layer1 first block without downsample
    assert bneck(imgs=2, N=3) == -1 and bneck(imgs=3, N=4) == -1  # layer2 image pairs need an even batch

    def stem(**kw):
        p = fusion.StemParams(src=fake, w=fake, bias=fake, out=fake, N=1, H=224, W=224, mode=1,
                              SH=112, SW=112, PH=56, PW=56)
        for k, v in kw.items():
            setattr(p, k, v)
        return lib.hz_stem_launch(C.byref(p), None)

    assert stem(w=None) == -1
    assert stem(SH=111) == -1 and stem(PH=55) == -1
    assert stem(mode=3) == -1
    assert stem(src=fake + 2) == -1                 # uint8 rows are read as dwords


def test_a_run_whose_intermediate_is_read_elsewhere_is_not_fused(r50):
    """The fused kernels write only the run's last output: a block whose conv2 output is also a
    graph output (a debugging tap) stays per-conv, the other blocks still fuse."""
    a, params, kw = r50
    g = a.build_graph(batch=1, input_uint8=True)
    fz = fusion.plan(g, params, fusion.enabled_kinds("all"))
    b2 = [f for f in fz.values() if f.kind == "bneck2"]
    tap = b2[1].nodes[1].outputs[0]  # conv2 of the second layer2 block
    g.outputs.append(tap)
    fz2 = fusion.plan(g, params, fusion.enabled_kinds("all"))
    assert [f.kind for f in fz2.values()].count("bneck2") == 3
    assert b2[1].start not in fz2


def test_resnet50_seams(r50):
    """layer3 has five conv3 -> conv1 seams, layer4 two (the first block of a stage starts with its
    downsample + conv1 pair, so no seam crosses a stage boundary); each seam's accumulator is
    planned as fp32 and is live from the 3x3 conv that presets it to the one that reads it."""
    from hipzap.engine.graph import plan_memory
    a, params, kw = r50
    g, fz = _plan(a, params, kw, "convpool,bneck,bneck2,seam", batch=1, input_uint8=True)
    seams = [f for f in fz.values() if f.kind == "seam"]
    names = [(f.nodes[0].attrs["name"], f.nodes[1].attrs["name"]) for f in seams]
    assert names == [(f"layer3.{b}.conv3", f"layer3.{b + 1}.conv1") for b in range(5)] + \
        [(f"layer4.{b}.conv3", f"layer4.{b + 1}.conv1") for b in range(2)]
    for f in seams:
        assert g.nodes[f.init].attrs["name"].endswith("conv2") and g.nodes[f.consumer].attrs["name"].endswith("conv2")
        assert f.end == f.start + 2 and f.init == f.start - 1 and f.consumer == f.end
    # the block fusions are unchanged next to the seams
    assert [f.kind for f in fz.values() if f.kind != "seam"] == ["convpool"] + ["bneck"] * 3 + ["bneck2"] * 4
    gp = fusion.planning_graph(g, fz)
    assert gp is not g and g.tensors[seams[0].nodes[1].outputs[0]].dtype == torch.bfloat16
    offsets, _ = plan_memory(gp, groups=[(f.start, f.end) for f in fz.values()])
    for f in seams:
        t1 = f.nodes[1].outputs[0]
        assert gp.tensors[t1].dtype == torch.float32 and t1 in gp.nodes[f.init].outputs
        z0, z1 = offsets[t1], offsets[t1] + gp.tensors[t1].nbytes
        # no tensor touched from the presetting conv through the reader shares the accumulator's bytes
        for j in range(f.init, f.consumer + 1):
            for t in g.nodes[j].inputs + g.nodes[j].outputs:
                if t == t1 or t is None or g.tensors[t].external:
                    continue
                o0, o1 = offsets[t], offsets[t] + gp.tensors[t].nbytes
                assert o1 <= z0 or z1 <= o0, (g.nodes[j].attrs.get("name"), g.tensors[t].name)


def test_seams_need_the_layer3_layer4_geometry(r50):
    a, params, kw = r50
    _, fz = _plan(a, params, kw, "seam", batch=2, input_uint8=False)
    assert sum(f.kind == "seam" for f in fz.values()) == 7
    r18 = registry.get("resnet18")
    p18, kw18 = r18.pack(randomize_bn(r18.make_model()).eval().state_dict(), "cpu")
    _, fz18 = _plan(r18, p18, kw18, "seam", batch=1, input_uint8=True)
    assert fz18 == {}  # basic blocks: no 1x1 -> 1x1 seam


def test_resnet50_kconvs(r50):
    """With ``kconv`` every seam's consumer 3x3 conv becomes a K-split launch: layer3 blocks 1-5 and
    layer4 blocks 1-2; each is preset by the seam before it, the interior ones preset the next seam,
    the last one of a stage is read by a plain conv3."""
    from hipzap.engine.graph import plan_memory
    a, params, kw = r50
    g, fz = _plan(a, params, kw, "convpool,bneck,bneck2,seam,kconv", batch=1, input_uint8=True)
    kc = [f for f in fz.values() if f.kind == "kconv"]
    assert [f.nodes[0].attrs["name"] for f in kc] == [f"layer3.{b}.conv2" for b in range(0, 6)] + \
        [f"layer4.{b}.conv2" for b in range(0, 3)]
    assert [f.next_seam is None for f in kc] == [False] * 5 + [True] + [False] * 2 + [True]
    for f in kc:
        if f.seam is None:  # a stage's first block: stride 2, preset by its conv1 (paired with the downsample)
            assert f.nodes[0].attrs["name"].endswith(".0.conv2") and g.nodes[f.preset].attrs["name"].endswith(".0.conv1")
        else:
            assert fz[f.seam].kind == "seam" and fz[f.seam].consumer == f.start and f.preset == f.seam + 1
        if f.next_seam is not None:
            assert fz[f.next_seam].init == f.start and f.reader is None
        else:
            assert g.nodes[f.reader].attrs["name"].endswith("conv3")
    gp = fusion.planning_graph(g, fz)
    offsets, _ = plan_memory(gp, groups=[(f.start, f.end) for f in fz.values()])
    for f in kc:
        a_t = f.nodes[0].outputs[0]
        assert gp.tensors[a_t].dtype == torch.float32 and a_t in gp.nodes[f.preset].outputs
        z0, z1 = offsets[a_t], offsets[a_t] + gp.tensors[a_t].nbytes
        for j in range(f.preset, f.start + 2):  # presetting launch .. the reader
            for t in g.nodes[j].inputs + g.nodes[j].outputs:
                if t == a_t or t is None or g.tensors[t].external:
                    continue
                o0, o1 = offsets[t], offsets[t] + gp.tensors[t].nbytes
                assert o1 <= z0 or z1 <= o0, (g.nodes[j].attrs.get("name"), g.tensors[t].name)


def test_resnet50_tail(r50):
    """``tail``: the last block's conv3 (1x1 512 -> 2048 + residual, 7 x 7) next to the pooled
    classifier becomes the seam kernel's pooling tail; the pool_fc node stays and reads the means.
    Not matched when the block output is read elsewhere, nor on a larger final feature map."""
    a, params, kw = r50
    g, fz = _plan(a, params, kw, "convpool,bneck,bneck2,seam,kconv,tail", batch=1, input_uint8=True)
    tails = [f for f in fz.values() if f.kind == "tail"]
    assert len(tails) == 1
    f = tails[0]
    assert f.nodes[0].attrs["name"] == "layer4.2.conv3" and g.nodes[f.reader].kind == "pool_fc"
    assert f.end == f.start + 1 and fz[f.start - 1].kind == "kconv"  # t2 is a K-split conv's fp32 sum
    g2 = a.build_graph(**dict(kw, batch=1, input_uint8=True))
    g2.outputs.append(f.nodes[0].outputs[0])  # a tap on the block output
    assert not any(x.kind == "tail" for x in fusion.plan(g2, params, fusion.enabled_kinds("tail")).values())
    from hipzap.models.resnet import build_graph
    g3 = build_graph("resnet50", 1, 1000, 288, True)  # 9 x 9 = 81 pixels
    assert not any(x.kind == "tail" for x in fusion.plan(g3, params, fusion.enabled_kinds("tail")).values())


@pytest.mark.parametrize("ds_at", ["kconv", "seam"])  # HIPZAP_XSEAM_DS
def test_resnet50_cross_stage_seam(r50, ds_at, monkeypatch):
    """``xseam``: layer3's last conv3 + layer4's first conv1 become one seam (the downsample node
    between them skipped), layer4's stride-2 3x3 its K-split consumer (preset by that seam's conv1
    half), and the next seam computes the downsample as its residual; the downsample's input stays
    live in the arena until that seam."""
    from hipzap.engine.graph import plan_memory
    a, params, kw = r50
    monkeypatch.setenv("HIPZAP_XSEAM_DS", ds_at)
    g, fz = _plan(a, params, kw, "convpool,bneck,bneck2,seam,kconv,tail,xseam", batch=1, input_uint8=True)
    xs = [f for f in fz.values() if f.kind == "seam" and f.end - f.start == 3]
    assert len(xs) == 1
    x = xs[0]
    assert [n.attrs["name"] for n in x.nodes] == ["layer3.5.conv3", "layer4.0.conv1"]
    assert g.nodes[x.start + 1].attrs["name"] == "layer4.0.downsample"
    kc = fz[x.consumer]
    assert kc.kind == "kconv" and kc.seam == x.start and kc.preset == x.start + 2 and kc.next_seam == x.consumer + 1
    assert fz[x.init].kind == "kconv" and fz[x.init].next_seam == x.start
    ds_node = g.nodes[x.start + 1]
    ds_seam = fz[x.consumer + 1]
    owner = kc if ds_at == "kconv" else ds_seam  # the launch that computes layer4's downsample
    other = ds_seam if ds_at == "kconv" else kc
    assert owner.ds is ds_node and owner.ds_from == x.start and other.ds is None
    assert sum(f.kind == "seam" for f in fz.values()) == 8
    gp = fusion.planning_graph(g, fz)
    y = x.nodes[0].outputs[0]
    assert y in gp.nodes[owner.start].inputs
    if ds_at == "kconv":
        assert ds_node.outputs[0] in gp.nodes[owner.start].outputs
    offsets, _ = plan_memory(gp, groups=[(f.start, f.end) for f in fz.values()])
    y0, y1 = offsets[y], offsets[y] + gp.tensors[y].nbytes
    for j in range(x.start, owner.end):  # nothing written from the xseam through the downsample's launch reuses y
        for t in g.nodes[j].outputs:
            if t != y and t in offsets:
                assert offsets[t] + gp.tensors[t].nbytes <= y0 or y1 <= offsets[t], g.nodes[j].attrs.get("name")
    # without kconv there is no consumer for the fp32 conv1 sum: no cross-stage seam
    _, fz2 = _plan(a, params, kw, "convpool,bneck,bneck2,seam,xseam", batch=1, input_uint8=True)
    assert not any(f.kind == "seam" and f.end - f.start == 3 for f in fz2.values())
    assert all(f.ds is None for f in fz2.values())


def test_resnet50_layer3_downsample_seam(r50):
    """``dsseam``: layer3's downsample node is skipped (no launch of its own) and computed inside
    layer3's first seam, whose t2 is the stride-2 K-split conv's fp32 sum; conv1 then binds alone.
    Its input (layer2's output) stays live until that seam."""
    a, params, kw = r50
    g, fz = _plan(a, params, kw, fusion.DEFAULT + ",dsseam", batch=1, input_uint8=True)
    sk = [f for f in fz.values() if f.kind == "skip"]
    assert len(sk) == 1 and sk[0].nodes[0].attrs["name"] == "layer3.0.downsample"
    s0 = fz[sk[0].seam]
    assert s0.ds is sk[0].nodes[0] and s0.ds_from == sk[0].start
    assert [n.attrs["name"] for n in s0.nodes] == ["layer3.0.conv3", "layer3.1.conv1"]
    assert fz[s0.init].kind == "kconv" and fz[s0.init].preset == s0.init - 1  # conv1 alone presets it
    gp = fusion.planning_graph(g, fz)
    assert sk[0].nodes[0].inputs[0] in gp.nodes[s0.start].inputs


def test_round5_launchers_refuse_malformed_params_before_any_hip_call():
    """The seam (tail, cross-stage, downsample), K-split (+ downsample job) and fused QKV +
    attention launchers validate geometry on the host and return before any HIP call (so this runs
    without a GPU): a shape their tiles do not assume would read out of bounds."""
    import ctypes as C
    from hipzap import _native as N
    from hipzap.ops import transformer as T
    lib = N.lib()
    fake = 1 << 20  # never dereferenced

    def seam(**kw):
        p = fusion.SeamParams(t2=fake, w3=fake, b3=fake, res=fake, y=fake, w1=fake, z=fake, N=1, HW=49, CM=512, cs=128)
        for k, v in kw.items():
            setattr(p, k, v)
        return lib.hz_launch_kernel(fusion.HZ_K_SEAM, C.byref(p), None)

    assert seam(CM=384) != 0 and seam(cs=96) != 0
    assert seam(tail=1, HW=81) != 0                       # the pooling tail: one 64-pixel tile per image
    assert seam(tail=1, CM=256, HW=49) != 0
    assert seam(cn=384, CM=256, HW=196) != 0              # cross-stage seam: CM 256 -> conv1 512 only
    assert seam(ds=1, t2_f32=0) != 0                      # the downsample seam follows a K-split conv
    assert seam(ds=1, t2_f32=1, xd=fake, wd=fake, bd=fake, xd_H=13, xd_W=13) != 0
    assert seam(ds=1, t2_f32=1, xd=fake, wd=fake, bd=fake, xd_H=16, xd_W=16) != 0  # 8x8 != 49 pixels

    def kconv(**kw):
        p = fusion.KconvParams(x=fake, w=fake, out=fake, N=1, H=14, W=14, C=512, Cout=512, x_f32=1, ck=64, stride=2)
        for k, v in kw.items():
            setattr(p, k, v)
        return lib.hz_launch_kernel(fusion.HZ_K_KCONV, C.byref(p), None)

    assert kconv(ck=48) != 0 and kconv(stride=3) != 0 and kconv(H=13) != 0
    assert kconv(dso=fake, dsx=fake, dsw=fake, dsb=fake, ds_C=512, ds_Cout=2048, ds_H=14, ds_W=14) != 0
    assert kconv(dso=fake, dsx=fake, dsw=fake, dsb=fake, ds_C=1024, ds_Cout=2048, ds_H=18, ds_W=18) != 0

    def qa(**kw):
        p = T.QkvAttParams(fake, fake, fake, 0, fake, 2, 128, 12, 768, 24, 768, 768, 0.125)
        for k, v in kw.items():
            setattr(p, k, v)
        return lib.hz_launch_kernel(T.K_QKVATT, C.byref(p), None)

    assert qa(L=129) != 0 and qa(D=700) != 0 and qa(ksteps=23) != 0 and qa(ldx=770) != 0 and qa(w=None) != 0


@pytest.mark.parametrize("image", [112, 128, 160, 192, 224, 288])
def test_kconv_and_tail_only_bind_geometries_the_launchers_accept(r50, image):
    """at another image size the default fusion set must not bind a K-split 3x3 conv the
    launcher refuses (pixel-group counts other than 7 / 2, a channel slice the kernel has no
    instantiation for, a padded image over its LDS bound) nor a pooling tail over a 1-pixel map
    (whose fp32 means would overrun the block output's bf16 buffer); those runs bind per conv."""
    from hipzap.models.resnet import build_graph
    a, params, kw = r50
    g = build_graph("resnet50", 1, 1000, image, True)
    fz = fusion.plan(g, params, fusion.enabled_kinds(fusion.DEFAULT))
    for f in fz.values():
        if f.kind == "kconv":
            n = f.nodes[0]
            _, h, w, c = g.shape(n.inputs[0])
            assert fusion.kconv_launchable(h, w, c, params[n.attrs["w"]].stride), (image, n.attrs["name"])
        if f.kind == "tail":
            _, h, w, _ = g.shape(f.nodes[0].outputs[0])
            assert 2 <= h * w <= 64
    if image == 224:  # the served geometry keeps every fused launch
        assert sum(f.kind == "kconv" for f in fz.values()) == 9
    if image in (160, 192):  # layer3 at 10x10 / 12x12: pixel-group counts 4 / 5 -> per-conv 3x3s
        assert not any(f.kind == "kconv" and g.shape(f.nodes[0].inputs[0])[3] == 256 and
                       params[f.nodes[0].attrs["w"]].stride == 1 for f in fz.values())


def test_kconv_launchable_mirrors_the_launcher_refusals():
    """Every geometry the host predicate rejects is refused by hz_kconv_launch before any HIP call
    (so the predicate is never looser than the launcher's own checks)."""
    import ctypes as C
    from hipzap import _native as N
    lib = N.lib()
    fake = 1 << 20
    for c in (256, 512):
        for stride in (1, 2):
            for h in range(4, 31, 2):
                if fusion.kconv_launchable(h, h, c, stride):
                    continue
                p = fusion.KconvParams(x=fake, w=fake, out=fake, N=1, H=h, W=h, C=c, Cout=c,
                                       ck=fusion.kconv_ck(c, stride), stride=stride)
                assert lib.hz_kconv_launch(C.byref(p), None) < 0, (c, stride, h)


def test_tail_refuses_a_one_pixel_map():
    import ctypes as C
    from hipzap import _native as N
    fake = 1 << 20
    p = fusion.SeamParams(t2=fake, w3=fake, b3=fake, res=fake, y=fake, N=1, HW=1, CM=512, cs=64, tail=1)
    assert N.lib().hz_seam_launch(C.byref(p), None) == -1
