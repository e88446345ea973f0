"""ResNet-18 / ResNet-50 (torchvision-compatible state_dict keys).

Two halves:
* ``ResNet`` — a plain eager ``nn.Module`` with torchvision's exact parameter names
  (``conv1``, ``bn1``, ``layer{1..4}.{i}.conv{1,2,3}``, ``downsample.{0,1}``, ``fc``). It is
  the checkpoint schema (``torch.save(model.state_dict())`` files load unchanged) and the
  fp32 numerics oracle. torchvision is not installed in this image, so it is written here.
* ``pack_resnet`` + ``build_graph`` — the MI355X lowering: BN folded into every conv at load
  time, weights packed for the MFMA implicit-GEMM kernel, and the network lowered to a
  static kernel graph (preprocess -> stem conv -> maxpool -> bottlenecks with the residual
  add + ReLU fused into the last conv's epilogue -> avgpool -> FC). The downsample conv runs
  on a side stream, concurrently with the block's main branch.

The reference repo has no vision model at all (north-star configs 1-3);
this is the model behind ``POST /predict`` and the headline benchmark.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..engine.graph import Graph
from ..ops.conv import PackedConv, pack_conv, pack_linear
from ..ops.vision import IMAGENET_MEAN, IMAGENET_STD


def _conv3x3(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 3, stride, 1, bias=False)


def _conv1x1(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 1, stride, 0, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv3x3(cin, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv1x1(cin, planes)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = _conv3x3(planes, planes, stride)  # torchvision v1.5: stride on the 3x3
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = _conv1x1(planes, planes * 4)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + idt)


ARCHS = {
    "resnet18": (BasicBlock, [2, 2, 2, 2]),
    "resnet34": (BasicBlock, [3, 4, 6, 3]),
    "resnet50": (Bottleneck, [3, 4, 6, 3]),
    "resnet101": (Bottleneck, [3, 4, 23, 3]),
}


class ResNet(nn.Module):
    def __init__(self, arch="resnet50", num_classes=1000):
        super().__init__()
        block, layers = ARCHS[arch]
        self.arch = arch
        self.block = block
        self.layers_cfg = layers
        self.num_classes = num_classes
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make(block, 64, layers[0])
        self.layer2 = self._make(block, 128, layers[1], 2)
        self.layer3 = self._make(block, 256, layers[2], 2)
        self.layer4 = self._make(block, 512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def _make(self, block, planes, blocks, stride=1):
        ds = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            ds = nn.Sequential(_conv1x1(self.inplanes, planes * block.expansion, stride),
                               nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, ds)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet18(num_classes=1000) -> ResNet:
    return ResNet("resnet18", num_classes)


def resnet50(num_classes=1000) -> ResNet:
    return ResNet("resnet50", num_classes)


def randomize_bn(model: nn.Module, seed: int = 0) -> nn.Module:
    """Give BN layers non-trivial random statistics (random-init weights, as the bench uses)."""
    g = torch.Generator().manual_seed(seed)
    for m in model.modules():
        if isinstance(m, nn.BatchNorm2d):
            c = m.num_features
            m.weight.data = 0.5 + torch.rand(c, generator=g)
            m.bias.data = 0.1 * torch.randn(c, generator=g)
            m.running_mean.data = 0.1 * torch.randn(c, generator=g)
            m.running_var.data = 0.5 + torch.rand(c, generator=g)
    return model


def infer_arch(sd: dict) -> tuple[str, int]:
    nblk = [len({k.split(".")[1] for k in sd if k.startswith(f"layer{i}.")}) for i in range(1, 5)]
    bottleneck = any(k.endswith("conv3.weight") for k in sd)
    for name, (blk, layers) in ARCHS.items():
        if layers == nblk and (blk is Bottleneck) == bottleneck:
            return name, sd["fc.weight"].shape[0]
    raise ValueError(f"unrecognised ResNet state_dict (blocks {nblk})")


# ---------------------------------------------------------------------------- lowering
def _bn(sd, prefix):
    return {k: sd[f"{prefix}.{k}"] for k in ("weight", "bias", "running_mean", "running_var")}


def pack_resnet(sd: dict, device="cpu", native: bool | None = None) -> dict[str, PackedConv]:
    """state_dict -> {name: PackedConv} with BN folded (runs once at cold start). Which state_dict
    tensors feed which packed parameter: engine/nppack.py pack_sources (shared with the
    torch-free packers).

    ``native`` (default on a GPU): every conv / linear is folded and packed by one launch of the
    device packer (csrc/pack.hip ``hz_pack_conv_launch``, the kernel of the torch-free .pth cold
    start) instead of ~10 torch ops each -- bitwise the same bytes; in a fresh process the torch
    ops cost 200-430 ms, almost all of it first-use kernel loading."""
    from ..engine.nppack import pack_sources
    sd = {k: v.to(device) for k, v in sd.items()}
    bottleneck = any(k.endswith("conv3.weight") for k in sd)
    dev = torch.device(device)
    if native is None:
        native = dev.type == "cuda" and _native_pack_available()
    P = {}
    for name, kind, w, bn, b in pack_sources(sd):
        if kind == "linear":
            P[name] = _pack_native(sd[w], sd[b] if b else None, None, 1, 0, None, linear=True) if native \
                else pack_linear(sd[w], sd[b] if b else None)
        else:
            stride, pad = _conv_stride_pad(name, sd[w].shape, bottleneck)
            cin_pad = 8 if name == "conv1" else None
            P[name] = _pack_native(sd[w], None, _bn(sd, bn), stride, pad, cin_pad) if native \
                else pack_conv(sd[w], None, _bn(sd, bn), stride, pad, cin_pad=cin_pad)
    if native:
        torch.cuda.current_stream(dev).synchronize()  # the fp32 sources may be freed on return
    return P


def _native_pack_available() -> bool:
    try:
        from .. import _native as N
        return hasattr(N.lib(), "hz_pack_conv_launch")
    except OSError:
        return False


def _pack_native(weight, bias, bn, stride, pad, cin_pad, linear=False) -> PackedConv:
    """ops/conv.py pack_conv / pack_linear on the device (csrc/pack.hip): same layout, same bytes."""
    import ctypes as C
    import math
    from .. import _native as N
    from ..ops.conv import GEMM_ROW_PAD, ROW_PAD
    f32 = lambda t: None if t is None else (t if t.dtype == torch.float32 else t.float()).contiguous()  # noqa: E731
    w = f32(weight.detach())
    cout, cin = w.shape[0], w.shape[1]
    r, s = (1, 1) if linear else (w.shape[2], w.shape[3])
    cin_p = cin if linear else (cin_pad or int(math.ceil(cin / 8) * 8))
    if linear:
        assert cin % 8 == 0
    ksteps = int(math.ceil(r * s * cin_p / 32))
    rows = int(math.ceil(cout / (GEMM_ROW_PAD if linear else ROW_PAD)) * (GEMM_ROW_PAD if linear else ROW_PAD))
    wf = torch.empty(rows // 16, ksteps, 64, 8, dtype=torch.bfloat16, device=w.device)
    bias_out = torch.empty(cout, dtype=torch.float32, device=w.device)
    p = N.PackConvParams()
    srcs = [w, f32(bias), *(f32(bn[k]) if bn is not None else None
                            for k in ("weight", "bias", "running_mean", "running_var"))]
    p.w, p.bias_in = w.data_ptr(), 0 if srcs[1] is None else srcs[1].data_ptr()
    p.gamma, p.beta, p.mean, p.var = (0 if t is None else t.data_ptr() for t in srcs[2:])
    p.wf, p.bias_out = wf.data_ptr(), bias_out.data_ptr()
    p.cout, p.cin, p.r, p.s, p.cin_p, p.rows, p.ksteps, p.eps = cout, cin, r, s, cin_p, rows, ksteps, 1e-5
    N.check(N.lib().hz_pack_conv_launch(C.byref(p), N.stream_ptr()), "hz_pack_conv_launch")
    return PackedConv(wf, bias_out, cin_p, cout, r, s, stride, pad)


def _conv_stride_pad(name: str, wshape, bottleneck: bool) -> tuple[int, int]:
    """torchvision ResNet geometry: the stem is 7x7/2 pad 3; a stage's first block strides 2 in its
    3x3 conv (bottleneck conv2, basic conv1) and its downsample (stages 2-4); 3x3 pads 1."""
    if name == "conv1":
        return 2, 3
    li, b, conv = name.split(".")
    first = b == "0" and li != "layer1"
    k = wshape[-1]
    if conv == "downsample":
        return (2 if first else 1), 0
    strided = first and ((bottleneck and conv == "conv2") or (not bottleneck and conv == "conv1"))
    return (2 if strided else 1), (1 if k == 3 else 0)


def build_graph(arch: str, batch: int, num_classes: int = 1000, image: int = 224,
                input_uint8: bool = False, side_stream: bool = False, fuse_head: bool = True) -> Graph:
    """Lower ResNet to a static kernel graph for a fixed batch size.

    ``side_stream`` puts the downsample conv on a forked stream. Off by default: measured on
    MI355X (scripts/diag_runtime.py), a multi-stream hipGraph costs ~370 us of host
    submission per replay vs ~30 us single-stream, which dwarfs the overlap it buys.
    """
    block, layers = ARCHS[arch]
    g = Graph(f"{arch}_bs{batch}")
    if input_uint8:
        x_in = g.tensor((batch, image, image, 3), torch.uint8, "image", external=True)
        mean, std = IMAGENET_MEAN, IMAGENET_STD
    else:
        x_in = g.tensor((batch, 3, image, image), torch.float32, "input", external=True)
        mean = std = None
    g.inputs.append(x_in)
    x = g.tensor((batch, image, image, 8), name="nhwc")
    g.add("preprocess", [x_in], [x], mean=mean, std=std)

    def conv(src, name, cout, k, stride, pad, act="relu", res=None, slot=0, out_f32=False, ext=False):
        nb, h, w, _ = g.shape(src)
        p = (h + 2 * pad - k) // stride + 1
        q = (w + 2 * pad - k) // stride + 1
        dt = torch.float32 if out_f32 else torch.bfloat16
        out = g.tensor((nb, p, q, cout), dt, name, external=ext)
        ins = [src] if res is None else [src, res]
        g.add("conv", ins, [out], slot=slot, w=name, act=act, out_f32=out_f32, name=name)
        return out

    x = conv(x, "conv1", 64, 7, 2, 3)
    nb, h, w, c = g.shape(x)
    mp = g.tensor((nb, (h + 1) // 2, (w + 1) // 2, c), name="maxpool")
    g.add("maxpool", [x], [mp], k=3, stride=2, pad=1)
    x = mp
    cin = 64
    for li, nblk in enumerate(layers, start=1):
        planes = 64 * 2 ** (li - 1)
        for b in range(nblk):
            pre = f"layer{li}.{b}"
            stride = 2 if (b == 0 and li > 1) else 1
            cout = planes * block.expansion
            has_ds = b == 0 and (stride != 1 or cin != cout)
            idt = x
            if has_ds:
                slot = 1 if side_stream else 0
                if side_stream:
                    g.add("fork", [], [], slot=1)
                idt = conv(x, f"{pre}.downsample", cout, 1, stride, 0, act="none", slot=slot)
            if block is Bottleneck:
                y = conv(x, f"{pre}.conv1", planes, 1, 1, 0)
                y = conv(y, f"{pre}.conv2", planes, 3, stride, 1)
                if has_ds and side_stream:
                    g.add("join", [], [], slot=1)
                x = conv(y, f"{pre}.conv3", cout, 1, 1, 0, res=idt)
            else:
                y = conv(x, f"{pre}.conv1", planes, 3, stride, 1)
                if has_ds and side_stream:
                    g.add("join", [], [], slot=1)
                x = conv(y, f"{pre}.conv2", cout, 3, 1, 1, res=idt)
            cin = cout
    nb, h, w, c = g.shape(x)
    if fuse_head:  # one kernel: global average pool + FC (csrc/vision.hip pool_fc_kernel)
        logits = g.tensor((nb, 1, 1, num_classes), torch.float32, "fc", external=True)
        g.add("pool_fc", [x], [logits], w="fc", name="pool_fc")
    else:
        pooled = g.tensor((nb, 1, 1, c), name="avgpool")
        g.add("avgpool", [x], [pooled])
        logits = conv(pooled, "fc", num_classes, 1, 1, 0, act="none", out_f32=True, ext=True)
    g.outputs.append(logits)
    return g
