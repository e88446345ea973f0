"""Model registry: name -> adapter (eager oracle, checkpoint packing, graph lowering)."""
from __future__ import annotations

import torch

_REG: dict = {}


def register(name):
    def deco(cls):
        _REG[name] = cls()
        return cls
    return deco


def get(name: str):
    if name not in _REG:
        raise KeyError(f"unknown model {name!r}; known: {sorted(_REG)}")
    return _REG[name]


def names() -> list[str]:
    return sorted(_REG)


class VisionAdapter:
    arch = "resnet50"
    num_classes = 1000
    image = 224

    def make_model(self, num_classes=None):
        from .resnet import ResNet
        return ResNet(self.arch, num_classes or self.num_classes)

    def pack(self, sd: dict, device):
        from .resnet import infer_arch, pack_resnet
        arch, ncls = infer_arch(sd)
        if arch != self.arch:
            raise ValueError(f"checkpoint is {arch}, engine expects {self.arch}")
        return pack_resnet(sd, device), {"num_classes": ncls}

    def meta_params(self, num_classes=None):
        """Packed-parameter shapes without weights (meta tensors): what non-root DP ranks
        allocate before receiving the broadcast blob."""
        from .resnet import pack_resnet
        with torch.device("meta"):
            m = self.make_model(num_classes)
        return pack_resnet(m.state_dict(), "meta"), {"num_classes": num_classes or self.num_classes}

    def build_graph(self, batch=1, num_classes=None, input_uint8=False, **kw):
        from .resnet import build_graph
        return build_graph(self.arch, batch, num_classes or self.num_classes, self.image, input_uint8, **kw)

    def example_input(self, batch=1, generator=None):
        return torch.randn(batch, 3, self.image, self.image, generator=generator)

    def postprocess_output(self, out: torch.Tensor) -> torch.Tensor:
        return out.reshape(out.shape[0], -1)


@register("resnet50")
class ResNet50(VisionAdapter):
    arch = "resnet50"


@register("resnet18")
class ResNet18(VisionAdapter):
    arch = "resnet18"
