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


_HF_NAMES = {"layers": "num_hidden_layers", "hidden": "hidden_size", "heads": "num_attention_heads",
             "ffn": "intermediate_size"}


def _hf_arch(arch: dict, **extra) -> dict:
    """hipzap cfg keys (``config_from_sd``) -> transformers config kwargs; unknown keys dropped."""
    names = dict(_HF_NAMES, **extra)
    return {names[k]: v for k, v in arch.items() if k in names and v is not None}


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

    def meta_params(self, num_classes=None, **_arch):
        """Packed-parameter shapes without weights (meta tensors): what non-root DP ranks
        allocate before receiving the broadcast blob. Keyword arguments are the source rank's
        broadcast architecture metadata (``pack``'s cfg), so a non-default head is honoured."""
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


class TextClassifierAdapter:
    """BERT-base sequence classification (north-star config 4); ``weights`` = bf16 or fp8."""
    seq_len = 128
    weights = "bf16"

    def make_model(self, num_labels=2):
        from .bert import make_model
        return make_model(num_labels)

    def pack(self, sd: dict, device):
        from .bert import pack_bert
        params, cfg = pack_bert(sd, device, weights=self.weights)
        cfg["seq_len"] = self.seq_len
        return params, cfg

    def meta_params(self, num_labels=2, ln_fold=None, **arch):
        from .bert import make_model, pack_bert
        with torch.device("meta"):
            m = make_model(num_labels, **_hf_arch(arch, max_pos="max_position_embeddings"))
        params, cfg = pack_bert(m.state_dict(), "meta", ln_fold=ln_fold, weights=self.weights)
        cfg["seq_len"] = self.seq_len
        return params, cfg

    def build_graph(self, batch=1, **kw):
        from .bert import build_graph
        return build_graph(batch, **kw)

    def example_input(self, batch=1, generator=None, seq_len=None):
        L = seq_len or self.seq_len
        ids = torch.randint(1000, 30000, (batch, L), generator=generator)
        from .bert import encode_inputs
        return encode_inputs(ids)

    def postprocess_output(self, out: torch.Tensor, meta=None) -> torch.Tensor:
        n = (meta or {}).get("num_labels", out.shape[-1])
        return out.reshape(out.shape[0], -1)[:, :n]


@register("bert-base")
class BertBase(TextClassifierAdapter):
    pass


@register("bert-base-fp8")
class BertBaseFp8(TextClassifierAdapter):
    weights = "fp8"


class ImageTransformerAdapter(VisionAdapter):
    """ViT-B/16 (north-star config 5); ``weights`` = bf16 or fp8 (e4m3 + per-channel scale)."""
    weights = "bf16"

    def make_model(self, num_classes=None):
        from .vit import make_model
        return make_model(num_classes or self.num_classes)

    def pack(self, sd: dict, device):
        from .vit import pack_vit
        return pack_vit(sd, device, weights=self.weights)

    def meta_params(self, num_classes=None, num_labels=None, **arch):
        from .vit import make_model, pack_vit
        with torch.device("meta"):
            m = make_model(num_labels or num_classes or self.num_classes,
                           **_hf_arch(arch, patch="patch_size", image="image_size"))
        return pack_vit(m.state_dict(), "meta", weights=self.weights, patch_lowering=arch.get("patch_lowering"))

    def build_graph(self, batch=1, **kw):
        from .vit import build_graph
        return build_graph(batch, **kw)

    def postprocess_output(self, out: torch.Tensor, meta=None) -> torch.Tensor:
        n = (meta or {}).get("num_labels", out.shape[-1])
        return out.reshape(out.shape[0], -1)[:, :n]


@register("vit-b16")
class ViTB16(ImageTransformerAdapter):
    weights = "bf16"


@register("vit-b16-fp8")
class ViTB16Fp8(ImageTransformerAdapter):
    weights = "fp8"
