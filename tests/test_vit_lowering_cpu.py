"""ViT patch-embedding lowering: patchify + GEMM only for 16 x 16 patches tiling the
image, the implicit-GEMM conv otherwise; chosen once at pack time, recorded in the packed config
and followed by the graph builder (and by a DP receiver's meta params)."""
import pytest
import torch

from hipzap.models import registry
from hipzap.models.vit import build_graph, make_model, pack_vit


def _tiny(patch, image):
    torch.manual_seed(0)
    return make_model(num_labels=10, hidden_size=64, num_hidden_layers=1, num_attention_heads=1,
                      intermediate_size=128, patch_size=patch, image_size=image).state_dict()


@pytest.mark.parametrize("patch,image,want", [(16, 224, "gemm"), (16, 64, "gemm"), (32, 224, "conv"),
                                              (8, 64, "conv")])
def test_lowering_follows_the_patch_geometry(patch, image, want):
    params, cfg = pack_vit(_tiny(patch, image))
    assert cfg["patch_lowering"] == want
    g = build_graph(1, **cfg)
    kinds = [n.kind for n in g.nodes]
    assert ("patchify" in kinds) == (want == "gemm")
    assert any(n.attrs.get("name") == "patch_embed" for n in g.nodes)
    # the packed weight matches the lowering the graph uses: conv packing vs a row-major matrix
    assert hasattr(params["patch"], "wf") == (want == "conv") or want == "gemm"


def test_env_switch_is_read_at_pack_time_only(monkeypatch):
    params, cfg = pack_vit(_tiny(16, 64))
    assert cfg["patch_lowering"] == "gemm"
    monkeypatch.setenv("HIPZAP_VIT_PATCH", "conv")  # a later env change must not flip the graph
    assert "patchify" in [n.kind for n in build_graph(1, **cfg).nodes]
    _, cfg2 = pack_vit(_tiny(16, 64))
    assert cfg2["patch_lowering"] == "conv"


def test_meta_params_honour_the_source_lowering(monkeypatch):
    a = registry.get("vit-b16")
    monkeypatch.setenv("HIPZAP_VIT_PATCH", "conv")
    _, cfg = a.meta_params(patch_lowering="gemm")
    assert cfg["patch_lowering"] == "gemm"
