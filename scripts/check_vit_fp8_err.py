#!/usr/bin/env python3
"""Error of the ViT-B/16 fp8 engine against the fp32 HF model and against hipzap's bf16 engine
(same random-init weights, 4 random images) -- sizes the tolerance of tests/test_fp8_gpu.py."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipzap.engine.engine import Engine  # noqa: E402
from hipzap.models import vit  # noqa: E402


def stats(out, ref):
    rel = ((out - ref).abs().max() / ref.abs().max()).item()
    cos = torch.nn.functional.cosine_similarity(out, ref, dim=1).min().item()
    top1 = (out.argmax(1) == ref.argmax(1)).float().mean().item()
    return {"rel_max": round(rel, 4), "cos_min": round(cos, 5), "top1_agree": top1}


def main():
    torch.manual_seed(0)
    m = vit.make_model(num_labels=1000)
    sd = m.state_dict()
    x = torch.randn(4, 3, 224, 224)
    with torch.no_grad():
        ref = m(pixel_values=x).logits
    f8 = Engine.from_state_dict("vit-b16-fp8", sd, "cuda:0", batch=4).infer(x)
    bf = Engine.from_state_dict("vit-b16", sd, "cuda:0", batch=4).infer(x)
    print(json.dumps({"fp8_vs_fp32": stats(f8, ref), "bf16_vs_fp32": stats(bf, ref), "fp8_vs_bf16": stats(f8, bf)}))


if __name__ == "__main__":
    main()
