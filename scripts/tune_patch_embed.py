#!/usr/bin/env python3
"""Tune the ViT patch-embedding GEMM (B*196 x 768 x K 768, models/vit.py) at the batch sizes the
ViT tables cover and write its key into those tables. Runs on a GPU:

    python scripts/tune_patch_embed.py [--batches 8 16 32 64]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipzap.engine import tune  # noqa: E402
from hipzap.engine.graph import Graph  # noqa: E402
from hipzap.models._tx import TxBuilder, pack_linear_padded  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, nargs="+", default=[8, 16, 32, 64])
    ap.add_argument("--models", nargs="+", default=["vit-b16-fp8", "vit-b16"])
    a = ap.parse_args()
    dev = "cuda:0"
    torch.manual_seed(0)
    P = {"patch": pack_linear_padded((torch.randn(768, 768) * 0.02).to(dev), torch.zeros(768, device=dev))}
    for B in a.batches:
        g = Graph(f"patch_bs{B}")
        prow = g.tensor((B * 196, 768), torch.bfloat16, "patch_rows")
        TxBuilder(g).gemm(prow, "patch", 768, name="patch_embed")
        for conc in (1, 4):
            paths = [tune.table_path(m, B, conc) for m in a.models]
            if not any(p.exists() for p in paths):
                continue
            table, report = tune.tune_graph(g, P, dev, verbose=True, concurrent=conc)
            _merge(paths, B, table, report)


def _merge(paths, B, table, report):
    for path in paths:
        if not path.exists():
            continue
        t = json.loads(path.read_text())
        t.update(table)  # (the 16x16/16 conv key stays: HIPZAP_VIT_PATCH=conv reads it)
        path.write_text(json.dumps(t, indent=1, sort_keys=True) + "\n")
        print(json.dumps({"batch": B, "table": str(path.name), "set": table,
                          "report": report}), flush=True)


if __name__ == "__main__":
    main()
