#!/usr/bin/env python3
"""Merge the pmc_models.sh passes per workload into per-kernel-family metrics (profiles/)."""
import json
import re
import sys
from collections import defaultdict


def family(name):
    m = re.search(r"::(\w+_kernel)(<[^(]*>)?", name)
    if not m:
        return "torch/other" if "at::native" in name else name[:40]
    return m.group(1) + (m.group(2) or "")


def main(d, workloads, out):
    rep = {}
    for w in workloads:
        fam = defaultdict(lambda: defaultdict(float))
        for p in ("P1", "P2", "P3", "P4"):
            try:
                js = json.load(open(f"{d}/{w}_{p}.json"))
            except FileNotFoundError:
                continue
            for name, ctrs in next(iter(js.values()))["per_kernel"].items():
                f = family(name)
                for c, v in ctrs.items():
                    if c == "dispatches":
                        fam[f]["dispatches_" + p] += v
                    else:
                        fam[f][c] += v
        rows = {}
        for f, c in fam.items():
            if "at::native" in f or f.startswith("__amd") or f == "torch/other":
                continue
            r = {"dispatches": c.get("dispatches_P1", 0)}
            if c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16") or c.get("SQ_INSTS_VALU_MFMA_MOPS_F8"):
                r["mfma_gflop_bf16"] = round(c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) * 512 / 1e9, 2)
                r["mfma_gflop_f8"] = round(c.get("SQ_INSTS_VALU_MFMA_MOPS_F8", 0) * 512 / 1e9, 2)
            if c.get("SQ_BUSY_CU_CYCLES"):
                r["mfma_busy_per_cu_busy"] = round(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / c["SQ_BUSY_CU_CYCLES"], 4)
            if c.get("SQ_LDS_IDX_ACTIVE"):
                r["lds_bank_conflict_ratio"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 4)
            if "FETCH_SIZE" in c:
                r["fetch_MB"] = round(c["FETCH_SIZE"] / 1024, 1)
            if "WRITE_SIZE" in c:
                r["write_MB"] = round(c["WRITE_SIZE"] / 1024, 1)
            if c.get("SQ_WAVES"):
                r["waves"] = int(c["SQ_WAVES"])
                r["avg_wave_cycles"] = round(c.get("SQ_WAVE_CYCLES", 0) / c["SQ_WAVES"], 1)
            rows[f] = r
        rep[w] = dict(sorted(rows.items(), key=lambda kv: -kv[1].get("mfma_gflop_bf16", 0) - kv[1].get("mfma_gflop_f8", 0)))
    json.dump(rep, open(out, "w"), indent=1)
    for w, rows in rep.items():
        print(f"== {w}")
        for f, r in list(rows.items())[:8]:
            print(f"  {f[:60]:60s} {r}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2].split(","), sys.argv[3])
