#!/usr/bin/env python3
"""Per-kernel PMC table for the ResNet-50 bs=1 chain (VERDICT r5 next #1a).

Merges several ``rocprofv3 --pmc ... --output-format csv`` passes (one directory per pass) of the
same served program into one row per chain position. A position is (kernel name, grid size):
the 29 launches of one request are distinct by name except the repeated seam / kconv launches,
which share their shapes, so their counters are averaged per dispatch. Besides the counters each
row carries the per-workgroup resources from the dispatch record (its VGPR count is not in
registers: take VGPRs from the compiler, profiles/r6_chain/kernel_resources.txt). GRBM_GUI_ACTIVE
under counter collection is mostly profiler overhead per dispatch: no durations here.

Usage: pmc_chain.py <out.json> <pass_dir>... ; prints a text table too.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"::(\w+_kernel)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def load(dirs):
    rows = defaultdict(lambda: defaultdict(float))
    meta = {}
    disp = defaultdict(lambda: defaultdict(set))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    name = r.get("Kernel_Name", "?")
                    if "hipzap" not in name and "anonymous" not in name:
                        continue
                    grid = int(r.get("Grid_Size", 0) or 0)
                    wg = int(r.get("Workgroup_Size", 0) or 0)
                    key = (short(name), grid // max(1, wg))
                    rows[key][r["Counter_Name"]] += float(r["Counter_Value"])
                    disp[key][r["Counter_Name"]].add((d, r.get("Dispatch_Id")))
                    if key not in meta:
                        meta[key] = {
                            "wg_threads": wg,
                            "vgpr": int(r.get("VGPR_Count", r.get("Arch_VGPR_Count", 0)) or 0),
                            "agpr": int(r.get("Accum_VGPR_Count", 0) or 0),
                            "sgpr": int(r.get("SGPR_Count", 0) or 0),
                            "lds_bytes": int(r.get("LDS_Block_Size", r.get("Lds_Block_Size", 0)) or 0),
                        }
    return rows, meta, disp


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    rows, meta, disp = load(dirs)
    table = []
    for key, c in rows.items():
        n = {k: max(1, len(v)) for k, v in disp[key].items()}
        avg = {k: v / n[k] for k, v in c.items()}  # per dispatch
        name, wgs = key
        m = meta[key]
        r = {"kernel": name, "workgroups": wgs, "dispatches": max(n.values()), "lds_bytes": m["lds_bytes"]}
        if avg.get("SQ_BUSY_CU_CYCLES"):
            r["mfma_busy_per_cu_busy"] = round(avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / avg["SQ_BUSY_CU_CYCLES"], 4)
        if avg.get("SQ_WAVE_CYCLES"):
            wc = avg["SQ_WAVE_CYCLES"]
            r["wave_wait_frac"] = round(avg.get("SQ_WAIT_ANY", 0) / wc, 3)          # s_waitcnt / barrier parked
            r["wave_issue_stall_frac"] = round(avg.get("SQ_WAIT_INST_ANY", 0) / wc, 3)
            r["wave_active_frac"] = round(avg.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3)
            if avg.get("SQ_WAVES"):
                r["avg_wave_cycles"] = round(wc / avg["SQ_WAVES"], 1)
        if "TCC_HIT_sum" in avg:
            h, mi = avg["TCC_HIT_sum"], avg.get("TCC_MISS_sum", 0)
            r["l2_hit"] = round(h / max(1.0, h + mi), 3)
        for k in ("TA_BUSY_avr", "TD_BUSY_avr"):
            if k in avg and avg.get("GRBM_GUI_ACTIVE"):
                r[k.lower().replace("_avr", "_frac")] = round(avg[k] / avg["GRBM_GUI_ACTIVE"], 3)
        if "TCC_EA0_ATOMIC_sum" in avg:
            r["l2_atomics"] = int(avg["TCC_EA0_ATOMIC_sum"])
        if avg.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_bank_conflict_ratio"] = round(avg.get("SQ_LDS_BANK_CONFLICT", 0) / avg["SQ_LDS_IDX_ACTIVE"], 4)
        if "FETCH_SIZE" in avg:
            r["fetch_KB"] = round(avg["FETCH_SIZE"], 1)
            r["fetch_KB_per_wg"] = round(avg["FETCH_SIZE"] / max(1, wgs), 2)
        if "WRITE_SIZE" in avg:
            r["write_KB"] = round(avg["WRITE_SIZE"], 1)
        if avg.get("GRBM_GUI_ACTIVE"):
            r["gpu_active_cycles"] = int(avg["GRBM_GUI_ACTIVE"])
        table.append(r)
    table.sort(key=lambda r: -r.get("wave_wait_frac", 0))
    with open(out, "w") as f:
        json.dump(table, f, indent=1)
    cols = ["workgroups", "lds_bytes", "mfma_busy_per_cu_busy",
            "wave_wait_frac", "wave_issue_stall_frac", "l2_hit", "ta_busy_frac", "td_busy_frac",
            "lds_bank_conflict_ratio", "fetch_KB_per_wg", "write_KB"]
    print(f"{'kernel':48s} " + " ".join(f"{c[:9]:>9s}" for c in cols))
    for r in table:
        print(f"{r['kernel'][:48]:48s} " + " ".join(f"{str(r.get(c, '-'))[:9]:>9s}" for c in cols))


if __name__ == "__main__":
    main()
