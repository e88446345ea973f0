#!/usr/bin/env python3
"""Summarise a `rocprofv3 --kernel-trace --stats --output-format csv` run of bench.py.

Writes (into the output dir): kernel_stats.csv (copied), one_inference_trace.txt (the
dispatch timeline of one steady-state inference: from one preprocess kernel to the next, with
start offset, duration, grid and workgroup sizes, VGPRs) and a short summary on stdout.
Usage: trace_summary.py <rocprof -d dir> <out dir> [marker]
``marker`` (default ``preprocess``): a substring of the kernel that starts each period
(e.g. ``lstm_cell_kernel`` for one AWD-LSTM decode step: pass ``lstm_cell_kernel<4>`` or the
layer-0 instantiation).
"""
import csv
import glob
import os
import shutil
import sys


def main():
    src, out = sys.argv[1], sys.argv[2]
    marker = sys.argv[3] if len(sys.argv) > 3 else "preprocess"
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True)
    traces = glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(out, "kernel_stats.csv"))
    if not traces:
        print("no kernel trace found")
        return
    rows = list(csv.DictReader(open(traces[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if marker != "preprocess":  # several kernels may match (e.g. every LSTM layer): keep period starts
        first = rows[starts[0]]["Kernel_Name"] if starts else None
        starts = [i for i in starts if rows[i]["Kernel_Name"] == first]
        starts = [i for k, i in enumerate(starts) if k == 0 or i - starts[k - 1] > 1]
    if len(starts) < 4:
        print("too few inferences in trace")
        return
    mid = len(starts) // 2
    seg = rows[starts[mid]: starts[mid + 1]]
    t0 = int(seg[0]["Start_Timestamp"])
    lines = ["# one steady-state inference: start_us dur_us grid wg vgpr kernel"]
    busy = 0

    def col(r, *names):
        for n in names:
            if r.get(n) not in (None, ""):
                return r[n]
        return "?"
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        name = r["Kernel_Name"][:110]
        grid = col(r, "Grid_Size", "Grid_Size_X")
        wg = col(r, "Workgroup_Size", "Workgroup_Size_X")
        vgpr = col(r, "VGPR_Count", "Arch_VGPR_Count")
        lines.append(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} grid={grid:>7} wg={wg:>5} vgpr={vgpr:>4} {name}")
    span = (int(seg[-1]["End_Timestamp"]) - t0) / 1e3
    lines.append(f"# {len(seg)} dispatches, span {span:.1f} us, kernel-busy {busy / 1e3:.1f} us "
                 "(profiled; durations inflate under the profiler)")
    with open(os.path.join(out, "one_inference_trace.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print(lines[-1])


if __name__ == "__main__":
    main()
