#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 SQLite output (``*_results.db``, ROCm 7 default format):
calls, total/avg/min/max duration, sorted by total. ``python scripts/rocpd_stats.py x.db [N]``

``--timeline FIRST LAST``: instead, the dispatch timeline of one request -- on the stream with
the most dispatches, the last complete run from a kernel whose name contains FIRST through the
next one containing LAST (start offset, duration, grid, workgroup, VGPRs, name)."""
import sqlite3
import sys


def timeline(c, name, first, last):
    rows = c.execute(f"select stream_id, start, end, grid_x, workgroup_x, vgpr_count, {name} from kernels "
                     "order by start").fetchall()
    counts = {}
    for r in rows:
        counts[r[0]] = counts.get(r[0], 0) + 1
    sid = max(counts, key=counts.get)
    rs = [r for r in rows if r[0] == sid]
    ends = [i for i, r in enumerate(rs) if last in r[6]]
    for e in reversed(ends):
        starts = [i for i in range(e, -1, -1) if first in rs[i][6]]
        if starts:
            seg = rs[starts[0]:e + 1]
            t0 = seg[0][1]
            print("# one request: start_us dur_us grid wg vgpr kernel")
            for _, st, en, gx, wx, vg, n in seg:
                print(f"{(st - t0) / 1e3:8.1f} {(en - st) / 1e3:7.1f} grid={gx:7d} wg={wx:5d} vgpr={vg:4d} {n[:100]}")
            busy = sum(en - st for _, st, en, *_ in seg)
            print(f"# {len(seg)} dispatches, span {(seg[-1][2] - t0) / 1e3:.1f} us, kernel-busy {busy / 1e3:.1f} us "
                  "(profiled; durations inflate under the profiler)")
            return
    print("# no complete request found")


def main():
    db = sys.argv[1]
    if len(sys.argv) > 4 and sys.argv[2] == "--timeline":
        c = sqlite3.connect(db)
        cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
        timeline(c, "kernel_name" if "kernel_name" in cols else "name", sys.argv[3], sys.argv[4])
        return
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     f"from kernels group by {name} order by sum(end-start) desc limit {top}").fetchall()
    total = sum(r[1] for r in c.execute(f"select {name}, sum(end-start) from kernels group by {name}")
                .fetchall()) or 1
    print(f"{'calls':>8} {'total_ms':>10} {'avg_us':>9} {'min_us':>9} {'max_us':>9} {'pct':>6}  kernel")
    for n, k, tot, avg, mn, mx in rows:
        print(f"{k:8d} {tot / 1e6:10.3f} {avg / 1e3:9.2f} {mn / 1e3:9.2f} {mx / 1e3:9.2f} {100 * tot / total:6.1f}  "
              f"{n[:110]}")


if __name__ == "__main__":
    main()
