#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 SQLite output (``*_results.db``, ROCm 7 default format):
calls, total/avg/min/max duration, sorted by total. ``python scripts/rocpd_stats.py x.db [N]``

``--timeline FIRST LAST``: instead, the dispatch timeline of one request -- on the stream with
the most dispatches, the last complete run from a kernel whose name contains FIRST through the
next one containing LAST (start offset, duration, grid, workgroup, VGPRs, name).

``--cutime FIRST LAST``: per-position CU-time accounting over EVERY complete request (FIRST ..
LAST) of every stream: median duration, workgroups, waves per workgroup, CU-us = workgroups x
duration / 256 CUs and wave-us = waves x duration / (256 CUs x 32 wave slots) of each dispatch
position, plus each position's share of a request's summed kernel time (VERDICT r4 "next round"
1a)."""
import statistics
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


def requests(c, name, first, last):
    """[(stream, [rows of one request])] for every complete FIRST..LAST run on every stream."""
    rows = c.execute(f"select stream_id, start, end, grid_x, workgroup_x, vgpr_count, {name} from kernels "
                     "order by start").fetchall()
    by: dict = {}
    for r in rows:
        by.setdefault(r[0], []).append(r)
    out = []
    for sid, rs in by.items():
        cur = None
        for r in rs:
            if first in r[6]:
                cur = [r]
            elif cur is not None:
                cur.append(r)
                if last in r[6]:
                    out.append((sid, cur))
                    cur = None
    return out


def cutime(c, name, first, last, cus=256):
    reqs = requests(c, name, first, last)
    if not reqs:
        print("# no complete request found")
        return
    n = statistics.mode(len(r) for _, r in reqs)
    reqs = [r for _, r in reqs if len(r) == n]
    span = statistics.median((r[-1][2] - r[0][1]) / 1e3 for r in reqs)
    print(f"# {len(reqs)} requests of {n} dispatches; median request span {span:.1f} us")
    print(f"{'pos':>3} {'dur_us':>7} {'wgs':>5} {'wv/wg':>5} {'CU-us':>7} {'wave-us':>7} {'pct':>5}  kernel")
    tot = [0.0, 0.0, 0.0]
    lines = []
    for i in range(n):
        d = statistics.median((r[i][2] - r[i][1]) / 1e3 for r in reqs)
        gx, wx = reqs[0][i][3], reqs[0][i][4]
        wgs = max(1, gx // max(1, wx))
        wv = (wx + 63) // 64
        cu, wave = wgs * d / cus, wgs * wv * d / (cus * 32)
        tot[0] += d
        tot[1] += cu
        tot[2] += wave
        lines.append((i, d, wgs, wv, cu, wave, reqs[0][i][6]))
    for i, d, wgs, wv, cu, wave, nm in lines:
        print(f"{i:3d} {d:7.2f} {wgs:5d} {wv:5d} {cu:7.3f} {wave:7.3f} {100 * d / tot[0]:5.1f}  {nm[:90]}")
    print(f"# sum: {tot[0]:.1f} us kernel time, {tot[1]:.2f} CU-us, {tot[2]:.3f} wave-us per request "
          "(profiled; durations inflate under the profiler)")


def main():
    db = sys.argv[1]
    if len(sys.argv) > 4 and sys.argv[2] == "--cutime":
        c = sqlite3.connect(db)
        cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
        cutime(c, "kernel_name" if "kernel_name" in cols else "name", sys.argv[3], sys.argv[4])
        return
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
