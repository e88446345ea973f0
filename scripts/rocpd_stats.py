#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 SQLite output (``*_results.db``, ROCm 7 default format):
calls, total/avg/min/max duration, sorted by total. ``python scripts/rocpd_stats.py x.db [N]``"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
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
