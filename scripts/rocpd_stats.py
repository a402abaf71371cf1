#!/usr/bin/env python
"""Per-kernel statistics (calls, total / average / min ns) from a rocprofv3 rocpd SQLite database,
printed as CSV (the same columns as rocprofv3's kernel_stats.csv).  Usage: rocpd_stats.py DB [--last N]
(--last: only the final N dispatches, i.e. the timed tail of a bench run)."""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=0)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cur = con.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    names = dict(cur.execute(f"select id, display_name from {ks}"))
    rows = list(cur.execute(f"select kernel_id, start, end from {kd} order by start"))
    if a.last:
        rows = rows[-a.last:]
    st = collections.defaultdict(list)
    for k, s, e in rows:
        st[names.get(k, str(k))].append(e - s)
    tot = sum(sum(v) for v in st.values())
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"')
    for n, v in sorted(st.items(), key=lambda kv: -sum(kv[1])):
        print(f'"{n}",{len(v)},{sum(v)},{sum(v) / len(v):.1f},{100 * sum(v) / tot:.2f},{min(v)},{max(v)}')
    if rows:
        print(f'# span of the listed dispatches: {(rows[-1][2] - rows[0][1]) / 1e3:.1f} us')


if __name__ == "__main__":
    main()
