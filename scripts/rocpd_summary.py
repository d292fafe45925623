#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd SQLite database (kernel trace) into markdown.

usage: python scripts/rocpd_summary.py gpurun_out/prof/query_results.db [title] > profiles/x.md
"""
import sqlite3
import sys


def main() -> None:
    db = sqlite3.connect(sys.argv[1])
    title = sys.argv[2] if len(sys.argv) > 2 else sys.argv[1]
    cur = db.cursor()
    print(f"# Kernel trace summary: {title}\n")
    print(f"Source: `rocprofv3 --kernel-trace --stats` database `{sys.argv[1]}`\n")
    print("| kernel | calls | total ms | avg us | min us | max us | grid | wg | VGPR | SGPR | LDS B |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    rows = cur.execute("""
        select name, count(*), sum(duration)/1e6, avg(duration)/1e3, min(duration)/1e3, max(duration)/1e3,
               max(grid_x), max(workgroup_x), max(vgpr_count), max(sgpr_count), max(lds_size)
        from kernels group by name order by sum(duration) desc""").fetchall()
    for r in rows:
        name = r[0] if len(r[0]) < 70 else r[0][:67] + "..."
        print(f"| `{name}` | {r[1]} | {r[2]:.3f} | {r[3]:.1f} | {r[4]:.1f} | {r[5]:.1f} | {r[6]} | {r[7]} | {r[8]} | {r[9]} | {r[10]} |")


if __name__ == "__main__":
    main()
