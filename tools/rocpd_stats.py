#!/usr/bin/env python3
"""Per-kernel duration statistics from a rocprofv3 database (`*_results.db`,
the default output of `rocprofv3 --kernel-trace` on ROCm 7.2).

    python tools/rocpd_stats.py <results.db> [--csv out.csv] [--min-calls N]

Columns: kernel, calls, total_us, mean_us, p50_us, p99_us, max_us,
max_over_mean.  Kernel names are shortened (templates kept, arguments
dropped).
"""
import argparse
import csv
import sqlite3
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    depth, out = 0, []
    for ch in name:  # drop the argument list, keep template arguments
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)[-110:]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default="")
    ap.add_argument("--min-calls", type=int, default=1)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute(
        "select s.display_name, d.end - d.start from rocpd_kernel_dispatch d "
        "join rocpd_info_kernel_symbol s on s.id = d.kernel_id").fetchall()
    acc = {}
    for name, ns in rows:
        acc.setdefault(short(name), []).append(ns / 1000.0)
    out = []
    for name, v in acc.items():
        if len(v) < a.min_calls:
            continue
        v.sort()
        mean = sum(v) / len(v)
        out.append({"kernel": name, "calls": len(v), "total_us": round(sum(v), 1), "mean_us": round(mean, 2),
                    "p50_us": round(v[len(v) // 2], 2), "p99_us": round(v[min(len(v) - 1, int(len(v) * 0.99))], 2),
                    "max_us": round(v[-1], 2), "max_over_mean": round(v[-1] / mean, 2) if mean > 0 else 0.0})
    out.sort(key=lambda r: -r["total_us"])
    w = csv.DictWriter(sys.stdout, fieldnames=list(out[0].keys()) if out else ["kernel"])
    w.writeheader()
    w.writerows(out)
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w2 = csv.DictWriter(f, fieldnames=list(out[0].keys()) if out else ["kernel"])
            w2.writeheader()
            w2.writerows(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
