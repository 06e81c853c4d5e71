"""Summarise a rocprofv3 kernel trace (rocpd SQLite `*_results.db` or `kernel_stats.csv`).

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db [--top 40] [--md out.md]

Prints per-kernel: launches, total / average / min / max duration, share of GPU
time; plus the total kernel time and the busy fraction of the traced span.
"""
import argparse
import csv
import os
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*\)$", "", name)  # drop parameter lists
    name = name.replace("vae2::", "")
    return name


def from_db(path):
    db = sqlite3.connect(path)
    rows = db.execute("select name, start, end from kernels").fetchall()
    return [(short(n), s, e) for n, s, e in rows]


def summarise(rows):
    agg = defaultdict(list)
    for n, s, e in rows:
        agg[n].append(e - s)
    total = sum(sum(v) for v in agg.values())
    span = (max(e for _, _, e in rows) - min(s for _, s, _ in rows)) if rows else 0
    out = []
    for n, d in agg.items():
        out.append((n, len(d), sum(d), sum(d) / len(d), min(d), max(d)))
    out.sort(key=lambda r: -r[2])
    return out, total, span


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--md", default=None)
    ap.add_argument("--kernel", default=None,
                    help="also report this kernel's average over its last --last dispatches")
    ap.add_argument("--last", type=int, default=0)
    a = ap.parse_args()
    if a.path.endswith(".db"):
        rows = from_db(a.path)
    elif os.path.isdir(a.path):
        import glob
        f = glob.glob(os.path.join(a.path, "**", "*kernel_trace.csv"), recursive=True)[0]
        rows = []
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((short(r["Kernel_Name"]), int(r["Start_Timestamp"]),
                             int(r["End_Timestamp"])))
    else:
        rows = []
        with open(a.path) as f:
            for r in csv.DictReader(f):
                rows.append((short(r["Kernel_Name"]), int(r["Start_Timestamp"]),
                             int(r["End_Timestamp"])))
    out, total, span = summarise(rows)
    extra = []
    if a.kernel:
        ds = sorted((s_, e_) for n, s_, e_ in rows if n.replace("void ", "") == a.kernel)
        sel = ds[-a.last:] if a.last else ds
        if sel:
            avg = sum(e_ - s_ for s_, e_ in sel) / len(sel)
            extra = ["", f"`{a.kernel}`: {len(ds)} dispatches in total, average over the last "
                         f"{len(sel)} (the bench's roofline phase): {avg / 1e3:.1f} us"]
    lines = [f"kernels: {len(rows)} dispatches, {total / 1e6:.2f} ms total kernel time, "
             f"span {span / 1e6:.2f} ms",
             "",
             "| kernel | calls | total ms | avg us | min us | max us | % |",
             "|---|---:|---:|---:|---:|---:|---:|"]
    for n, c, tt, av, mn, mx in out[:a.top]:
        lines.append(f"| `{n}` | {c} | {tt / 1e6:.3f} | {av / 1e3:.1f} | {mn / 1e3:.1f} | "
                     f"{mx / 1e3:.1f} | {100 * tt / total:.1f} |")
    lines += extra
    text = "\n".join(lines)
    print(text)
    if a.md:
        os.makedirs(os.path.dirname(os.path.abspath(a.md)), exist_ok=True)
        with open(a.md, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    sys.exit(main())
