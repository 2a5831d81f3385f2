#!/usr/bin/env python3
"""GPU idle gaps in a rocprofv3 kernel trace: the union of every kernel's
[start, end) over the whole device (any stream, any queue), and the idle
intervals between its busy segments, over the last `--window` fraction of the
trace (the timed steps; warmup and setup excluded).

  python3 profiles/trace_gaps.py TRACE_DIR [--window 0.5] [--out summary.json]

Reported: busy / idle time, the idle gaps (count, median, p90, max, how many
exceed 3 us), and mean duration of this library's kernels by name.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def load(d: str):
    ks = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                ks.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row["Kernel_Name"],
                           int(row.get("Queue_Id", 0) or 0)))
    ks.sort()
    return ks


def short(name: str) -> str:
    m = re.search(r"(\w+_kernel)", name)
    return m.group(1) if m else name[:60]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--window", type=float, default=0.5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ks = load(a.trace_dir)
    if not ks:
        raise SystemExit("no kernels")
    ours = [k for k in ks if "bagua::" in k[2] or any(t in k[2] for t in ("minmax_", "onebit_", "dequant_reduce"))]
    t_lo = ours[int(len(ours) * (1 - a.window))][0]
    t_hi = ours[-1][1]
    win = [k for k in ks if k[0] >= t_lo and k[1] <= t_hi]
    segs = []
    for s, e, _, _ in win:
        if segs and s <= segs[-1][1]:
            segs[-1][1] = max(segs[-1][1], e)
        else:
            segs.append([s, e])
    gaps = sorted((segs[i + 1][0] - segs[i][1]) / 1e3 for i in range(len(segs) - 1))
    busy = sum(e - s for s, e in segs) / 1e3
    span = (t_hi - t_lo) / 1e3
    dur = defaultdict(list)
    for s, e, n, _ in win:
        dur[short(n)].append((e - s) / 1e3)
    # overlap: kernel time summed over kernels / busy time (> 1: kernels of different streams ran together)
    ksum = sum((e - s) for s, e, _, _ in win) / 1e3
    q = lambda p: gaps[min(len(gaps) - 1, int(p * (len(gaps) - 1)))] if gaps else 0.0  # noqa: E731
    doc = {"source": os.path.abspath(a.trace_dir), "window": f"last {a.window:.0%} of this library's kernels",
           "span_us": round(span, 1), "busy_us": round(busy, 1), "idle_us": round(span - busy, 1),
           "kernel_time_over_busy": round(ksum / busy, 3) if busy else None,
           "gaps": {"count": len(gaps), "median_us": round(q(0.5), 2), "p90_us": round(q(0.9), 2),
                    "max_us": round(gaps[-1], 2) if gaps else 0.0, "over_3us": sum(g > 3.0 for g in gaps)},
           "kernel_us_mean": {k: round(sum(v) / len(v), 2) for k, v in sorted(dur.items()) if len(v) >= 2},
           "kernel_launches": {k: len(v) for k, v in sorted(dur.items())}}
    s = json.dumps(doc, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
