"""Analyse the per-rank kernel traces of tools/queue_probe.py: for every rank,
which hardware queues the RCCL kernels and the codec kernels ran on, and how
much of the codec kernels' time ran while an RCCL kernel of the same process
was running (beside it, on another queue) versus after one ended.

  python3 tools/queue_overlap.py gpurun_out/q4 [label]

Prints one JSON line: per rank, {queues used by each kind, codec busy time,
codec time overlapped with RCCL kernels, fraction, the number of codec kernels
that started while an RCCL kernel was running}.
"""
import csv
import glob
import json
import os
import sys

CODEC = ("minmax_", "dequant_reduce", "reduce_", "onebit_")


def kind(name: str) -> str:
    low = name.lower()
    if "nccl" in low or "rccl" in low:
        return "rccl"
    if any(k in name for k in CODEC):
        return "codec"
    return "other"


def overlap(a, iv):
    s, e = a
    tot = 0
    for x, y in iv:
        lo, hi = max(s, x), min(e, y)
        if hi > lo:
            tot += hi - lo
    return tot


def main():
    root = sys.argv[1]
    label = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(root.rstrip("/"))
    out = {"label": label, "ranks": {}}
    for rdir in sorted(glob.glob(os.path.join(root, "rank*"))):
        rows = []
        for path in glob.glob(os.path.join(rdir, "**", "*kernel_trace.csv"), recursive=True):
            with open(path) as f:
                rows += list(csv.DictReader(f))
        if not rows:
            continue
        ks = [(kind(r["Kernel_Name"]), int(r["Queue_Id"]), int(r.get("Stream_Id", -1) or -1),
               int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows]
        rccl = sorted((s, e) for k, q, st, s, e, _ in ks if k == "rccl")
        codec = [(s, e) for k, q, st, s, e, _ in ks if k == "codec"]
        busy = sum(e - s for s, e in codec)
        ov = sum(overlap(c, rccl) for c in codec)
        started_inside = sum(1 for s, e in codec if any(x < s < y for x, y in rccl))
        out["ranks"][os.path.basename(rdir)] = {
            "queues_rccl": sorted({q for k, q, *_ in ks if k == "rccl"}),
            "queues_codec": sorted({q for k, q, *_ in ks if k == "codec"}),
            "streams_rccl": sorted({st for k, q, st, *_ in ks if k == "rccl"}),
            "streams_codec": sorted({st for k, q, st, *_ in ks if k == "codec"}),
            "rccl_kernels": len(rccl), "codec_kernels": len(codec),
            "codec_busy_us": round(busy / 1e3, 1), "codec_overlapped_with_rccl_us": round(ov / 1e3, 1),
            "overlap_frac": round(ov / busy, 3) if busy else None,
            "codec_kernels_started_during_rccl": started_inside,
            "rccl_busy_us": round(sum(e - s for s, e in rccl) / 1e3, 1),
        }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
