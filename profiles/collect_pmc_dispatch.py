#!/usr/bin/env python3
"""Per-dispatch HBM bytes of this library's kernels from two SEPARATE rocprofv3
counter passes (FETCH_SIZE, WRITE_SIZE), keyed by the kernel's full template name
and grid size, so the roles one kernel plays inside an op (e.g. the pipelined
op's quantise pieces vs its requantise pieces, both minmax_quantize_kernel with
different template arguments) stay apart.  Optionally joins the durations of a
--kernel-trace run of the same command.

  python3 profiles/collect_pmc_dispatch.py FETCH_DIR WRITE_DIR OUT.json [TRACE_DIR]

Corrections as profiles/collect_pmc.py (MI355X_MICROARCH.md §HBM): bytes =
(2 * FETCH_SIZE + WRITE_SIZE) * 1024 for 16-B-per-lane streaming accesses.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

OURS = ("bagua::", "minmax_", "onebit_", "dequant_reduce", "ring_mix", "ring_apply", "reduce_chunks")


def key(name: str, grid) -> str | None:
    if not any(t in name for t in OURS):
        return None
    m = re.search(r"(\w+_kernel)(<[^()]*>)?", name)
    base = (m.group(1) + (m.group(2) or "")) if m else name[:120]
    base = base.replace("bagua::", "")
    return f"{base} grid={grid}"


def read_counter(d: str, counter: str):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                k = key(row.get("Kernel_Name", ""), row.get("Grid_Size"))
                if k:
                    rows.append((int(row["Dispatch_Id"]), k, float(row["Counter_Value"])))
    rows.sort()
    return rows


def read_trace(d: str):
    dur = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                g = int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"])
                k = key(row.get("Kernel_Name", ""), g)
                if k:
                    dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    return dur


def main() -> None:
    fetch_dir, write_dir, out = sys.argv[1], sys.argv[2], sys.argv[3]
    trace = read_trace(sys.argv[4]) if len(sys.argv) > 4 else {}
    fetch = read_counter(fetch_dir, "FETCH_SIZE")
    write = read_counter(write_dir, "WRITE_SIZE")
    by_key = defaultdict(lambda: {"fetch_kib": [], "write_kib": []})
    for _, k, v in fetch:
        by_key[k]["fetch_kib"].append(v)
    for _, k, v in write:
        by_key[k]["write_kib"].append(v)
    summary = {}
    for k, d in sorted(by_key.items()):
        f = sum(d["fetch_kib"]) / max(1, len(d["fetch_kib"]))
        w = sum(d["write_kib"]) / max(1, len(d["write_kib"]))
        s = {"launches": [len(d["fetch_kib"]), len(d["write_kib"])], "FETCH_SIZE_KiB": round(f, 1),
             "WRITE_SIZE_KiB": round(w, 1), "hbm_bytes_per_launch": int(round((2 * f + w) * 1024))}
        if k in trace:
            t = sorted(trace[k])
            s["trace_median_us"] = round(t[len(t) // 2], 2)
            s["trace_launches"] = len(t)
            s["tb_s_on_hbm_bytes"] = round(s["hbm_bytes_per_launch"] / (t[len(t) // 2] * 1e-6) / 1e12, 3)
        summary[k] = s
    doc = {"source": f"rocprofv3 --pmc FETCH_SIZE ({fetch_dir}) / --pmc WRITE_SIZE ({write_dir}), separate passes",
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md)",
           "per_kernel": summary,
           "dispatch_order_fetch": [(i, k, round(v * 2 * 1024)) for i, k, v in fetch][:400]}
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
