#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into HBM bytes per kernel launch.

Usage (on the GPU box, two SEPARATE counter passes, as MI355X_MICROARCH.md
§rocprofv3 prescribes: FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2):

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT/fetch -o run -- python3 bench.py ...
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d OUT/write -o run -- python3 bench.py ...
  python3 profiles/collect_pmc.py OUT/fetch OUT/write profiles/r01_pmc_traffic.json

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE is in KiB and on gfx950
reports exactly half the bytes of a wide (16 B/lane) coalesced streaming
read, so it is doubled; WRITE_SIZE (KiB) is exact for 16 B/lane streaming
stores.  Narrower accesses (the 4-B payload loads/stores) are uncalibrated:
the summary keeps the raw values beside the corrected ones.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ("minmax_resident_encode_kernel",
           "minmax_partials_kernel", "minmax_quantize_kernel", "minmax_dequantize_kernel",
           "onebit_encode_kernel", "onebit_decode_kernel", "dequant_reduce_kernel",
           "ring_mix_kernel", "ring_apply_kernel")


def short(name: str) -> str | None:
    for k in KERNELS:
        if k in name:
            return k
    return None


def read_counter(d: str, counter: str) -> dict[str, list[float]]:
    vals: dict[str, list[float]] = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                k = short(row.get("Kernel_Name", ""))
                if k:
                    vals[k].append(float(row["Counter_Value"]))
    return vals


def main() -> None:
    fetch_dir, write_dir, out = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch = read_counter(fetch_dir, "FETCH_SIZE")
    write = read_counter(write_dir, "WRITE_SIZE")
    per_launch, raw = {}, {}
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(k, [0])) / max(1, len(fetch.get(k, [])))
        w = sum(write.get(k, [0])) / max(1, len(write.get(k, [])))
        per_launch[k] = int(round((2 * f + w) * 1024))
        raw[k] = {"FETCH_SIZE_KiB": round(f, 1), "WRITE_SIZE_KiB": round(w, 1),
                  "launches": [len(fetch.get(k, [])), len(write.get(k, []))]}
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of bench.py",
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md)",
           "per_launch_hbm_bytes": per_launch, "raw": raw}
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
