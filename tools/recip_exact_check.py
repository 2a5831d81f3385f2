"""Exhaustive check behind reduce.hip avg_finish: for p = 2, 4, 8, 16 and every f32 bit pattern,
x * (1/p) == x / p bit for bit (NaN payloads aside).  ~1 min on the CPU:
    python tools/recip_exact_check.py
"""
import numpy as np, sys
bad = 0
for p in (2, 4, 8, 16):
    inv = np.float32(1.0) / np.float32(p)
    for start in range(0, 1 << 32, 1 << 26):
        u = np.arange(start, start + (1 << 26), dtype=np.uint64).astype(np.uint32)
        x = u.view(np.float32)
        with np.errstate(all="ignore"):
            a = (x / np.float32(p)).view(np.uint32)
            b = (x * inv).view(np.uint32)
        diff = a != b
        # NaN payloads may differ only if both are NaN
        nan = np.isnan(a.view(np.float32)) & np.isnan(b.view(np.float32))
        bad += int(np.count_nonzero(diff & ~nan))
    print(p, "mismatches so far", bad, flush=True)
print("total mismatches", bad)
