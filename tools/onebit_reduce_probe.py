#!/usr/bin/env python3
"""Dev microbenchmark: the 1-bit centralized op's fused middle step
(bagua_onebit_reduce_requantize: decode the p received segments of the own
chunk, reduce them in the reference's tree order, re-encode; + its finalize),
timed with HIP events on one GPU for p = 1..16 chunks of a 1 GiB fp32 (or
512 MiB bf16) bucket.  Prints the re-encoded segment's hash for A/B runs.

    python tools/onebit_reduce_probe.py [--dtype f32|bf16]
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bagua-core_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    from bagua_core import _native as N
    K = N.K
    dcode, tdt, esz = (0, torch.float32, 4) if args.dtype == "f32" else (2, torch.bfloat16, 2)
    n = (1 << 30) // 4
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    x = (torch.randn(n, device=dev, generator=g) * 1e-3).to(tdt)
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    out = {}
    for p in (1, 2, 4, 8, 16):
        cs = n // p
        S = K.bagua_onebit_compressed_bytes(cs, p)
        wsb = K.bagua_onebit_workspace_bytes(cs, p)
        comp = torch.empty(S, dtype=torch.uint8, device=dev)
        res_out = torch.zeros(S, dtype=torch.uint8, device=dev)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        N.check(K.bagua_onebit_compress(dcode, x.data_ptr(), n, cs, p, comp.data_ptr(), S, ws.data_ptr(), wsb, -1, sp),
                "compress")

        def call():
            return K.bagua_onebit_reduce_requantize(dcode, comp.data_ptr(), S, cs, p, None, 1, res_out.data_ptr(), S,
                                                    0, ws.data_ptr(), wsb, sp)
        assert call() == 0
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(st)
        for _ in range(args.reps):
            call()
        ev[1].record(st)
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) * 1e3 / args.reps
        co = S // p
        seg = res_out[:co].cpu().numpy().tobytes()
        # moves p segments of the own chunk's bits in and one segment out
        out[f"p{p}"] = {"us": round(us, 2), "elements": cs, "ns_per_kelem": round(us * 1e6 / cs, 2),
                        "gbs": round((p + 1) * co / (us * 1e-6) / 1e9, 1),
                        "sha": hashlib.sha256(seg).hexdigest()[:16]}
    print(json.dumps({"dtype": args.dtype, "bucket_bytes": n * esz, **out}))


if __name__ == "__main__":
    main()
