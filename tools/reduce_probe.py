#!/usr/bin/env python3
"""Dev microbenchmark: the fused dequantise+reduce kernel (the middle step of
the compressed all-reduce) and the dequantise kernel, timed with HIP events on
one GPU for p = 2..16 chunks of a 1 GiB fp32 (or 512 MiB bf16) bucket.

    python tools/reduce_probe.py [--lib path/to/libbagua_kernels.so] [--dtype f32|bf16]

`--lib` times another build of the kernel library INSTEAD of the in-tree one
(loaded with RTLD_DEEPBIND so its internal calls stay inside it; run the two
builds in separate processes for an A/B and compare the printed output hashes).
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
    ap.add_argument("--lib", default="")
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    from bagua_core import _native as N
    lib = N.kernels
    if args.lib:
        lib = ctypes.CDLL(os.path.abspath(args.lib), mode=os.RTLD_LOCAL | os.RTLD_DEEPBIND)
    for name in ("bagua_minmax_u8_decompress_reduce", "bagua_minmax_u8_decompress"):
        f = getattr(lib, name)
        src = getattr(N.K, name)
        f.restype, f.argtypes = src.restype, src.argtypes
    dcode, tdt, esz = (0, torch.float32, 4) if args.dtype == "f32" else (2, torch.bfloat16, 2)
    n = (1 << 30) // 4
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    x = (torch.randn(n, device=dev, generator=g) * 1e-3).to(tdt)
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    out = {}
    for p in (2, 4, 8, 16):
        cs = n // p
        K = N.K
        S = K.bagua_minmax_u8_compressed_bytes(dcode, cs, p)
        wsb = K.bagua_minmax_u8_workspace_bytes(cs, p)
        comp = torch.empty(S, dtype=torch.uint8, device=dev)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        N.check(K.bagua_minmax_u8_compress(dcode, x.data_ptr(), n, cs, p, comp.data_ptr(), S, ws.data_ptr(), wsb, -1,
                                           sp), "compress")
        res = {}
        red = torch.empty(cs, dtype=tdt, device=dev)
        dec = torch.empty(n, dtype=tdt, device=dev)
        calls = {"reduce": lambda: lib.bagua_minmax_u8_decompress_reduce(dcode, comp.data_ptr(), S, cs, p,
                                                                          red.data_ptr(), 1, sp),
                 "dequant": lambda: lib.bagua_minmax_u8_decompress(dcode, comp.data_ptr(), S, cs, p, dec.data_ptr(),
                                                                   sp)}
        for k, c in calls.items():
            assert c() == 0
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record(st)
            for _ in range(args.reps):
                c()
            ev[1].record(st)
            torch.cuda.synchronize()
            res[f"{k}_us"] = round(ev[0].elapsed_time(ev[1]) * 1e3 / args.reps, 2)
        res["sha"] = hashlib.sha256(red.view(torch.uint8).cpu().numpy().tobytes() +
                                    dec.view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]
        # reduce moves p*cs payload bytes in + cs*esz out; dequantise S in + n*esz out
        res["reduce_gbs"] = round((p * cs + cs * esz) / (res["reduce_us"] * 1e-6) / 1e9, 1)
        res["dequant_gbs"] = round((S + n * esz) / (res["dequant_us"] * 1e-6) / 1e9, 1)
        out[f"p{p}"] = res
    print(json.dumps({"lib": args.lib or "in-tree", "dtype": args.dtype, "bucket_bytes": n * esz, **out}))


if __name__ == "__main__":
    main()
