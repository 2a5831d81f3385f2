"""Why the codec kernels run slower per byte at 1 GiB than at 256 MiB: each kernel
timed by its own HIP events (bagua_time_next_kernels) at both sizes, in three
Infinity-Cache states set up just before it by an untimed torch kernel on the same
stream:

  clean   a 1 GiB read of an unrelated buffer (the 256 MiB Infinity Cache holds
          clean lines of it; nothing of the kernel's own data)
  dirty   a 1 GiB write of an unrelated buffer with default-policy stores (the
          cache holds 256 MiB of dirty lines the kernel's traffic must write back)
  chain   the codec's own predecessor, as a step runs it (encode after the last
          decode, decode after the encode): what the bench and the op see

Algorithmic bytes per launch (SURVEY §8(d), N fp32 elements, p = 1):
  minmax_partials 4N, minmax_quantize 5N + 32, minmax_dequantize 5N + 32,
  onebit_encode 4N + N/8 (+ tile partials), onebit_decode N/8 + 4N.

  python tools/cache_state_probe.py [--reps 7] [--out file.jsonl]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "bagua-core_amd"))

from bagua_core import _native as N  # noqa: E402

F32 = 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--sizes", default="67108864,268435456")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    K = N.K
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    scratch = torch.empty(1 << 28, device=dev)  # 1 GiB, unrelated to the codec's buffers
    lines = []
    for n in [int(s) for s in a.sizes.split(",")]:
        g = torch.Generator(device=dev).manual_seed(0x5EED)
        x = torch.randn(n, device=dev, generator=g) * 1e-3
        y = torch.empty_like(x)
        S = K.bagua_minmax_u8_compressed_bytes(F32, n, 1)
        So = K.bagua_onebit_compressed_bytes(n, 1)
        comp = torch.empty(S, dtype=torch.uint8, device=dev)
        compo = torch.empty(So, dtype=torch.uint8, device=dev)
        wsb = max(K.bagua_minmax_u8_workspace_bytes(n, 1), K.bagua_onebit_workspace_bytes(n, 1))
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        xp, yp, cp, cop, wp = x.data_ptr(), y.data_ptr(), comp.data_ptr(), compo.data_ptr(), ws.data_ptr()
        calls = {
            "minmax_partials_kernel": (lambda: K.bagua_minmax_u8_compress_stage(1, F32, xp, n, n, 1, cp, S, wp, wsb, -1,
                                                                                sp), 4 * n),
            "minmax_quantize_kernel": (lambda: K.bagua_minmax_u8_compress_stage(2, F32, xp, n, n, 1, cp, S, wp, wsb, -1,
                                                                                sp), 5 * n + 32),
            "minmax_dequantize_kernel": (lambda: K.bagua_minmax_u8_decompress(F32, cp, S, n, 1, yp, sp), 5 * n + 32),
            "onebit_encode_kernel": (lambda: K.bagua_onebit_compress(F32, xp, n, n, 1, cop, So, wp, wsb, -1, sp),
                                     4 * n + n // 8 + 4 * ((n + 1023) // 1024)),
            "onebit_decode_kernel": (lambda: K.bagua_onebit_decompress(F32, cop, So, n, 1, yp, sp), n // 8 + 32 + 4 * n),
        }
        # the predecessor each kernel has inside a codec step
        chain = {"minmax_partials_kernel": "minmax_dequantize_kernel",
                 "minmax_quantize_kernel": "minmax_partials_kernel",
                 "minmax_dequantize_kernel": "minmax_quantize_kernel",
                 "onebit_encode_kernel": "onebit_decode_kernel",
                 "onebit_decode_kernel": "onebit_encode_kernel"}
        for c, _ in calls.values():  # every buffer written once (valid headers for the decodes)
            N.check(c(), "warm")
        torch.cuda.synchronize()
        for name, (call, alg) in calls.items():
            for state in ("clean", "dirty", "chain"):
                us = []
                for _ in range(a.reps):
                    with torch.cuda.stream(stream):
                        if state == "clean":
                            scratch.sum()
                        elif state == "dirty":
                            scratch.fill_(1.0)
                    if state == "chain":
                        N.check(calls[chain[name]][0](), "predecessor")
                    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))]
                    ev[0][0].record(stream)
                    ev[0][1].record(stream)
                    N.time_next_kernels(ev)
                    N.check(call(), name)
                    N.check(K.bagua_time_next_kernels(None, None, 0), "disarm")
                    stream.synchronize()
                    us.append(ev[0][0].elapsed_time(ev[0][1]) * 1e3)
                us.sort()
                med = us[len(us) // 2]
                ln = {"elements": n, "mib": 4 * n >> 20, "kernel": name, "state": state, "median_us": round(med, 2),
                      "min_us": round(us[0], 2), "alg_bytes": alg, "tb_s": round(alg / (med * 1e-6) / 1e12, 3),
                      "frac_of_8tb_s": round(alg / (med * 1e-6) / 8e12, 4)}
                lines.append(ln)
                print(json.dumps(ln), flush=True)
        del x, y, comp, compo, ws
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            for ln in lines:
                f.write(json.dumps(ln) + "\n")


if __name__ == "__main__":
    main()
