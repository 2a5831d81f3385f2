"""The config-2 codec step (256 MiB fp32 MinMax-UInt8 encode + decode) while a
compute-bound kernel stream runs beside it, as in Bagua, where the comm ops
overlap the backward pass (DESIGN.md §5.1 "Under contention").

  python tools/contention_probe.py [--gemm 8192] [--modes resident,two_pass]

Per encode mode (the one-launch encode, or BAGUA_RESIDENT=0's two kernels):
  alone       : codec steps on stream A only
  concurrent  : bf16 GEMMs (M=N=K=--gemm, torch.matmul -> hipBLASLt) queued on
                stream B, and codec steps on stream A sized to last about as long
                as the GEMM queue alone did
Reported: the encode's per-launch duration (kernel-recorded HIP events), the
decode's, the codec loop's wall time, the workgroups of the one-launch encode
that gave up waiting in the exchange (device counter), and the GEMM queue's
wall time / TFLOP/s alone and beside the codec.  One JSON line per mode and
GEMM size.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "bagua-core_amd"))

from bagua_core import _native as N  # noqa: E402

K = N.K


def stats(a):
    a = np.asarray(a, np.float64)
    return {"mean": round(float(a.mean()), 2), "p50": round(float(np.median(a)), 2),
            "p90": round(float(np.percentile(a, 90)), 2), "max": round(float(a.max()), 2), "n": int(a.size)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gemm", default="8192,4096")
    ap.add_argument("--gemms", type=int, default=60, help="GEMMs queued on stream B")
    ap.add_argument("--modes", default="resident,two_pass")
    ap.add_argument("--elements", type=int, default=1 << 26)
    a = ap.parse_args()
    n = a.elements
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0x5EED)
    x = torch.randn(n, device=dev, generator=g) * 1e-3
    y = torch.empty_like(x)
    S = K.bagua_minmax_u8_compressed_bytes(0, n, 1)
    wsb = K.bagua_minmax_u8_workspace_bytes(n, 1)
    comp = torch.empty(S, dtype=torch.uint8, device=dev)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    sa, sb = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    spa = ctypes.c_void_p(sa.cuda_stream)
    torch.cuda.synchronize()
    want = None

    def give_ups():
        c = ctypes.c_uint64(0)
        N.check(K.bagua_minmax_u8_resident_give_ups(spa, ctypes.byref(c)), "give_ups")
        return int(c.value)

    def codec(steps):
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)]
        for row in ev:
            for e in row:
                e.record(sa)
        w0, w1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        w0.record(sa)
        for k in range(steps):
            K.bagua_time_next_kernel(ev[k][0].cuda_event, ev[k][1].cuda_event)
            N.check(K.bagua_minmax_u8_compress(0, x.data_ptr(), n, n, 1, comp.data_ptr(), S, ws.data_ptr(), wsb, -1,
                                               spa), "compress")
            K.bagua_time_next_kernel(ev[k][2].cuda_event, ev[k][3].cuda_event)
            N.check(K.bagua_minmax_u8_decompress(0, comp.data_ptr(), S, n, 1, y.data_ptr(), spa), "decompress")
        w1.record(sa)
        return ev, (w0, w1)

    def codec_result(ev, w):
        enc = [r[0].elapsed_time(r[1]) * 1e3 for r in ev]
        dec = [r[2].elapsed_time(r[3]) * 1e3 for r in ev]
        return enc, dec, w[0].elapsed_time(w[1])

    for m in [int(v) for v in a.gemm.split(",")]:
        A = torch.randn(m, m, device=dev, dtype=torch.bfloat16)
        B = torch.randn(m, m, device=dev, dtype=torch.bfloat16)
        C = torch.empty(m, m, device=dev, dtype=torch.bfloat16)

        def gemms(count):
            w0, w1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(sb):
                w0.record(sb)
                for _ in range(count):
                    torch.matmul(A, B, out=C)
                w1.record(sb)
            return w0, w1

        gemms(5)
        torch.cuda.synchronize()
        w = gemms(a.gemms)
        torch.cuda.synchronize()
        gemm_alone_ms = w[0].elapsed_time(w[1])
        flops = 2.0 * m * m * m * a.gemms
        for mode in a.modes.split(","):
            if mode == "two_pass":
                os.environ["BAGUA_RESIDENT"] = "0"
            else:
                os.environ.pop("BAGUA_RESIDENT", None)
            ev, cw = codec(5)
            torch.cuda.synchronize()
            ev, cw = codec(40)
            torch.cuda.synchronize()
            enc0, dec0, wall0 = codec_result(ev, cw)
            steps = max(10, int(gemm_alone_ms / (wall0 / 40)))
            gu0 = give_ups()
            torch.cuda.synchronize()
            gw = gemms(a.gemms)   # B first, so every codec step starts against running GEMMs
            ev, cw = codec(steps)
            torch.cuda.synchronize()
            enc1, dec1, wall1 = codec_result(ev, cw)
            gu1 = give_ups()
            gemm_ms = gw[0].elapsed_time(gw[1])
            h = comp.cpu()
            if want is None:
                want = h
            same = bool(torch.equal(h, want))
            print(json.dumps({
                "gemm_mnk": m, "mode": mode, "bytes_identical_across_modes": same,
                "alone": {"encode_us": stats(enc0), "decode_us": stats(dec0), "step_us": round(wall0 / 40 * 1e3, 2)},
                "concurrent": {"encode_us": stats(enc1), "decode_us": stats(dec1),
                               "step_us": round(wall1 / steps * 1e3, 2), "codec_steps": steps,
                               "give_ups_workgroups": gu1 - gu0, "resident_launches": steps if mode == "resident" else 0},
                "gemm": {"count": a.gemms, "alone_ms": round(gemm_alone_ms, 3), "concurrent_ms": round(gemm_ms, 3),
                         "alone_tflops": round(flops / gemm_alone_ms / 1e9, 1),
                         "concurrent_tflops": round(flops / gemm_ms / 1e9, 1),
                         "slowdown": round(gemm_ms / gemm_alone_ms, 3)},
            }), flush=True)
        os.environ.pop("BAGUA_RESIDENT", None)
        del A, B, C


if __name__ == "__main__":
    main()
