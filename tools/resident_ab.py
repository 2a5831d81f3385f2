"""Interleaved A/B of kernel-library builds on the config-2 step (256 MiB fp32,
MinMax-UInt8 encode + decode), in ONE process on one box: every library is
loaded side by side (ctypes, RTLD_LOCAL, by path), and rounds alternate the
order, so box and clock drift hit every build alike.

  python tools/resident_ab.py --lib r01=ab_libs/r01/libbagua_kernels.so \
      --lib head=bagua-core_amd/lib/libbagua_kernels.so [--rounds 8 --steps 40]

Per build: every encode and decode launch is timed by the kernel's own HIP
events (bagua_time_next_kernel -> hipExtLaunchKernel, no dispatch gap), so the
output has the per-launch distribution (mean, p50, p90, max) and the step wall
time of an event-free loop.  Builds that export bagua_minmax_u8_resident_give_ups
report how many workgroups gave up waiting in the exchange.  With --trace the
last build also runs a stamped pass (bagua_minmax_u8_resident_trace, a buffer
per launch) and prints the phase split of its slowest launches.

One JSON line per (round, build), then one summary line per build.
"""
import argparse
import ctypes
import json
import os
import time

import numpy as np
import torch

_vp, _sz, _i32, _u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64


def load(path):
    L = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL | os.RTLD_NOW)
    L.bagua_minmax_u8_compressed_bytes.restype = _sz
    L.bagua_minmax_u8_compressed_bytes.argtypes = [_i32, _i32, _i32]
    L.bagua_minmax_u8_workspace_bytes.restype = _sz
    L.bagua_minmax_u8_workspace_bytes.argtypes = [_i32, _i32]
    L.bagua_minmax_u8_compress.argtypes = [_i32, _vp, _i32, _i32, _i32, _vp, _sz, _vp, _sz, _i32, _vp]
    L.bagua_minmax_u8_decompress.argtypes = [_i32, _vp, _sz, _i32, _i32, _vp, _vp]
    L.bagua_time_next_kernel.argtypes = [_vp, _vp]
    L.bagua_minmax_u8_resident_trace.argtypes = [_vp]
    L.bagua_minmax_u8_resident_path.argtypes = [_i32, _vp, _i32, _i32, _i32, _vp, _sz, _i32, _vp]
    L.bagua_onebit_compressed_bytes.restype = _sz
    L.bagua_onebit_compressed_bytes.argtypes = [_i32, _i32]
    L.bagua_onebit_workspace_bytes.restype = _sz
    L.bagua_onebit_workspace_bytes.argtypes = [_i32, _i32]
    L.bagua_onebit_compress.argtypes = [_i32, _vp, _i32, _i32, _i32, _vp, _sz, _vp, _sz, _i32, _vp]
    L.bagua_onebit_decompress.argtypes = [_i32, _vp, _sz, _i32, _i32, _vp, _vp]
    try:
        L.bagua_minmax_u8_resident_give_ups.argtypes = [_vp, ctypes.POINTER(_u64)]
        gu = L.bagua_minmax_u8_resident_give_ups
    except AttributeError:
        gu = None
    return L, gu


def stats(a):
    a = np.asarray(a, np.float64)
    return {"mean": round(float(a.mean()), 2), "p50": round(float(np.median(a)), 2),
            "p90": round(float(np.percentile(a, 90)), 2), "max": round(float(a.max()), 2), "n": int(a.size)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", required=True, help="name=path")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--elements", type=int, default=1 << 26)
    ap.add_argument("--trace", action="store_true")
    ap.add_argument("--onebit", action="store_true", help="the 1-bit codec (config 3) instead of MinMax")
    a = ap.parse_args()
    libs = []
    for spec in a.lib:
        name, path = spec.split("=", 1)
        L, gu = load(path)
        libs.append((name, L, gu))
    n = a.elements
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0x5EED)
    x = torch.randn(n, device=dev, generator=g) * 1e-3
    y = torch.empty_like(x)
    st = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    L0 = libs[0][1]
    if a.onebit:
        S = L0.bagua_onebit_compressed_bytes(n, 1)
        wsb = max(L.bagua_onebit_workspace_bytes(n, 1) for _, L, _ in libs)
    else:
        S = L0.bagua_minmax_u8_compressed_bytes(0, n, 1)
        wsb = max(L.bagua_minmax_u8_workspace_bytes(n, 1) for _, L, _ in libs)
    comp = torch.empty(S, dtype=torch.uint8, device=dev)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)

    def enc(L):
        f = L.bagua_onebit_compress if a.onebit else L.bagua_minmax_u8_compress
        return f(0, x.data_ptr(), n, n, 1, comp.data_ptr(), S, ws.data_ptr(), wsb, -1, sp)

    def dec(L):
        f = L.bagua_onebit_decompress if a.onebit else L.bagua_minmax_u8_decompress
        return f(0, comp.data_ptr(), S, n, 1, y.data_ptr(), sp)

    torch.cuda.synchronize()
    ref = None
    for name, L, _ in libs:  # every build must produce the same bytes
        assert enc(L) == 0
        torch.cuda.synchronize()
        h = comp.cpu()
        if ref is None:
            ref = h
        assert torch.equal(h, ref), f"{name}: compressed bytes differ"

    def run(L, steps, events):
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)] if events else None
        if events:
            for row in ev:
                for e in row:
                    e.record(st)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            if events:
                L.bagua_time_next_kernel(ev[k][0].cuda_event, ev[k][1].cuda_event)
            enc(L)
            if events:
                L.bagua_time_next_kernel(ev[k][2].cuda_event, ev[k][3].cuda_event)
            dec(L)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / steps * 1e6
        if not events:
            return wall, None, None
        te = [r[0].elapsed_time(r[1]) * 1e3 for r in ev]
        td = [r[2].elapsed_time(r[3]) * 1e3 for r in ev]
        return wall, te, td

    allenc = {nm: [] for nm, _, _ in libs}
    alldec = {nm: [] for nm, _, _ in libs}
    allwall = {nm: [] for nm, _, _ in libs}
    for r in range(a.rounds):
        order = libs if r % 2 == 0 else libs[::-1]
        for name, L, gu in order:
            run(L, 5, False)
            wall, _, _ = run(L, a.steps, False)
            _, te, td = run(L, a.steps, True)
            allenc[name] += te
            alldec[name] += td
            allwall[name].append(wall)
            print(json.dumps({"round": r, "build": name, "step_wall_us": round(wall, 2), "encode_us": stats(te),
                              "decode_us": stats(td)}), flush=True)
    for name, L, gu in libs:
        out = {"build": name, "summary": True, "encode_us": stats(allenc[name]), "decode_us": stats(alldec[name]),
               "step_wall_us": stats(allwall[name])}
        if gu is not None and not a.onebit:
            cnt = ctypes.c_uint64(0)
            gu(sp, ctypes.byref(cnt))
            out["give_ups_total"] = int(cnt.value)
            out["launches_total"] = a.rounds * (2 * a.steps + 5) + 1
        print(json.dumps(out), flush=True)
    if a.trace and not a.onebit:
        name, L, gu = libs[-1]
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        steps = a.steps * 2
        tr = torch.zeros(steps, 8 * cus, dtype=torch.int64, device=dev)
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(steps)]
        for row in ev:
            for e in row:
                e.record(st)
        torch.cuda.synchronize()
        for k in range(steps):
            L.bagua_minmax_u8_resident_trace(ctypes.c_void_p(tr[k].data_ptr()))
            L.bagua_time_next_kernel(ev[k][0].cuda_event, ev[k][1].cuda_event)
            L.bagua_minmax_u8_compress(0, x.data_ptr(), n, n, 1, comp.data_ptr(), S, ws.data_ptr(), wsb, -1, sp)
            L.bagua_minmax_u8_resident_trace(None)
            L.bagua_minmax_u8_decompress(0, comp.data_ptr(), S, n, 1, y.data_ptr(), sp)
        torch.cuda.synchronize()
        dur = np.array([r[0].elapsed_time(r[1]) * 1e3 for r in ev])
        t = tr.cpu().numpy().reshape(steps, cus, 8).astype(np.float64) / 100.0  # 100 MHz wall clock -> us
        t -= t[:, :, 0].min(axis=1)[:, None, None]

        def phases(k):
            u = t[k]
            return {"launch_us": round(float(dur[k]), 2),
                    "start_spread_us": round(float(u[:, 0].max()), 2),
                    "pass1_end_max_us": round(float(u[:, 1].max()), 2),
                    "pass1_end_min_us": round(float(u[:, 1].min()), 2),
                    "exchange_end_max_us": round(float(u[:, 2].max()), 2),
                    "exchange_wait_max_us": round(float((u[:, 2] - u[:, 1]).max()), 2),
                    "pass2_stream_max_us": round(float((u[:, 4] - u[:, 2]).max()), 2),
                    "end_max_us": round(float(u[:, 3].max()), 2),
                    "slowest_wg": int(u[:, 3].argmax()),
                    "slowest_wg_pass1_us": round(float(u[u[:, 3].argmax(), 1] - u[u[:, 3].argmax(), 0]), 2)}

        order = np.argsort(dur)
        print(json.dumps({"build": name, "trace": "median launch", **phases(int(order[len(order) // 2]))}), flush=True)
        for k in order[-3:][::-1]:
            print(json.dumps({"build": name, "trace": "slow launch", "index": int(k), **phases(int(k))}), flush=True)


if __name__ == "__main__":
    main()
