"""Interleaved A/B of kernel-library builds on the same box, in one process.

Loads the in-tree libbagua_kernels.so (B, the candidate) and, with --base, a second
build of it (A, e.g. the previous commit built into ab_libs/base/), each through its
own ctypes handle, and times the same workloads on both, alternating A and B every
round so clock and thermal drift hit both alike.  Every launch is timed by the
library's own kernel-recorded events (bagua_time_next_kernel: hipExtLaunchKernel start
/ stop events around exactly that launch), and every workload's output bytes are
compared between A and B (a speed change must not move a byte).

  python3 tools/kernel_ab.py [--base ab_libs/base/libbagua_kernels.so]
        [--rounds 4] [--reps 10] [--only quant_bf16_ring,one_rank_1g]

Prints one JSON object: per workload, A and B median us per launch and the
algorithmic GB/s (DESIGN.md §5 bytes), plus `same_bytes`.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "bagua-core_amd"))

from bagua_core import _native as N  # noqa: E402  (signatures of the in-tree build)

F32, BF16 = 0, 2


def load(path: str):
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in N.KERNEL_SIGNATURES.items():
        try:
            f = getattr(lib, name)
        except AttributeError:
            continue
        f.restype, f.argtypes = res, args
    return lib


def workloads(dev, sp):
    """name -> (setup(lib) -> (launch(), output tensor), algorithmic bytes)"""
    g = torch.Generator(device=dev).manual_seed(11)
    nb, nf, ng = 1 << 27, 1 << 26, 1 << 28
    ring = {k: (torch.randn(nb, device=dev, generator=g) * 1e-3).to(torch.bfloat16) for k in "twlr"}
    xf = torch.randn(nf, device=dev, generator=g) * 1e-3
    xg = torch.randn(ng, device=dev, generator=g) * 1e-3
    W = {}

    def ring_bufs(lib):
        S = lib.bagua_minmax_u8_compressed_bytes(BF16, nb, 1)
        wsb = lib.bagua_minmax_u8_workspace_bytes(nb, 1)
        return (torch.empty(S, dtype=torch.uint8, device=dev), torch.empty(wsb, dtype=torch.uint8, device=dev), S, wsb)

    def mix_setup(lib):
        cb, ws, S, wsb = ring_bufs(lib)
        t = ring["t"].clone()

        def go():
            t.copy_(ring["t"])  # untimed: the timed launch is the mix
            return lambda: lib.bagua_ring_mix_minmax(BF16, t.data_ptr(), ring["l"].data_ptr(), ring["r"].data_ptr(),
                                                     ring["w"].data_ptr(), nb, ws.data_ptr(), wsb, sp)
        return go, t
    W["mix_bf16"] = (mix_setup, 10 * nb)

    def quant_ring_setup(lib):
        cb, ws, S, wsb = ring_bufs(lib)
        t = ring["t"].clone()
        assert lib.bagua_ring_mix_minmax(BF16, t.data_ptr(), ring["l"].data_ptr(), ring["r"].data_ptr(),
                                         ring["w"].data_ptr(), nb, ws.data_ptr(), wsb, sp) == 0
        return (lambda: (lambda: lib.bagua_minmax_u8_compress_stage(2, BF16, t.data_ptr(), nb, nb, 1, cb.data_ptr(), S,
                                                                     ws.data_ptr(), wsb, -1, sp))), cb
    W["quant_bf16_ring"] = (quant_ring_setup, 3 * nb + 32)

    def apply_setup(lib):
        cb, ws, S, wsb = ring_bufs(lib)
        t = ring["t"].clone()
        assert lib.bagua_ring_mix_minmax(BF16, t.data_ptr(), ring["l"].data_ptr(), ring["r"].data_ptr(),
                                         ring["w"].data_ptr(), nb, ws.data_ptr(), wsb, sp) == 0
        assert lib.bagua_minmax_u8_compress_stage(2, BF16, t.data_ptr(), nb, nb, 1, cb.data_ptr(), S, ws.data_ptr(),
                                                  wsb, -1, sp) == 0
        outs = {k: ring[k].clone() for k in "twlr"}

        def go():
            for k in "twlr":
                outs[k].copy_(ring[k])
            return lambda: lib.bagua_ring_apply_minmax(BF16, cb.data_ptr(), cb.data_ptr(), cb.data_ptr(), S, nb,
                                                       outs["t"].data_ptr(), outs["w"].data_ptr(),
                                                       outs["l"].data_ptr(), outs["r"].data_ptr(), sp)
        return go, outs["l"]
    W["apply_bf16"] = (apply_setup, 17 * nb)

    def twopass_setup(lib, n, x, stage):
        S = lib.bagua_minmax_u8_compressed_bytes(F32, n, 1)
        wsb = lib.bagua_minmax_u8_workspace_bytes(n, 1)
        cb = torch.empty(S, dtype=torch.uint8, device=dev)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        assert lib.bagua_minmax_u8_compress_stage(1, F32, x.data_ptr(), n, n, 1, cb.data_ptr(), S, ws.data_ptr(),
                                                  wsb, -1, sp) == 0
        if stage == 2:
            return (lambda: (lambda: lib.bagua_minmax_u8_compress_stage(2, F32, x.data_ptr(), n, n, 1, cb.data_ptr(), S,
                                                                         ws.data_ptr(), wsb, -1, sp))), cb
        assert lib.bagua_minmax_u8_compress_stage(2, F32, x.data_ptr(), n, n, 1, cb.data_ptr(), S, ws.data_ptr(),
                                                  wsb, -1, sp) == 0
        y = torch.empty_like(x)
        return (lambda: (lambda: lib.bagua_minmax_u8_decompress(F32, cb.data_ptr(), S, n, 1, y.data_ptr(), sp))), y
    W["quant_f32_256m"] = (lambda lib: twopass_setup(lib, nf, xf, 2), 5 * nf + 32)
    W["dequant_f32_256m"] = (lambda lib: twopass_setup(lib, nf, xf, 3), 5 * nf + 32)
    W["dequant_f32_1g"] = (lambda lib: twopass_setup(lib, ng, xg, 3), 5 * ng + 32)

    def one_rank_setup(lib, onebit):
        wsb = (lib.bagua_onebit_one_rank_workspace_bytes(ng) if onebit else lib.bagua_minmax_u8_workspace_bytes(ng, 1))
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        y = xg.clone()
        fn = lib.bagua_onebit_centralized_one_rank if onebit else lib.bagua_minmax_u8_centralized_one_rank

        def go():
            y.copy_(xg)
            return lambda: fn(F32, y.data_ptr(), ng, 1, ws.data_ptr(), wsb, sp)
        return go, y
    # Bagua's default 25 MiB bucket (the scheduler workload's unit): the one-rank op's two
    # kernels, and the one-launch encode of the same bucket (what a one-launch one-rank op
    # would cost before its larger write)
    ns = (25 << 20) // 4
    xs = torch.randn(ns, device=dev, generator=g) * 1e-3

    def small_setup(lib, encode):
        if encode:
            S = lib.bagua_minmax_u8_compressed_bytes(F32, ns, 1)
            wsb = lib.bagua_minmax_u8_workspace_bytes(ns, 1)
            cb = torch.empty(S, dtype=torch.uint8, device=dev)
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            return (lambda: (lambda: lib.bagua_minmax_u8_compress(F32, xs.data_ptr(), ns, ns, 1, cb.data_ptr(), S,
                                                                  ws.data_ptr(), wsb, -1, sp))), cb
        wsb = lib.bagua_minmax_u8_workspace_bytes(ns, 1)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        y = xs.clone()

        def go():
            y.copy_(xs)
            return lambda: lib.bagua_minmax_u8_centralized_one_rank(F32, y.data_ptr(), ns, 1, ws.data_ptr(), wsb, sp)
        return go, y
    W["one_rank_minmax_25m"] = (lambda lib: small_setup(lib, False), 12 * ns)
    W["one_rank_encode_25m"] = (lambda lib: small_setup(lib, True), 9 * ns)
    W["one_rank_minmax_1g"] = (lambda lib: one_rank_setup(lib, False), 12 * ng)
    W["one_rank_onebit_1g"] = (lambda lib: one_rank_setup(lib, True), 8 * ng + ng // 4)

    # whole comm ops at one rank through the C ABI (libbagua_core.so, a loopback communicator
    # on this stream): in-tree build only (op_*), timed by events around the call
    def op_setup(kind):
        from bagua_core.communicator import loopback_communicators
        comm = loopback_communicators(1, 0)[0]
        cst = ctypes.c_void_p(comm.stream_ptr())
        if kind == "ring":
            ts = {k: ring[k].clone() for k in "twlr"}
            raws = {k: N.bagua_tensor_t(ts[k].data_ptr(), nb, nb, BF16, 0) for k in "twlr"}

            def go():
                for k in "twlr":
                    ts[k].copy_(ring[k])
                torch.cuda.synchronize()
                return lambda: N.C.bagua_decentralized_low_precision_synchronous(
                    comm.handle, *[ctypes.byref(raws[k]) for k in "twlr"], N.COMPRESSION_MINMAX_UINT8)
            return go, ts["l"], comm
        y = xg.clone()
        raw = N.bagua_tensor_t(y.data_ptr(), ng, ng, F32, 0)
        method = N.COMPRESSION_ONEBIT if kind == "onebit" else N.COMPRESSION_MINMAX_UINT8

        def go():
            y.copy_(xg)
            torch.cuda.synchronize()
            return lambda: N.C.bagua_centralized_low_precision_synchronous(comm.handle, ctypes.byref(raw), 1, method)
        return go, y, comm
    W["op_ring_bf16_p1"] = (lambda lib: op_setup("ring"), 30 * nb)
    W["op_onebit_1g_p1"] = (lambda lib: op_setup("onebit"), 8 * ng + ng // 4)
    W["op_minmax_1g_p1"] = (lambda lib: op_setup("minmax"), 12 * ng)
    return W


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base", default="")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--only", default="")
    ap.add_argument("--variants", default="",
                    help='JSON list of environment dicts: the in-tree build under each (knob sweeps), '
                         'instead of the A/B of two builds')
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    libs = {"B": load(N.KERNELS_PATH)}
    envs = {"B": {}}
    if a.variants:
        base = libs["B"]
        libs, envs = {}, {}
        for i, e in enumerate(json.loads(a.variants)):
            libs[f"v{i}"], envs[f"v{i}"] = base, {k: str(v) for k, v in e.items()}
    elif a.base:
        libs["A"] = load(os.path.abspath(a.base))
        envs["A"] = {}
    W = workloads(dev, sp)
    names = [n for n in W if not a.only or n in a.only.split(",")]
    res = {}
    for name in names:
        setup, alg = W[name]
        times = {k: [] for k in libs}
        outs = {}
        for rnd in range(a.rounds):
            for k in (sorted(libs) if rnd % 2 == 0 else sorted(libs, reverse=True)):
                lib = libs[k]
                if not hasattr(lib, "bagua_onebit_centralized_one_rank") and "onebit" in name:
                    continue
                if name.startswith("op_") and lib is not libs.get("B", lib):
                    continue  # whole ops run through the in-tree libbagua_core.so only
                saved = {e: os.environ.get(e) for e in envs[k]}
                os.environ.update(envs[k])
                with torch.cuda.stream(st):
                    made = setup(lib)
                    go, out = made[0], made[1]
                    tst = torch.cuda.ExternalStream(made[2].stream_ptr()) if len(made) > 2 else st
                    for i in range(a.reps + 2):
                        fn = go()  # per-launch untimed reset (in-place workloads)
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        multi = name.startswith(("one_rank", "op_"))  # several launches: events around the call
                        e0.record(tst)
                        if multi:
                            rc = fn()
                            e1.record(tst)
                        else:
                            e1.record(tst)
                            assert lib.bagua_time_next_kernel(ctypes.c_void_p(e0.cuda_event),
                                                              ctypes.c_void_p(e1.cuda_event)) == 0
                            rc = fn()
                        assert rc == 0, (name, k, rc)
                        tst.synchronize()
                        if i >= 2:
                            times[k].append(e0.elapsed_time(e1) * 1e3)
                    outs[k] = out.view(torch.uint8).clone()
                torch.cuda.synchronize()
                for e, v in saved.items():
                    if v is None:
                        os.environ.pop(e, None)
                    else:
                        os.environ[e] = v
        entry = {}
        for k, v in times.items():
            if v:
                med = statistics.median(v)
                entry[k] = {"us_median": round(med, 2), "us_min": round(min(v), 2), "gb_s": round(alg / med / 1e3, 1),
                            "frac_of_8tbs": round(alg / med / 1e3 / 8000, 4)}
        if len(outs) >= 2:
            ref = outs[sorted(outs)[0]]
            entry["same_bytes"] = all(bool(torch.equal(ref, o)) for o in outs.values())
        if a.variants:
            entry["env"] = envs
        entry["alg_bytes"] = alg
        res[name] = entry
        print(json.dumps({name: entry}), file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
