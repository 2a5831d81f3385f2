#!/usr/bin/env python3
"""Dev probe: the config-2 step (MinMax encode + decode of a 256 MiB fp32 bucket)
launched eagerly vs replayed from a HIP graph (both kernels captured once),
wall time per step over the same number of steps, interleaved.

    python tools/graph_step_probe.py [--steps 200]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bagua-core_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    from bagua_core import _native as N
    K = N.K
    n = 1 << 26
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0x5EED)
    x = torch.randn(n, device=dev, generator=g) * 1e-3
    y = torch.empty_like(x)
    S = K.bagua_minmax_u8_compressed_bytes(0, n, 1)
    wsb = K.bagua_minmax_u8_workspace_bytes(n, 1)
    comp = torch.empty(S, dtype=torch.uint8, device=dev)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream()

    def step(s):
        sp = ctypes.c_void_p(s.cuda_stream)
        assert K.bagua_minmax_u8_compress(0, x.data_ptr(), n, n, 1, comp.data_ptr(), S, ws.data_ptr(), wsb, -1, sp) == 0
        assert K.bagua_minmax_u8_decompress(0, comp.data_ptr(), S, n, 1, y.data_ptr(), sp) == 0

    with torch.cuda.stream(st):
        for _ in range(5):
            step(st)
    torch.cuda.synchronize()
    eager_y = y.clone()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=st, capture_error_mode="relaxed"):
        step(st)
    torch.cuda.synchronize()

    def eager(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(st):
            for _ in range(k):
                step(st)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e6

    def replay(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(st):
            for _ in range(k):
                graph.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e6

    res = {"eager_us": [], "graph_us": []}
    for _ in range(3):
        res["eager_us"].append(round(eager(args.steps), 2))
        res["graph_us"].append(round(replay(args.steps), 2))
    res["bit_identical"] = bool(torch.equal(y, eager_y))
    res["gib_s_eager"] = round(4 * n / (min(res["eager_us"]) * 1e-6) / (1 << 30), 1)
    res["gib_s_graph"] = round(4 * n / (min(res["graph_us"]) * 1e-6) / (1 << 30), 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
