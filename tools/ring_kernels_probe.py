"""Config-5 ring kernels (decentralized_low_precision_synchronous.rs:45-64,126-151) one
by one, with THREE DISTINCT compressed payloads for the apply pass: the shipped
ring_mix -> MinMax quantise (stage 2) -> ring_apply sequence of the fused op on
2^27 bf16 elements, where the buffers received from the left and right peer are
copies of `mine` made OUTSIDE the timed kernels (a one-rank op reads its own bytes
for both peers, so two of the apply pass's three payload streams would alias one
134 MB buffer and flatter its rate).  Every kernel is timed by its own HIP events
(bagua_time_next_kernels); run under rocprofv3 --kernel-trace --stats or --pmc for
the per-kernel durations and HBM bytes.

Algorithmic bytes per launch, N elements of T (sizeof 2), the MinMax payload N + 32:
  ring_mix            t, l, r, w read, t written              -> 5 x 2N = 10N
  minmax_quantize     t read, payload written                 -> 2N + N   = 3N
  ring_apply          3 payloads read; l, r read + written;
                      w read; t written; w written (t)        -> 3N + 7 x 2N = 17N

  python tools/ring_kernels_probe.py [--elements N] [--steps K] [--json out]
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

BF16 = 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elements", type=int, default=1 << 27)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    n = a.elements
    K = N.K
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    g = torch.Generator(device=dev).manual_seed(5)
    t, w, l, r = [(torch.randn(n, device=dev, generator=g) * 1e-3).to(torch.bfloat16) for _ in range(4)]
    S = K.bagua_minmax_u8_compressed_bytes(BF16, n, 1)
    mine, lb, rb = [torch.zeros(S, dtype=torch.uint8, device=dev) for _ in range(3)]
    wsb = K.bagua_minmax_u8_workspace_bytes(n, 1)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    alg = {"ring_mix_kernel": 10 * n, "minmax_quantize_kernel": 3 * n + 32, "ring_apply_kernel": 17 * n + 96}
    times = {k: [] for k in alg}
    names_seen = []

    def step(timed):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
        for x, y in ev:
            x.record(stream)
            y.record(stream)
        if timed:
            N.time_next_kernels(ev[:2])
        N.check(K.bagua_ring_mix_minmax(BF16, t.data_ptr(), l.data_ptr(), r.data_ptr(), w.data_ptr(), n,
                                        ws.data_ptr(), wsb, sp), "mix")
        N.check(K.bagua_minmax_u8_compress_stage(2, BF16, t.data_ptr(), n, n, 1, mine.data_ptr(), S, ws.data_ptr(),
                                                 wsb, -1, sp), "quantise")
        names = N.timed_kernel_names() if timed else []
        with torch.cuda.stream(stream):  # the peers' payloads: distinct buffers, untimed copies
            lb.copy_(mine)
            rb.copy_(mine)
        if timed:
            N.time_next_kernels(ev[2:])
        N.check(K.bagua_ring_apply_minmax(BF16, mine.data_ptr(), lb.data_ptr(), rb.data_ptr(), S, n, t.data_ptr(),
                                          w.data_ptr(), l.data_ptr(), r.data_ptr(), sp), "apply")
        if timed:
            names = names + N.timed_kernel_names()
            N.check(K.bagua_time_next_kernels(None, None, 0), "disarm")
            stream.synchronize()
            for (x, y), nm in zip(ev, names):
                if nm in times:
                    times[nm].append(x.elapsed_time(y) * 1e3)
            names_seen[:] = names

    for _ in range(3):
        step(False)
    for _ in range(a.steps):
        step(True)
    torch.cuda.synchronize()
    out = {"elements": n, "dtype": "bf16", "distinct_payloads": True, "steps": a.steps, "kernels": {}}
    for k, v in times.items():
        if not v:
            continue
        us = sorted(v)[len(v) // 2]
        out["kernels"][k] = {"median_us": round(us, 2), "mean_us": round(sum(v) / len(v), 2),
                             "alg_bytes": alg[k], "tb_s": round(alg[k] / (us * 1e-6) / 1e12, 3),
                             "frac_of_8tb_s": round(alg[k] / (us * 1e-6) / 8e12, 4)}
    out["kernel_order"] = names_seen
    s = json.dumps(out)
    print(s)
    if a.json:
        with open(a.json, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
