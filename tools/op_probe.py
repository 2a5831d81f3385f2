"""The compressed centralized op (centralized_low_precision_synchronous.rs:16-73) at
config-4 size, every kernel of it timed by its own HIP events, for rocprofv3
(--kernel-trace --stats, or one --pmc counter per run) to attribute time and HBM
bytes to the op's building blocks as the op itself runs them (not standalone).

  p = 1: a one-rank RCCL communicator; p > 1: p virtual ranks on the loopback
  transport (one host thread each, one GPU; their kernels overlap in time, so use
  p > 1 for counters, p = 1 for durations).

  python tools/op_probe.py --ranks 8 --method minmax --pieces 4 \
      [--elements 268435456] [--iters 3] [--json out.json]

The JSON lists, for rank 0's last op, every kernel in launch order with its
duration (us) -- the same order rocprofv3 records for that rank.
"""
import argparse
import ctypes
import json
import os
import sys
import threading

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "bagua-core_amd"))

import bagua_core  # noqa: E402
from bagua_core import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=1)
    ap.add_argument("--method", choices=["minmax", "onebit"], default="minmax")
    ap.add_argument("--pieces", type=int, default=4)
    ap.add_argument("--tapered", action="store_true")
    ap.add_argument("--elements", type=int, default=1 << 28)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    p, n = a.ranks, a.elements - a.elements % a.ranks
    method = N.COMPRESSION_MINMAX_UINT8 if a.method == "minmax" else N.COMPRESSION_ONEBIT
    sched = a.pieces | (N.PIECES_TAPERED if a.tapered else 0)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if p == 1:
        stream = torch.cuda.Stream(device=dev)
        comms = [bagua_core.BaguaSingleCommunicatorPy(0, 1, 0, stream.cuda_stream,
                                                      bagua_core.BaguaSingleCommunicatorPy.generate_nccl_unique_id_str())]
        streams = [stream]
    else:
        from bagua_core.communicator import loopback_communicators
        comms = loopback_communicators(p, 0)
        streams = [None] * p
    xs = []
    for r in range(p):
        g = torch.Generator(device=dev).manual_seed(0x5EED + r)
        xs.append(torch.randn(n, device=dev, generator=g) * 1e-3)
    torch.cuda.synchronize()
    raws = [bagua_core.BaguaTensorPy(x, f"g{r}").raw() for r, x in enumerate(xs)]
    record = {}

    def rank(r, timed):
        ev = None
        if timed and r == 0:
            st = torch.cuda.ExternalStream(comms[0].stream_ptr()) if p > 1 else streams[0]
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(32)]
            for x, y in ev:
                x.record(st)
                y.record(st)
            N.time_next_kernels(ev)
        N.check(N.C.bagua_centralized_low_precision_pipelined(comms[r].handle, ctypes.byref(raws[r]), 1, method,
                                                              sched), f"rank {r}")
        if ev is not None:
            names = N.timed_kernel_names()
            N.check(N.K.bagua_time_next_kernels(None, None, 0), "disarm")
            torch.cuda.synchronize()
            record["kernels"] = [{"i": i, "kernel": nm, "us": round(ev[i][0].elapsed_time(ev[i][1]) * 1e3, 2)}
                                 for i, nm in enumerate(names)]

    for it in range(a.iters):
        timed = it == a.iters - 1
        ths = [threading.Thread(target=rank, args=(r, timed)) for r in range(p)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        torch.cuda.synchronize()
        print(f"[op_probe] iteration {it} done", file=sys.stderr, flush=True)
    out = {"ranks": p, "method": a.method, "pieces": a.pieces, "tapered": a.tapered, "elements_per_rank": n,
           "kernels": record.get("kernels", [])}
    s = json.dumps(out)
    print(s)
    if a.json:
        with open(a.json, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
