"""Config-5 ring op (decentralized_low_precision_synchronous.rs:42-152) at one rank:
2^27 bf16 elements per tensor, the op through the C ABI on a single-rank RCCL
communicator, ms per step (run under rocprofv3 --kernel-trace --stats for the
per-kernel split).

  python tools/ring_probe.py [--elements N] [--steps K] [--pieces P]
"""
import argparse
import ctypes
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "bagua-core_amd"))

import bagua_core  # noqa: E402
from bagua_core import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elements", type=int, default=1 << 27)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--pieces", type=int, default=1)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16", "f32"])
    a = ap.parse_args()
    tdt = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32}[a.dtype]
    stream = torch.cuda.Stream()
    uid = bagua_core.BaguaSingleCommunicatorPy.generate_nccl_unique_id_str()
    comm = bagua_core.BaguaSingleCommunicatorPy(0, 1, 0, stream.cuda_stream, uid)
    g = torch.Generator(device="cuda").manual_seed(5)
    bufs = [(torch.randn(a.elements, device="cuda", generator=g) * 1e-3).to(tdt) for _ in range(4)]
    raws = [bagua_core.BaguaTensorPy(b, k).raw() for b, k in zip(bufs, "twlr")]

    def step():
        N.check(N.C.bagua_decentralized_low_precision_pipelined(comm.handle, *[ctypes.byref(r) for r in raws],
                                                                N.COMPRESSION_MINMAX_UINT8, a.pieces), "ring op")

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    print(f"ring op {a.dtype} n={a.elements} pieces={a.pieces}: {(time.perf_counter() - t0) * 1e3 / a.steps:.3f} ms/step")


if __name__ == "__main__":
    main()
