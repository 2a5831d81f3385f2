"""A/B of the one-rank op's min/max load policy at config-4 size (1 GiB fp32).

The op (minmax_u8.hip one_rank_impl) runs the min/max pass forward, then the table
pass backwards.  BAGUA_ONE_RANK_KEEP_MIB=k loads all but the last k MiB of the
min/max pass non-temporally (unset: every load with the default policy).  Variants
interleave over rounds; each prints one JSON line with the op's wall time per call
and both kernels' own event times (bagua_time_next_kernels).

usage: python3 tools/one_rank_keep_probe.py [--mib 1024] [--rounds 3] [--keeps -1,0,64,128,192,256]
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bagua-core_amd"))

import torch  # noqa: E402

from bagua_core import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--keeps", default="-1,0,64,128,192,256")
    a = ap.parse_args()
    n = (a.mib << 20) // 4
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    g = torch.Generator(device=dev).manual_seed(0x5EED)
    x = torch.randn(n, device=dev, generator=g) * 1e-3
    wsb = N.K.bagua_minmax_u8_workspace_bytes(n, 1)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    sp = ctypes.c_void_p(stream.cuda_stream)

    def op():
        N.check(N.K.bagua_minmax_u8_centralized_one_rank(0, x.data_ptr(), n, 1, ws.data_ptr(), wsb, sp), "op")

    keeps = [int(k) for k in a.keeps.split(",")]
    for r in range(a.rounds):
        for k in keeps:
            if k < 0:
                os.environ.pop("BAGUA_ONE_RANK_KEEP_MIB", None)
            else:
                os.environ["BAGUA_ONE_RANK_KEEP_MIB"] = str(k)
            for _ in range(5):
                op()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                op()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.steps * 1e3
            kern = {}
            for _ in range(3):
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(2)]
                for e0, e1 in ev:
                    e0.record(stream)
                    e1.record(stream)
                N.time_next_kernels(ev)
                op()
                names = N.timed_kernel_names()
                N.check(N.K.bagua_time_next_kernels(None, None, 0), "disarm")
                torch.cuda.synchronize()
                for i, nm in enumerate(names):
                    kern.setdefault(nm, []).append(ev[i][0].elapsed_time(ev[i][1]) * 1e3)
            print(json.dumps({"round": r, "keep_mib": k, "mib": a.mib, "ms_per_op": round(ms, 4),
                              "kernel_us": {nm: round(sum(v) / len(v), 1) for nm, v in kern.items()}}), flush=True)


if __name__ == "__main__":
    main()
