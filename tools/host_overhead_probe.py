"""Host-side cost of enqueueing the codec and the comm op (no GPU wait inside the
timed loop, the GPU works behind): where the per-bucket host time of the
scheduler workload goes (profiles/r03_backend_trace_summary.json shows the GPU
idle 12-15 us between 25 MiB buckets).

  python tools/host_overhead_probe.py [--elements N]

Prints one JSON line: host us per call of each entry point (median of batches),
and the GPU time per call for comparison.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "bagua-core_amd"))

import bagua_core  # noqa: E402
from bagua_core import _native as N  # noqa: E402

K = N.K


def host_us(fn, calls=200, batches=5):
    """median host time per call; the stream is drained between batches"""
    out = []
    for _ in range(batches):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out.append(((t1 - t0) / calls * 1e6, (t2 - t0) / calls * 1e6))
    h = float(np.median([o[0] for o in out]))
    w = float(np.median([o[1] for o in out]))
    return round(h, 2), round(w, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elements", type=int, default=(25 << 20) // 4)
    a = ap.parse_args()
    n = a.elements
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    x = torch.randn(n, device=dev) * 1e-3
    y = torch.empty_like(x)
    S, W = K.bagua_minmax_u8_compressed_bytes(0, n, 1), K.bagua_minmax_u8_workspace_bytes(n, 1)
    comp = torch.empty(S, dtype=torch.uint8, device=dev)
    ws = torch.empty(W, dtype=torch.uint8, device=dev)
    xp, yp, cp, wp = x.data_ptr(), y.data_ptr(), comp.data_ptr(), ws.data_ptr()
    res = {"elements": n, "launch": "hipExtLaunchKernel"}
    res["compress_two_kernels"] = host_us(lambda: K.bagua_minmax_u8_compress(0, xp, n, n, 1, cp, S, wp, W, -1, sp))
    res["compress_stage1_one_kernel"] = host_us(
        lambda: K.bagua_minmax_u8_compress_stage(1, 0, xp, n, n, 1, cp, S, wp, W, -1, sp))
    res["decompress_one_kernel"] = host_us(lambda: K.bagua_minmax_u8_decompress(0, cp, S, n, 1, yp, sp))
    # the one-rank op's middle step alone (partials-only pass + requantise with the final values)
    res["reduce_requantize_final_two_kernels"] = host_us(
        lambda: K.bagua_minmax_u8_reduce_requantize_final(0, cp, S, n, 1, yp, 1, None, 0, 0, wp, W, sp))
    pool_ptr = ctypes.c_uint64(0)
    streams = (ctypes.c_uint64 * 1)(st.cuda_stream)

    def pool_cycle():
        N.C.bagua_pool_alloc(0, S, ctypes.byref(pool_ptr))
        N.C.bagua_pool_free_after(pool_ptr.value, streams, 1)
    res["pool_alloc_free_after"] = host_us(pool_cycle)
    res["hip_get_device"] = host_us(lambda: N.K.bagua_last_hip_error())
    ev0, ev1 = torch.cuda.Event(), torch.cuda.Event()
    res["hipEventRecord_pair"] = host_us(lambda: (ev0.record(st), ev1.record(st)))
    uid = bagua_core.BaguaSingleCommunicatorPy.generate_nccl_unique_id_str()
    comm = bagua_core.BaguaSingleCommunicatorPy(0, 1, 0, st.cuda_stream, uid)
    raw = bagua_core.BaguaTensorPy(x, "g").raw()
    N.check(N.C.bagua_comm_set_async(comm.handle, 1), "async")
    res["centralized_op_async"] = host_us(
        lambda: N.C.bagua_centralized_low_precision_synchronous(comm.handle, ctypes.byref(raw), 1,
                                                                N.COMPRESSION_MINMAX_UINT8), calls=100)
    N.check(N.C.bagua_comm_set_async(comm.handle, 0), "sync")
    res["centralized_op_sync"] = host_us(
        lambda: N.C.bagua_centralized_low_precision_synchronous(comm.handle, ctypes.byref(raw), 1,
                                                                N.COMPRESSION_MINMAX_UINT8), calls=50)
    res["note"] = "(host us per call, host+GPU wall us per call) -- medians of 5 batches"
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
