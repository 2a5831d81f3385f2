"""Variants of the config-5 apply pass (ring_apply_kernel, decentralized.hip;
BAGUA_RING_APPLY_CFG) on 2^27 bf16 elements: store policy per output, nt loads,
contiguous ranges, unroll, grid size.

  python tools/ring_apply_sweep.py [--cfgs 0,1,2,...] [--rounds 4]

1. every variant's four outputs must equal variant 0's bit for bit (one apply
   from the same saved state);
2. interleaved rounds: per variant, the apply alone repeated (kernel-recorded
   HIP events: bagua_time_next_kernel) and the whole ring op at one rank (the
   mix pass of the next step reads what the apply stored, so store policy
   shows up there too), ms per step.
One JSON line per (round, cfg) and a summary per cfg.
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
BF16 = 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="0,1,2,3,4,5,6,7,8,9")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--elements", type=int, default=1 << 27)
    ap.add_argument("--mix", action="store_true", help="also A/B the mix pass (BAGUA_RING_MIX_CONTIG)")
    a = ap.parse_args()
    n = a.elements
    cfgs = [int(c) for c in a.cfgs.split(",")]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    g = torch.Generator(device=dev).manual_seed(11)
    tens = {k: (torch.randn(n, device=dev, generator=g) * 1e-3).to(torch.bfloat16) for k in "twlr"}
    S = K.bagua_minmax_u8_compressed_bytes(BF16, n, 1)
    wsb = K.bagua_minmax_u8_workspace_bytes(n, 1)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    comp = {}
    for k in ("mine", "left", "right"):
        src = (torch.randn(n, device=dev, generator=g) * 1e-3).to(torch.bfloat16)
        comp[k] = torch.empty(S, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        N.check(K.bagua_minmax_u8_compress(BF16, src.data_ptr(), n, n, 1, comp[k].data_ptr(), S, ws.data_ptr(), wsb,
                                           -1, sp), "compress")
    torch.cuda.synchronize()
    init = {k: v.clone() for k, v in tens.items()}

    def apply_once():
        return K.bagua_ring_apply_minmax(BF16, comp["mine"].data_ptr(), comp["left"].data_ptr(),
                                         comp["right"].data_ptr(), S, n, tens["t"].data_ptr(), tens["w"].data_ptr(),
                                         tens["l"].data_ptr(), tens["r"].data_ptr(), sp)

    ref = None
    for c in cfgs:
        os.environ["BAGUA_RING_APPLY_CFG"] = str(c)
        for k in tens:
            tens[k].copy_(init[k])
        torch.cuda.synchronize()
        N.check(apply_once(), f"apply cfg {c}")
        torch.cuda.synchronize()
        out = torch.cat([tens[k].view(torch.int16) for k in "twlr"]).cpu()
        if ref is None:
            ref = out
        assert torch.equal(out, ref), f"cfg {c}: outputs differ from cfg {cfgs[0]}"

    uid = bagua_core.BaguaSingleCommunicatorPy.generate_nccl_unique_id_str()
    comm = bagua_core.BaguaSingleCommunicatorPy(0, 1, 0, stream.cuda_stream, uid)
    raws = [bagua_core.BaguaTensorPy(tens[k], k).raw() for k in "twlr"]

    def op():
        N.check(N.C.bagua_decentralized_low_precision_pipelined(comm.handle, *[ctypes.byref(r) for r in raws],
                                                                N.COMPRESSION_MINMAX_UINT8, 1), "ring op")

    res = {c: {"apply_us": [], "op_ms": []} for c in cfgs}
    for rnd in range(a.rounds):
        order = cfgs if rnd % 2 == 0 else cfgs[::-1]
        for c in order:
            os.environ["BAGUA_RING_APPLY_CFG"] = str(c)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
            for e0, e1 in ev:
                e0.record(stream)
                e1.record(stream)
            for _ in range(3):
                apply_once()
            for e0, e1 in ev:
                K.bagua_time_next_kernel(e0.cuda_event, e1.cuda_event)
                apply_once()
            torch.cuda.synchronize()
            us = float(np.mean([e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]))
            for _ in range(2):
                op()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                op()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / a.steps
            res[c]["apply_us"].append(us)
            res[c]["op_ms"].append(ms)
            print(json.dumps({"round": rnd, "cfg": c, "apply_us": round(us, 2), "op_ms": round(ms, 4)}), flush=True)
    alg = 17 * n  # SURVEY-style bytes of the apply pass: 3 payloads + 3 tensors read (2 B), 4 tensors written
    for c in cfgs:
        us = float(np.mean(res[c]["apply_us"]))
        print(json.dumps({"cfg": c, "summary": True, "apply_us_mean": round(us, 2),
                          "apply_us_min": round(min(res[c]["apply_us"]), 2),
                          "apply_tbs": round(alg / (us * 1e-6) / 1e12, 3),
                          "apply_frac_of_8tbs": round(alg / (us * 1e-6) / 8e12, 4),
                          "op_ms_mean": round(float(np.mean(res[c]["op_ms"])), 4),
                          "identical_outputs": True}), flush=True)
    os.environ.pop("BAGUA_RING_APPLY_CFG", None)
    if a.mix:
        mix_ab(a, n, tens, init, comp["mine"], S, ws, wsb, stream, sp)


def mix_ab(a, n, tens, init, out, S, ws, wsb, stream, sp):
    """ring_mix_kernel grid-strided vs contiguous ranges (BAGUA_RING_MIX_CONTIG):
    identical mixed tensor and identical quantised bytes (the quantise pass folds
    the mix's min/max partials), then the mix alone timed, interleaved."""
    def mix():
        return K.bagua_ring_mix_minmax(BF16, tens["t"].data_ptr(), tens["l"].data_ptr(), tens["r"].data_ptr(),
                                       tens["w"].data_ptr(), n, ws.data_ptr(), wsb, sp)

    ref = None
    for c in ("0", "1"):
        os.environ["BAGUA_RING_MIX_CONTIG"] = c
        for k in tens:
            tens[k].copy_(init[k])
        torch.cuda.synchronize()
        N.check(mix(), "mix")
        N.check(K.bagua_minmax_u8_compress_stage(2, BF16, tens["t"].data_ptr(), n, n, 1, out.data_ptr(), S,
                                                 ws.data_ptr(), wsb, -1, sp), "quantise")
        torch.cuda.synchronize()
        got = (tens["t"].view(torch.int16).cpu(), out.cpu())
        if ref is None:
            ref = got
        assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]), "mix variants differ"
    res = {"0": [], "1": []}
    for rnd in range(a.rounds):
        for c in (("0", "1") if rnd % 2 == 0 else ("1", "0")):
            os.environ["BAGUA_RING_MIX_CONTIG"] = c
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
            for e0, e1 in ev:
                e0.record(stream)
                e1.record(stream)
            for _ in range(3):
                mix()
            for e0, e1 in ev:
                K.bagua_time_next_kernel(e0.cuda_event, e1.cuda_event)
                mix()
            torch.cuda.synchronize()
            res[c].append(float(np.mean([e0.elapsed_time(e1) * 1e3 for e0, e1 in ev])))
    for c in ("0", "1"):
        us = float(np.mean(res[c]))
        print(json.dumps({"mix_contig": c == "1", "summary": True, "mix_us_mean": round(us, 2),
                          "mix_tbs": round(10 * n / (us * 1e-6) / 1e12, 3),
                          "mix_frac_of_8tbs": round(10 * n / (us * 1e-6) / 8e12, 4), "identical_outputs": True}),
              flush=True)
    os.environ.pop("BAGUA_RING_MIX_CONTIG", None)


if __name__ == "__main__":
    main()
