"""Launch-shape sweep of the streaming codec kernels on the config-2/3 steps
(256 MiB fp32 bucket): workgroups per launch of the MinMax dequantise, the
two-pass quantise and the 1-bit encode / decode (BAGUA_TUNE_* knobs, read per
call; launch_util.hpp tune_int).  A grid-strided kernel with a few workgroups
per CU vs one tile per workgroup (the hardware dispatcher then balances the
tail; the ring apply pass gained 20 % that way, profiles/r03_ring_apply_sweep3.jsonl).

  python tools/grid_sweep.py [--rounds 4 --steps 30]

Every variant's compressed bytes and decoded floats must equal the first
variant's of its workload.  One JSON line per (round, variant), then summaries.
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

VARIANTS = [
    # (workload, label, env)
    ("minmax", "dequant4096", {}),
    ("minmax", "dequant8192", {"BAGUA_TUNE_DEQUANT_BLOCKS": "8192"}),
    ("minmax", "dequant16384", {"BAGUA_TUNE_DEQUANT_BLOCKS": "16384"}),
    ("minmax", "dequant65536", {"BAGUA_TUNE_DEQUANT_BLOCKS": "65536"}),
    ("twopass", "quant2048", {"BAGUA_RESIDENT": "0"}),
    ("twopass", "quant8192", {"BAGUA_RESIDENT": "0", "BAGUA_TUNE_QUANT_BLOCKS": "8192"}),
    ("twopass", "quant16384", {"BAGUA_RESIDENT": "0", "BAGUA_TUNE_QUANT_BLOCKS": "16384"}),
    ("onebit", "enc1024_dec2048", {}),
    ("onebit", "enc4096_dec2048", {"BAGUA_TUNE_OB_ENCODE_BLOCKS": "4096"}),
    ("onebit", "enc16384_dec2048", {"BAGUA_TUNE_OB_ENCODE_BLOCKS": "16384"}),
    ("onebit", "enc1024_dec8192", {"BAGUA_TUNE_OB_DECODE_BLOCKS": "8192"}),
    ("onebit", "enc1024_dec16384", {"BAGUA_TUNE_OB_DECODE_BLOCKS": "16384"}),
]
KNOBS = ("BAGUA_RESIDENT", "BAGUA_TUNE_DEQUANT_BLOCKS", "BAGUA_TUNE_QUANT_BLOCKS", "BAGUA_TUNE_OB_ENCODE_BLOCKS",
         "BAGUA_TUNE_OB_DECODE_BLOCKS")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--elements", type=int, default=1 << 26)
    ap.add_argument("--only", default="", help="comma list of workloads")
    a = ap.parse_args()
    n = a.elements
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    g = torch.Generator(device=dev).manual_seed(0x5EED)
    x = torch.randn(n, device=dev, generator=g) * 1e-3
    y = torch.empty_like(x)
    Sm, Wm = K.bagua_minmax_u8_compressed_bytes(0, n, 1), K.bagua_minmax_u8_workspace_bytes(n, 1)
    So, Wo = K.bagua_onebit_compressed_bytes(n, 1), K.bagua_onebit_workspace_bytes(n, 1)
    comp = torch.empty(max(Sm, So), dtype=torch.uint8, device=dev)
    ws = torch.empty(max(Wm, Wo), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    xp, yp, cp, wp = x.data_ptr(), y.data_ptr(), comp.data_ptr(), ws.data_ptr()
    calls = {
        "minmax": [lambda: K.bagua_minmax_u8_compress(0, xp, n, n, 1, cp, Sm, wp, Wm, -1, sp),
                   lambda: K.bagua_minmax_u8_decompress(0, cp, Sm, n, 1, yp, sp)],
        "twopass": [lambda: K.bagua_minmax_u8_compress_stage(1, 0, xp, n, n, 1, cp, Sm, wp, Wm, -1, sp),
                    lambda: K.bagua_minmax_u8_compress_stage(2, 0, xp, n, n, 1, cp, Sm, wp, Wm, -1, sp),
                    lambda: K.bagua_minmax_u8_decompress(0, cp, Sm, n, 1, yp, sp)],
        "onebit": [lambda: K.bagua_onebit_compress(0, xp, n, n, 1, cp, So, wp, Wo, -1, sp),
                   lambda: K.bagua_onebit_decompress(0, cp, So, n, 1, yp, sp)],
    }
    names = {"minmax": ["encode", "decode"], "twopass": ["partials", "quantize", "decode"],
             "onebit": ["encode", "decode"]}
    sizes = {"minmax": Sm, "twopass": Sm, "onebit": So}
    only = set(a.only.split(",")) if a.only else None
    variants = [v for v in VARIANTS if not only or v[0] in only]

    def setenv(env):
        for k in KNOBS:
            os.environ.pop(k, None)
        os.environ.update(env)

    ref = {}
    for wl, label, env in variants:  # identical bytes within each workload
        setenv(env)
        for c in calls[wl]:
            N.check(c(), label)
        torch.cuda.synchronize()
        got = (comp[:sizes[wl]].cpu(), y.cpu())
        key = "onebit" if wl == "onebit" else "minmax"
        if key not in ref:
            ref[key] = got
        assert torch.equal(got[0], ref[key][0]) and torch.equal(got[1], ref[key][1]), f"{label}: output differs"

    res = {label: {"k": [], "step": []} for _, label, _ in variants}
    for r in range(a.rounds):
        order = variants if r % 2 == 0 else variants[::-1]
        for wl, label, env in order:
            setenv(env)
            cl = calls[wl]
            ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in cl]
                  for _ in range(a.steps)]
            for row in ev:
                for e0, e1 in row:
                    e0.record(st)
                    e1.record(st)
            for _ in range(5):
                for c in cl:
                    c()
            w0, w1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            w0.record(st)
            for _ in range(a.steps):
                for c in cl:
                    c()
            w1.record(st)
            for k in range(a.steps):
                for i, c in enumerate(cl):
                    K.bagua_time_next_kernel(ev[k][i][0].cuda_event, ev[k][i][1].cuda_event)
                    c()
            torch.cuda.synchronize()
            per = [float(np.mean([ev[k][i][0].elapsed_time(ev[k][i][1]) * 1e3 for k in range(a.steps)]))
                   for i in range(len(cl))]
            step = w0.elapsed_time(w1) * 1e3 / a.steps
            res[label]["k"].append(per)
            res[label]["step"].append(step)
            print(json.dumps({"round": r, "workload": wl, "variant": label, "step_us": round(step, 2),
                              "kernel_us": {nm: round(v, 2) for nm, v in zip(names[wl], per)}}), flush=True)
    for wl, label, env in variants:
        per = np.mean(np.array(res[label]["k"]), axis=0)
        step = float(np.mean(res[label]["step"]))
        print(json.dumps({"summary": True, "workload": wl, "variant": label, "env": env, "step_us": round(step, 2),
                          "gib_s": round(4.0 * n / (step * 1e-6) / (1 << 30), 1),
                          "kernel_us": {nm: round(float(v), 2) for nm, v in zip(names[wl], per)},
                          "identical_outputs": True}), flush=True)
    setenv({})


if __name__ == "__main__":
    main()
