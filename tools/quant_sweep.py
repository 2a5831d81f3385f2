"""Workgroups of the MinMax quantise pass (minmax_quantize_kernel) where it runs
after another kernel's min/max partials: the config-5 ring op (bf16, partials
from ring_mix_kernel) and the two-pass f32 encode (partials from
minmax_partials_kernel).  BAGUA_TUNE_QUANT_BLOCKS per call; bytes must not change.

  python tools/quant_sweep.py [--rounds 4 --steps 20]
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
BLOCKS = (2048, 4096, 8192, 16384, 32768)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    g = torch.Generator(device=dev).manual_seed(3)
    cases = {}
    # config 5: bf16, 2^27 elements, partials from the mix pass
    nb = 1 << 27
    tw = {k: (torch.randn(nb, device=dev, generator=g) * 1e-3).to(torch.bfloat16) for k in "twlr"}
    Sb, Wb = K.bagua_minmax_u8_compressed_bytes(2, nb, 1), K.bagua_minmax_u8_workspace_bytes(nb, 1)
    cb, wsb = torch.empty(Sb, dtype=torch.uint8, device=dev), torch.empty(Wb, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    N.check(K.bagua_ring_mix_minmax(2, tw["t"].data_ptr(), tw["l"].data_ptr(), tw["r"].data_ptr(), tw["w"].data_ptr(),
                                    nb, wsb.data_ptr(), Wb, sp), "mix")
    cases["ring_bf16"] = (lambda: K.bagua_minmax_u8_compress_stage(2, 2, tw["t"].data_ptr(), nb, nb, 1, cb.data_ptr(),
                                                                    Sb, wsb.data_ptr(), Wb, -1, sp), cb, 3 * nb)
    # two-pass f32 encode, 2^26 elements
    nf = 1 << 26
    x = torch.randn(nf, device=dev, generator=g) * 1e-3
    Sf, Wf = K.bagua_minmax_u8_compressed_bytes(0, nf, 1), K.bagua_minmax_u8_workspace_bytes(nf, 1)
    cf, wsf = torch.empty(Sf, dtype=torch.uint8, device=dev), torch.empty(Wf, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    N.check(K.bagua_minmax_u8_compress_stage(1, 0, x.data_ptr(), nf, nf, 1, cf.data_ptr(), Sf, wsf.data_ptr(), Wf, -1,
                                             sp), "partials")
    cases["twopass_f32"] = (lambda: K.bagua_minmax_u8_compress_stage(2, 0, x.data_ptr(), nf, nf, 1, cf.data_ptr(), Sf,
                                                                      wsf.data_ptr(), Wf, -1, sp), cf, 5 * nf)
    ref = {}
    for name, (fn, out, _) in cases.items():
        for qb in BLOCKS:
            os.environ["BAGUA_TUNE_QUANT_BLOCKS"] = str(qb)
            N.check(fn(), name)
            torch.cuda.synchronize()
            h = out.cpu()
            if name not in ref:
                ref[name] = h
            assert torch.equal(h, ref[name]), f"{name} {qb}: bytes differ"
    res = {(n, qb): [] for n in cases for qb in BLOCKS}
    for r in range(a.rounds):
        order = BLOCKS if r % 2 == 0 else BLOCKS[::-1]
        for name, (fn, _, _) in cases.items():
            for qb in order:
                os.environ["BAGUA_TUNE_QUANT_BLOCKS"] = str(qb)
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(a.steps)]
                for e0, e1 in ev:
                    e0.record(st)
                    e1.record(st)
                for _ in range(3):
                    fn()
                for e0, e1 in ev:
                    K.bagua_time_next_kernel(e0.cuda_event, e1.cuda_event)
                    fn()
                torch.cuda.synchronize()
                res[(name, qb)].append(float(np.mean([e0.elapsed_time(e1) * 1e3 for e0, e1 in ev])))
    for name, (_, _, alg) in cases.items():
        for qb in BLOCKS:
            us = float(np.mean(res[(name, qb)]))
            print(json.dumps({"case": name, "quant_blocks": qb, "us": round(us, 2),
                              "tbs": round(alg / (us * 1e-6) / 1e12, 3), "identical_outputs": True}), flush=True)
    os.environ.pop("BAGUA_TUNE_QUANT_BLOCKS", None)


if __name__ == "__main__":
    main()
