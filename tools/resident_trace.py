"""Phase timing of the one-launch MinMax encode (minmax_resident.hip) per
kernel configuration, from the kernel's own wall_clock64 stamps
(bagua_minmax_u8_resident_trace): pass 1, exchange, pass 2, per workgroup.

  python tools/resident_trace.py [--elements N] [--cfgs 0,1,2]

Prints one JSON line per configuration (medians over workgroups and runs, us).
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elements", type=int, default=1 << 26)
    ap.add_argument("--cfgs", default="0,1,2,3,4,5")
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--decode", action="store_true", help="run the decode between encodes (bench step)")
    ap.add_argument("--dump", default="", help="also save the raw stamps (runs x workgroups x 8, us) to this .npy")
    a = ap.parse_args()
    n = a.elements
    dev = torch.device("cuda", 0)
    x = torch.randn(n, device=dev) * 1e-3
    y = torch.empty_like(x)
    S = K.bagua_minmax_u8_compressed_bytes(0, n, 1)
    comp = torch.empty(S, dtype=torch.uint8, device=dev)
    wsb = K.bagua_minmax_u8_workspace_bytes(n, 1)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    tr = torch.zeros(8 * cus, dtype=torch.int64, device=dev)
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    khz = 100000  # wall_clock64: 100 MHz on MI300-class parts (hipDeviceAttributeWallClockRate)
    for cfg in [int(c) for c in a.cfgs.split(",")]:
        os.environ["BAGUA_RESIDENT_CFG"] = str(cfg)
        assert K.bagua_minmax_u8_resident_path(0, x.data_ptr(), n, n, 1, comp.data_ptr(), S, -1, sp) == 1
        rows = []
        for r in range(a.runs + 2):
            K.bagua_minmax_u8_resident_trace(tr.data_ptr() if r >= 2 else None)
            N.check(K.bagua_minmax_u8_compress(0, x.data_ptr(), n, n, 1, comp.data_ptr(), S, ws.data_ptr(), wsb, -1,
                                               sp), "compress")
            K.bagua_minmax_u8_resident_trace(None)
            if a.decode:
                N.check(K.bagua_minmax_u8_decompress(0, comp.data_ptr(), S, n, 1, y.data_ptr(), sp), "decompress")
            if r >= 2:
                torch.cuda.synchronize()
                t = tr.cpu().numpy().reshape(cus, 8).astype(np.float64) * (1e3 / khz)  # us
                t -= t[:, 0].min()
                rows.append(t)
        t = np.stack(rows)  # runs x wg x 8
        if a.dump:
            np.save(a.dump.replace(".npy", f"_cfg{cfg}.npy"), t)
        out = {
            "cfg": cfg,
            "start_spread_us": float(np.median(t[:, :, 0].max(axis=1))),
            "pass1_us_median_wg": float(np.median(t[:, :, 1] - t[:, :, 0])),
            "pass1_end_max_us": float(np.median(t[:, :, 1].max(axis=1))),
            "exchange_us_median_wg": float(np.median(t[:, :, 2] - t[:, :, 1])),
            "exchange_end_max_us": float(np.median(t[:, :, 2].max(axis=1))),
            "pass2_us_median_wg": float(np.median(t[:, :, 3] - t[:, :, 2])),
            "pass2_stream_us": float(np.median(t[:, :, 4] - t[:, :, 2])),
            "pass2_lds_us": float(np.median(t[:, :, 5] - t[:, :, 4])),
            "pass2_regs_us": float(np.median(t[:, :, 3] - t[:, :, 5])),
            "end_max_us": float(np.median(t[:, :, 3].max(axis=1))),
        }
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
