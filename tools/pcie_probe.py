"""PCIe probe for the host-resident path: how fast can the 256 MiB
bucket go in (pinned H2D) and out (D2H) concurrently, and does splitting each
copy into chunks on several streams (more copy engines) help?  Prints JSON lines."""
import json
import time

import torch


def run(n_bytes: int, chunks: int, streams_per_dir: int, steps: int = 6) -> dict:
    dev = torch.device("cuda", 0)
    h_src = torch.empty(n_bytes, dtype=torch.uint8).pin_memory()
    h_dst = torch.empty(n_bytes, dtype=torch.uint8).pin_memory()
    d_in = torch.empty(n_bytes, dtype=torch.uint8, device=dev)
    d_out = torch.empty(n_bytes, dtype=torch.uint8, device=dev)
    s_in = [torch.cuda.Stream() for _ in range(streams_per_dir)]
    s_out = [torch.cuda.Stream() for _ in range(streams_per_dir)]
    step = n_bytes // chunks

    def go(h2d: bool, d2h: bool):
        for c in range(chunks):
            lo, hi = c * step, (c + 1) * step if c < chunks - 1 else n_bytes
            if h2d:
                with torch.cuda.stream(s_in[c % streams_per_dir]):
                    d_in[lo:hi].copy_(h_src[lo:hi], non_blocking=True)
            if d2h:
                with torch.cuda.stream(s_out[c % streams_per_dir]):
                    h_dst[lo:hi].copy_(d_out[lo:hi], non_blocking=True)

    res = {"bytes": n_bytes, "chunks": chunks, "streams_per_dir": streams_per_dir}
    for name, h2d, d2h in (("h2d", True, False), ("d2h", False, True), ("both", True, True)):
        go(h2d, d2h)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            go(h2d, d2h)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        res[name + "_ms"] = round(dt * 1e3, 3)
        res[name + "_gib_s_per_dir"] = round(n_bytes / dt / 2 ** 30, 2)
    return res


if __name__ == "__main__":
    import sys
    combos = ((1, 1), (2, 1), (4, 1), (8, 1), (16, 1), (32, 1), (4, 2), (4, 4), (16, 8))
    if len(sys.argv) > 1:
        combos = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]]
    for chunks, spd in combos:
        print(json.dumps(run(256 << 20, chunks, spd)), flush=True)
