"""One rank of the pipelined compressed all-reduce, for kernel traces of how
its streams map onto hardware queues (GPU_MAX_HW_QUEUES).

Every rank is its own process on the box's one GPU, with its own NCCL_HOSTID,
so RCCL links the ranks through its socket transport (as in
tests/test_gpu_rccl_procs.py): the RCCL kernels then run for as long as the
socket transfer takes, which makes it obvious in a trace whether the codec
kernels on the op's stream run BESIDE them (separate hardware queues) or only
after them (one queue, in order).  Start each rank under its own profiler:

  for r in 0 1; do GPU_MAX_HW_QUEUES=4 rocprofv3 --kernel-trace --output-format csv \
      -d gpurun_out/q4/rank$r -o run -- python3 tools/queue_probe.py $r 2 /tmp/qp & done; wait
  python3 tools/queue_overlap.py gpurun_out/q4

Prints one JSON line per rank (the op's ms per step, the queue setting).
"""
import ctypes
import json
import os
import sys
import time

rank, world, workdir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
n = int(sys.argv[4]) if len(sys.argv) > 4 else 1 << 24
steps = int(sys.argv[5]) if len(sys.argv) > 5 else 6
os.environ["NCCL_HOSTID"] = f"bagua-queue-probe-{rank}"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
os.environ.setdefault("NCCL_IB_DISABLE", "1")

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "bagua-core_amd"))

import torch  # noqa: E402

import bagua_core as bc  # noqa: E402
from bagua_core import _native as N  # noqa: E402


def uid() -> str:
    os.makedirs(workdir, exist_ok=True)
    path = os.path.join(workdir, "uid.txt")
    if rank == 0:
        with open(path + ".tmp", "w") as f:
            f.write(bc.BaguaSingleCommunicatorPy.generate_nccl_unique_id_str())
        os.replace(path + ".tmp", path)
    deadline = time.time() + 120
    while not os.path.exists(path):
        if time.time() > deadline:
            raise TimeoutError("no unique id")
        time.sleep(0.02)
    with open(path) as f:
        return f.read().strip()


def main():
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    comm = bc.BaguaSingleCommunicatorPy(rank, world, 0, stream.cuda_stream, uid())
    g = torch.Generator(device="cuda").manual_seed(0x5EED + rank)
    x = torch.randn(n, device="cuda", generator=g) * 1e-3
    torch.cuda.synchronize()
    raw = bc.BaguaTensorPy(x, "bucket").raw()

    def step(pieces):
        N.check(N.C.bagua_centralized_low_precision_pipelined(comm.handle, ctypes.byref(raw), 1,
                                                              N.COMPRESSION_MINMAX_UINT8, pieces), "op")
        comm.synchronize()

    step(4)
    t0 = time.perf_counter()
    for _ in range(steps):
        step(4)
    dt = (time.perf_counter() - t0) / steps
    print(json.dumps({"rank": rank, "world": world, "elements": n, "pieces": 4, "ms_per_step": round(dt * 1e3, 2),
                      "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}), flush=True)
    comm.barrier() if hasattr(comm, "barrier") else None
    if rank == 0:
        try:
            os.remove(os.path.join(workdir, "uid.txt"))
        except OSError:
            pass


if __name__ == "__main__":
    main()
