"""Worker of tests/test_gpu_rccl_procs.py: one rank of a REAL multi-process RCCL
communicator, all ranks sharing the box's one MI355X.

RCCL refuses two ranks of one communicator on the same GPU of the same host
("Duplicate GPU detected", keyed by host hash + PCI bus id).  Each worker sets
its own NCCL_HOSTID, so every rank is a host of its own to RCCL and the ranks
talk through RCCL's socket transport over the loopback interface.  That is not
the xGMI path (no speed claim is made), but it is RCCL itself matching the
grouped send/recv, alltoall and allgather calls the ops post, across separate
processes — the multi-rank semantics the loopback transport only emulates.

usage: python rccl_worker.py <scenario> <rank> <world> <workdir> [key=value ...]
Inputs come from <workdir>/inputs.npz, results go to <workdir>/out<rank>.npz.
"""
from __future__ import annotations

import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bagua-core_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

F32, F16, BF16 = 0, 1, 2
TORCH = {F32: torch.float32, F16: torch.float16, BF16: torch.bfloat16}


def _uid(workdir: str, name: str, creator: bool, bc) -> str:
    """rank `creator` publishes a fresh ncclUniqueId under `name`; the others wait for it"""
    path = os.path.join(workdir, f"uid_{name}.txt")
    if creator:
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write(bc.BaguaSingleCommunicatorPy.generate_nccl_unique_id_str())
        os.replace(tmp, path)
    deadline = time.time() + 60
    while not os.path.exists(path):
        if time.time() > deadline:
            raise TimeoutError(f"no unique id {name}")
        time.sleep(0.02)
    with open(path) as f:
        return f.read().strip()


def _dev(x: np.ndarray, dtype: int) -> torch.Tensor:
    if dtype == BF16:
        return torch.from_numpy(x.view(np.int16).copy()).view(torch.bfloat16).cuda()
    return torch.from_numpy(x.copy()).cuda()


def _host(t: torch.Tensor) -> np.ndarray:
    torch.cuda.synchronize()
    return t.contiguous().view(torch.uint8).cpu().numpy()


def main() -> None:
    scenario, rank, world, workdir = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    kw = dict(a.split("=", 1) for a in sys.argv[5:])
    import bagua_core as bc
    N = bc._native
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    with np.load(os.path.join(workdir, "inputs.npz"), allow_pickle=False) as z:
        inputs = {k: z[k] for k in z.files}
    dtype = int(kw.get("dtype", F32))
    out = {}

    def comm_of(name: str, r: int, n: int, creator: bool):
        return bc.BaguaSingleCommunicatorPy(r, n, 0, stream.cuda_stream, _uid(workdir, name, creator, bc))

    if scenario == "collectives":
        # the plain collectives (communicators/mod.rs:473-1043) on real ranks
        comm = comm_of("all", rank, world, rank == 0)
        x = torch.from_numpy(inputs[f"x{rank}"].copy()).cuda()
        a = x.clone()
        comm.allreduce_inplace(bc.BaguaTensorPy(a, "a"), 0)  # SUM
        g = x[: x.numel() // world * world].clone()
        comm.allgather_inplace(bc.BaguaTensorPy(g, "g"))
        t = x[: x.numel() // world * world].clone()
        comm.alltoall_inplace(bc.BaguaTensorPy(t, "t"))
        b = x.clone()
        comm.broadcast(bc.BaguaTensorPy(b, "b"), world - 1)
        rd = x.clone()
        comm.reduce_inplace(bc.BaguaTensorPy(rd, "rd"), 0, 0)
        comm.synchronize()
        out = {"allreduce": _host(a), "allgather": _host(g), "alltoall": _host(t), "broadcast": _host(b)}
        if rank == 0:
            out["reduce"] = _host(rd)
        comm.barrier()
    elif scenario == "centralized":
        comm = comm_of("all", rank, world, rank == 0)
        method = {"MinMaxUInt8": N.COMPRESSION_MINMAX_UINT8, "OneBit": N.COMPRESSION_ONEBIT}[kw["method"]]
        pieces = int(kw.get("pieces", 0))
        average = int(kw.get("average", 1))
        t = _dev(inputs[f"x{rank}"], dtype)
        raw = bc.BaguaTensorPy(t, "g").raw()
        for _ in range(int(kw.get("repeat", 1))):  # the op twice in a row on one communicator
            if pieces < 0:
                fn = N.C.bagua_centralized_low_precision_synchronous_unfused
                N.check(fn(comm.handle, ctypes.byref(raw), average, method), "unfused op")
            else:
                N.check(N.C.bagua_centralized_low_precision_pipelined(comm.handle, ctypes.byref(raw), average, method,
                                                                      pieces), "pipelined op")
            comm.synchronize()
            out[f"t{_}"] = _host(t)
            t.copy_(_dev(inputs[f"x{rank}"], dtype))
            torch.cuda.synchronize()  # the reset (current stream) lands before the next op (comm stream)
        comm.barrier()
    elif scenario == "decentralized":
        if "multipath" in kw:  # read when the communicator is created (rank 0's value wins)
            os.environ["BAGUA_RING_MULTIPATH"] = kw["multipath"]
        comm = comm_of("all", rank, world, rank == 0)
        ts = [_dev(inputs[f"{k}{rank}"], dtype) for k in "twlr"]
        raws = [bc.BaguaTensorPy(x, k).raw() for x, k in zip(ts, "twlr")]
        pieces = int(kw.get("pieces", 0))
        N.check(N.C.bagua_decentralized_low_precision_pipelined(comm.handle, *[ctypes.byref(r) for r in raws],
                                                                N.COMPRESSION_MINMAX_UINT8, pieces),
                "decentralized op")
        comm.synchronize()
        out = {k: _host(x) for k, x in zip("twlr", ts)}
        comm.barrier()
    elif scenario == "hierarchical":
        per_node = int(kw["per_node"])
        node, local = divmod(rank, per_node)
        intra = comm_of(f"node{node}", local, per_node, local == 0)
        inter = comm_of("leaders", node, world // per_node, rank == 0) if local == 0 else None
        t = _dev(inputs[f"x{rank}"], F32)
        raw = bc.BaguaTensorPy(t, "g").raw()
        N.check(N.C.bagua_centralized_low_precision_hierarchical(intra.handle, inter.handle if inter else None,
                                                                 ctypes.byref(raw), 1, N.COMPRESSION_MINMAX_UINT8),
                "hierarchical op")
        intra.synchronize()
        out = {"t": _host(t)}
        intra.barrier()
    elif scenario == "backend":
        # the native scheduler (BaguaCommBackendPy) over real ranks: buckets of two
        # tensors each, marked ready in reverse order as backward would
        comm = comm_of("all", rank, world, rank == 0)
        nb = int(kw.get("buckets", 3))
        flats = [_dev(inputs[f"b{b}_{rank}"], F32) for b in range(nb)]
        tensors, buckets = [], []
        for b, flat in enumerate(flats):
            ts = [bc.BaguaTensorPy(v, f"b{b}.t{i}") for i, v in enumerate(flat.view(2, -1).unbind(0))]
            bk = bc.BaguaBucketPy(f"bucket{b}", ts)
            bk.append_centralized_synchronous_op(comm, None, False, True, False, "MinMaxUInt8")
            tensors.append(ts)
            buckets.append(bk)
        backend = bc.BaguaCommBackendPy(nb, 0)
        lanes = int(kw.get("lanes", 0))
        if lanes:
            backend.set_lanes(lanes)
        backend.register_ordered_buckets(list(reversed(buckets)))
        # `steps` back-to-back steps, each bucket's output the next step's input (with
        # several lanes, consecutive buckets run on different streams of ONE RCCL
        # communicator: their collectives must still pair up in issue order on every rank)
        for step in range(int(kw.get("steps", 1))):
            # the ready events must outlive the scheduled executions that wait for them (the
            # scheduler keeps the raw handle, as the reference's BaguaTensor does)
            events = []
            for b in reversed(range(nb)):
                ev = torch.cuda.Event()
                ev.record()
                events.append(ev)
                for t in tensors[b]:
                    backend.mark_communication_ready(t, ev.cuda_event)
            done = backend.wait_pending_comm_ops()
            del events
            assert done == nb, done
        out = {f"b{b}": _host(f) for b, f in enumerate(flats)}
        out["lanes"] = np.array([backend.lanes()])
        comm.barrier()
        del backend
    elif scenario == "mismatch":
        # ranks posting different op schedules.  Rank 1's own environment tapers the pieces
        # and rank 0's does not: rank 0's value must win at creation (else the first op
        # below would post mismatched grouped send/recv and hang).  BAGUA_CHECK_SCHEDULE is
        # set on rank 0 only -- it must reach rank 1 the same way.  Then rank 0 asks for 4
        # pieces and rank 1 for 2: both must fail with invalid argument, tensors untouched,
        # and the communicator must still run a matching op afterwards.
        if rank == 0:
            os.environ["BAGUA_CHECK_SCHEDULE"] = "1"
        else:
            os.environ["BAGUA_PIPELINE_TAPER"] = "1"
        comm = comm_of("all", rank, world, rank == 0)
        t = _dev(inputs[f"x{rank}"], F32)
        raw = bc.BaguaTensorPy(t, "g").raw()
        op = N.C.bagua_centralized_low_precision_pipelined
        M = N.COMPRESSION_MINMAX_UINT8
        rc_same = op(comm.handle, ctypes.byref(raw), 1, M, 5)  # 5 pieces: tapered only on rank 1's env
        comm.synchronize()
        out["same"] = _host(t)
        t.copy_(_dev(inputs[f"x{rank}"], F32))
        torch.cuda.synchronize()
        rc_pieces = op(comm.handle, ctypes.byref(raw), 1, M, 4 if rank == 0 else 2)
        comm.synchronize()
        out["after_pieces"] = _host(t)
        rc_kind = (op(comm.handle, ctypes.byref(raw), 1, M, 3) if rank == 0 else
                   N.C.bagua_centralized_low_precision_synchronous_unfused(comm.handle, ctypes.byref(raw), 1, M))
        comm.synchronize()
        out["after_kind"] = _host(t)
        rc_again = op(comm.handle, ctypes.byref(raw), 1, M, 3)
        comm.synchronize()
        out["again"] = _host(t)
        out["rc"] = np.array([rc_same, rc_pieces, rc_kind, rc_again])
        out["cfg"] = np.array(list(comm.schedule_config().values()))
        comm.barrier()
    elif scenario == "stuck":
        # rank 1 never posts the op: rank 0's scheduler monitor must fail it after its
        # limit, abort the communicator and let wait_pending_comm_ops raise
        comm = comm_of("all", rank, world, rank == 0)
        flag = os.path.join(workdir, "rank0_done")
        if rank == 0:
            x = _dev(inputs["x0"], F32)
            bk = bc.BaguaBucketPy("stuck_bucket", [bc.BaguaTensorPy(x, "x")])
            bk.append_centralized_synchronous_op(comm, None, False, True, False, "MinMaxUInt8")
            backend = bc.BaguaCommBackendPy(1, 0)
            limit = float(kw.get("limit", 3))
            backend.set_op_timeout(limit)
            backend.register_ordered_buckets([bk])
            ev = torch.cuda.Event()
            ev.record()
            t0 = time.time()
            backend.mark_communication_ready(bk.tensors()[0], ev.cuda_event)
            msg = ""
            try:
                backend.wait_pending_comm_ops()
            except RuntimeError as e:
                msg = str(e)
            elapsed = time.time() - t0
            failures = backend.failures()
            del backend  # must not hang on the aborted op
            out = {"elapsed": np.array([elapsed]), "raised": np.array([bool(msg)]),
                   "failures": np.array([len(failures)]), "aborted": np.array([comm.check_abort()])}
            print(f"rank 0: wait_pending_comm_ops -> {msg!r} after {elapsed:.2f} s", flush=True)
            with open(flag, "w") as f:
                f.write("done")
        else:
            deadline = time.time() + 60
            while not os.path.exists(flag) and time.time() < deadline:
                time.sleep(0.05)
            comm.abort()
            out = {"peer": np.array([1])}
        np.savez(os.path.join(workdir, f"out{rank}.npz"), **out)
        print(f"rank {rank}/{world} {scenario} ok", flush=True)
        os._exit(0)  # the aborted communicator is not torn down any further
    else:
        raise SystemExit(f"unknown scenario {scenario}")
    np.savez(os.path.join(workdir, f"out{rank}.npz"), **out)
    print(f"rank {rank}/{world} {scenario} ok", flush=True)


if __name__ == "__main__":
    main()
