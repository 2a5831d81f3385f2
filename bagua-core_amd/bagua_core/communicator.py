"""BaguaSingleCommunicatorPy — RCCL communicator (bagua-core-py/src/lib.rs:14-194).

Creation follows the reference exactly: rank 0 calls the static
`generate_nccl_unique_id_str()` (base64 of the ncclUniqueId), the caller
distributes the string (upstream Bagua uses its own store; here any channel,
e.g. torch.distributed over gloo), and every rank constructs
`BaguaSingleCommunicatorPy(rank, nranks, device_id, stream_ptr, id)`.
Collectives are enqueued asynchronously on `stream_ptr`, as in the reference.
"""
from __future__ import annotations

import ctypes

from . import _native as N
from .tensor import BaguaTensorPy


class BaguaSingleCommunicatorPy:
    def __init__(self, rank: int, nranks: int, device_id: int, stream_ptr: int, nccl_unique_id_str: str):
        self._rank, self._nranks, self._device_id = int(rank), int(nranks), int(device_id)
        self._stream_ptr = int(stream_ptr)
        handle = N.C.bagua_single_communicator_c_create(self._rank, self._nranks, self._device_id, self._stream_ptr,
                                                        nccl_unique_id_str.encode())
        if not handle:
            raise RuntimeError(f"cannot create RCCL communicator (rank {rank}/{nranks}, device {device_id})")
        self._handle = ctypes.c_void_p(handle)

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            N.C.bagua_single_communicator_c_destroy(ctypes.byref(h))

    @classmethod
    def _from_handle(cls, handle: int, rank: int, nranks: int, device_id: int, stream_ptr: int, keep=()):
        obj = cls.__new__(cls)
        obj._rank, obj._nranks, obj._device_id, obj._stream_ptr = rank, nranks, device_id, stream_ptr
        obj._handle = ctypes.c_void_p(handle)
        obj._keep = keep
        return obj

    @staticmethod
    def generate_nccl_unique_id_str() -> str:
        buf = ctypes.create_string_buffer(512)
        N.check(N.C.bagua_generate_nccl_unique_id_str(buf, len(buf)), "ncclGetUniqueId")
        return buf.value.decode()

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._handle

    def nranks(self) -> int:
        n = ctypes.c_size_t()
        N.C.bagua_single_communicator_c_nranks(ctypes.byref(self._handle), ctypes.byref(n))
        return n.value

    def rank(self) -> int:
        return self._rank

    def device_id(self) -> int:
        return self._device_id

    def stream_ptr(self) -> int:
        return self._stream_ptr

    def abort(self) -> None:
        N.C.bagua_comm_abort(self._handle)

    def check_abort(self) -> bool:
        return bool(N.C.bagua_comm_check_abort(self._handle))

    def schedule_config(self) -> dict:
        """the schedule switches fixed at creation, equal on every rank (bagua_core.h)"""
        out = (ctypes.c_int32 * 5)()
        N.check(N.C.bagua_comm_schedule_config(self._handle, out, 5), "schedule_config")
        return dict(zip(("pieces_cap", "min_piece", "taper", "multipath", "check"), out))

    # ---- collectives (communicators/mod.rs:473-1043) --------------------------
    def _call(self, fn, what, *tensors, extra=()):
        raws = [t.raw() for t in tensors]
        N.check(fn(self._handle, *[ctypes.byref(r) for r in raws], *extra), what)

    def allreduce(self, send_tensor: BaguaTensorPy, recv_tensor: BaguaTensorPy, op: int) -> None:
        self._call(N.C.bagua_comm_allreduce, "allreduce", send_tensor, recv_tensor, extra=(op,))

    def allreduce_inplace(self, tensor: BaguaTensorPy, op: int) -> None:
        self._call(N.C.bagua_comm_allreduce_inplace, "allreduce_inplace", tensor, extra=(op,))

    def broadcast(self, tensor: BaguaTensorPy, root_rank: int) -> None:
        self._call(N.C.bagua_comm_broadcast, "broadcast", tensor, extra=(root_rank,))

    def reduce(self, send_tensor: BaguaTensorPy, recv_tensor: BaguaTensorPy, dst: int, op: int) -> None:
        self._call(N.C.bagua_comm_reduce, "reduce", send_tensor, recv_tensor, extra=(dst, op))

    def reduce_inplace(self, tensor: BaguaTensorPy, dst: int, op: int) -> None:
        self._call(N.C.bagua_comm_reduce_inplace, "reduce", tensor, extra=(dst, op))

    def send(self, tensor: BaguaTensorPy, peer_rank: int) -> None:
        self._call(N.C.bagua_comm_send, "send", tensor, extra=(peer_rank,))

    def recv(self, tensor: BaguaTensorPy, peer_rank: int) -> None:
        self._call(N.C.bagua_comm_recv, "recv", tensor, extra=(peer_rank,))

    def alltoall(self, send_tensor: BaguaTensorPy, recv_tensor: BaguaTensorPy) -> None:
        self._call(N.C.bagua_comm_alltoall, "alltoall", send_tensor, recv_tensor)

    def alltoall_inplace(self, tensor: BaguaTensorPy) -> None:
        self._call(N.C.bagua_comm_alltoall_inplace, "alltoall_inplace", tensor)

    def allgather(self, send_tensor: BaguaTensorPy, recv_tensor: BaguaTensorPy) -> None:
        self._call(N.C.bagua_comm_allgather, "allgather", send_tensor, recv_tensor)

    def allgather_inplace(self, tensor: BaguaTensorPy) -> None:
        self._call(N.C.bagua_comm_allgather_inplace, "allgather_inplace", tensor)

    def barrier(self) -> None:
        N.check(N.C.bagua_comm_barrier(self._handle), "barrier")

    # bagua-core-py/src/lib.rs:117-135,145-185: collective wrappers that no compressed op uses
    # (outside the compressed-gradient path) -- named, so a caller gets a clear
    # error instead of an AttributeError
    def _outside(self, name: str):
        raise NotImplementedError(f"{name} carries no compression and is outside the compressed-gradient path "
                                  "this library replaces (DESIGN.md §1)")

    def alltoall_v(self, send_tensor, send_counts, send_displs, recv_tensor, recv_counts, recv_displs) -> None:
        self._outside("alltoall_v")

    def gather(self, send_tensor, recv_tensor, dst: int) -> None:
        self._outside("gather")

    def gather_inplace(self, tensor, count: int, dst: int) -> None:
        self._outside("gather_inplace")

    def scatter(self, send_tensor, recv_tensor, src: int) -> None:
        self._outside("scatter")

    def scatter_inplace(self, tensor, count: int, src: int) -> None:
        self._outside("scatter_inplace")

    def reduce_scatter(self, send_tensor, recv_tensor, op: int) -> None:
        self._outside("reduce_scatter")

    def reduce_scatter_inplace(self, tensor, op: int) -> None:
        self._outside("reduce_scatter_inplace")

    def synchronize(self) -> None:
        N.check(N.C.bagua_comm_synchronize(self._handle), "stream synchronize")


class _LoopbackGroup:
    def __init__(self, nranks: int, device_id: int):
        self.handle = N.C.bagua_loopback_group_create(nranks, device_id)
        if not self.handle:
            raise RuntimeError("cannot create loopback group")

    def __del__(self):
        if getattr(self, "handle", None):
            N.C.bagua_loopback_group_destroy(self.handle)
            self.handle = None


def loopback_communicators(nranks: int, device_id: int = 0) -> list:
    """`nranks` communicators of an in-process loopback group on one device
    (test harness: drive each from its own thread; see bagua_core.h)."""
    import torch
    group = _LoopbackGroup(nranks, device_id)
    comms = []
    for r in range(nranks):
        stream = torch.cuda.Stream(device=device_id)
        h = N.C.bagua_loopback_communicator_create(group.handle, r, stream.cuda_stream)
        if not h:
            raise RuntimeError("cannot create loopback communicator")
        comms.append(BaguaSingleCommunicatorPy._from_handle(h, r, nranks, device_id, stream.cuda_stream,
                                                            keep=(group, stream)))
    return comms
