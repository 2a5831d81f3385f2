"""BaguaBucketPy and the comm ops on the compressed-gradient path.

Mirrors `BaguaBucketPy` (bagua-core-py/src/lib.rs:352-487) / `BaguaBucket`
(bagua-core-internal/src/datatypes/mod.rs:1072-1267).  Each appended op is a
thin record; executing it calls ONE C-ABI entry point of libbagua_core.so
that runs the whole op (codec kernels + RCCL collectives) on the
communicator's stream:

  CentralizedLowPrecisionSynchronous   -> bagua_centralized_low_precision_synchronous
  CentralizedFullPrecisionSynchronous  -> bagua_centralized_full_precision_synchronous
  DecentralizedLowPrecisionSynchronous -> bagua_decentralized_low_precision_synchronous

The bucket's communication tensor follows get_communication_tensor
(datatypes/mod.rs:963-1070): if the tensors are laid out back to back in
memory the op runs in place on that span, otherwise they are copied into a
flat buffer on the communicator stream and copied back afterwards.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Callable, Optional

import torch

from . import _native as N
from .communicator import BaguaSingleCommunicatorPy
from .tensor import BaguaTensorPy, compression_code


@dataclass
class CentralizedLowPrecisionSynchronous:
    communicator: BaguaSingleCommunicatorPy
    average: bool
    compression: str
    fused: bool = True

    def execute(self, t: N.bagua_tensor_t) -> None:
        fn = (N.C.bagua_centralized_low_precision_synchronous if self.fused
              else N.C.bagua_centralized_low_precision_synchronous_unfused)
        N.check(fn(self.communicator.handle, ctypes.byref(t), int(self.average), compression_code(self.compression)),
                "centralized low precision synchronous op")


@dataclass
class CentralizedFullPrecisionSynchronous:
    communicator: BaguaSingleCommunicatorPy
    average: bool

    def execute(self, t: N.bagua_tensor_t) -> None:
        N.check(N.C.bagua_centralized_full_precision_synchronous(self.communicator.handle, ctypes.byref(t),
                                                                 int(self.average)),
                "centralized full precision synchronous op")


@dataclass
class DecentralizedLowPrecisionSynchronous:
    communicator: BaguaSingleCommunicatorPy
    compression: str
    weight: BaguaTensorPy
    left_peer_weight: BaguaTensorPy
    right_peer_weight: BaguaTensorPy

    def execute(self, t: N.bagua_tensor_t) -> None:
        w, l, r = self.weight.raw(), self.left_peer_weight.raw(), self.right_peer_weight.raw()
        N.check(N.C.bagua_decentralized_low_precision_synchronous(
            self.communicator.handle, ctypes.byref(t), ctypes.byref(w), ctypes.byref(l), ctypes.byref(r),
            compression_code(self.compression)), "decentralized low precision synchronous op")


@dataclass
class PythonOp:
    op: Callable

    def execute(self, t: N.bagua_tensor_t) -> None:  # python_ffi_op.rs: call with the bucket name
        self.op()


class BaguaBucketPy:
    def __init__(self, name: str, tensors: list):
        if not tensors:
            raise RuntimeError("BucketError: bucket is empty")
        first = tensors[0].raw()
        for t in tensors:
            r = t.raw()
            if r.dtype != first.dtype:
                raise RuntimeError("BucketError: tensors in the same bucket should be of the same dtype")
            if r.device_id != first.device_id:
                raise RuntimeError("BucketError: tensors in the same bucket should be of the same device")
            if r.num_elem_allocated < r.num_elem:
                raise RuntimeError("TensorError: num_elem_allocated should always be greater than num_elem")
        self.name = name
        self._tensors = list(tensors)
        self._ops: list = []
        self._ready: dict[str, bool] = {}  # by tensor name (unique per register_ordered_buckets)

    # ---- bookkeeping (lib.rs:371-486) ------------------------------------------
    def tensors(self) -> list:
        return list(self._tensors)

    def clear_ops(self) -> None:
        self._ops.clear()

    def print_ops(self) -> None:
        print(self._ops)

    def ops(self) -> list:
        return list(self._ops)

    def append_python_op(self, op: Callable) -> None:
        assert callable(op), "python op should be a callable"
        self._ops.append(PythonOp(op))

    def append_centralized_synchronous_op(self, communicator_internode: Optional[BaguaSingleCommunicatorPy],
                                          communicator_intranode: Optional[BaguaSingleCommunicatorPy] = None,
                                          hierarchical: bool = False, average: bool = True,
                                          scattergather: bool = False, compression: Optional[str] = None) -> None:
        comm = self._single(communicator_internode, communicator_intranode, hierarchical)
        if compression is None:
            if scattergather:
                raise NotImplementedError("scattergather full-precision op is outside the compressed-gradient path")
            self._ops.append(CentralizedFullPrecisionSynchronous(comm, average))
        else:
            compression_code(compression)
            self._ops.append(CentralizedLowPrecisionSynchronous(comm, average, compression))

    def append_low_precision_decentralized_synchronous_op(
            self, communicator_internode: Optional[BaguaSingleCommunicatorPy],
            communicator_intranode: Optional[BaguaSingleCommunicatorPy], hierarchical: bool = False,
            peer_selection_mode: str = "ring", compression: str = "MinMaxUInt8", weight: BaguaTensorPy = None,
            left_peer_weight: BaguaTensorPy = None, right_peer_weight: BaguaTensorPy = None) -> None:
        comm = self._single(communicator_internode, communicator_intranode, hierarchical)
        if peer_selection_mode != "ring":
            # datatypes/mod.rs:1170-1174
            raise NotImplementedError("unsupported peer_selection_mode for low precision decentralized algorithm "
                                      "(should be `ring`)")
        compression_code(compression)
        self._ops.append(DecentralizedLowPrecisionSynchronous(comm, compression, weight, left_peer_weight,
                                                              right_peer_weight))

    @staticmethod
    def _single(internode, intranode, hierarchical):
        if hierarchical:
            raise NotImplementedError("hierarchical communicators are outside the compressed-gradient path")
        if internode is None:
            raise RuntimeError("cannot create communicator: communicator_internode is None")
        return internode

    # ---- readiness (datatypes/mod.rs:1256-1266, 793-813) -------------------------
    def mark_tensor_ready(self, tensor: BaguaTensorPy) -> None:
        # keyed by name, as the reference keeps readiness on the shared tensor
        # (datatypes/mod.rs:793-813): any wrapper of a registered tensor counts
        self._ready[tensor.name()] = True

    def ready_for_comm(self) -> bool:
        return all(self._ready.get(t.name(), False) or t.name().startswith("bagua_padding_tensor")
                   for t in self._tensors)

    def reset_comm_ready(self) -> None:
        self._ready.clear()

    # ---- execution ---------------------------------------------------------------
    def _contiguous(self) -> bool:
        esz = N.C.bagua_dtype_bytes(self._tensors[0].raw().dtype)
        cur = None
        for t in self._tensors:
            r = t.raw()
            if cur is not None and r.ptr != cur:
                return False
            cur = r.ptr + r.num_elem_allocated * esz
        return True

    def execute_ops(self, stream_ptr: Optional[int] = None) -> None:
        """Run every op on the bucket's communication tensor (the comm worker
        loop body, bagua-core-internal/src/lib.rs:231-246).  Synchronous: the
        ops wait for their stream before returning (datatypes/mod.rs:1062-1066)."""
        if not self._ops:
            return
        raws = [t.raw() for t in self._tensors]
        dtype, device = raws[0].dtype, raws[0].device_id
        total = sum(r.num_elem_allocated for r in raws)
        if self._contiguous():
            flat = N.bagua_tensor_t(raws[0].ptr, total, total, dtype, device)
            for op in self._ops:
                op.execute(flat)
            return
        # non-contiguous: flatten on the communicator stream, run, copy back
        stream_ptr = stream_ptr if stream_ptr is not None else _op_stream(self._ops[0])
        stream = torch.cuda.ExternalStream(stream_ptr, device=torch.device("cuda", device)) if stream_ptr \
            else torch.cuda.default_stream(device)
        torch_ts = [t.torch_tensor() for t in self._tensors]
        with torch.cuda.stream(stream):
            buf = torch.cat([x.reshape(-1) for x in torch_ts])
        flat = N.bagua_tensor_t(buf.data_ptr(), total, total, dtype, device)
        for op in self._ops:
            op.execute(flat)
        with torch.cuda.stream(stream):
            off = 0
            for x in torch_ts:
                n = x.numel()
                x.view(-1).copy_(buf[off:off + n])
                off += n
        stream.synchronize()


def _op_stream(op) -> int:
    comm = getattr(op, "communicator", None)
    return comm.stream_ptr() if comm is not None else 0
