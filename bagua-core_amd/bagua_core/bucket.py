"""BaguaBucketPy and the comm ops on the compressed-gradient path.

Mirrors `BaguaBucketPy` (bagua-core-py/src/lib.rs:352-487) / `BaguaBucket`
(bagua-core-internal/src/datatypes/mod.rs:1072-1267).  The bucket itself is
native (`BaguaBucketC`, csrc/runtime/backend.cpp): its tensors, readiness and
op list live in libbagua_core.so, and executing it (directly or from the
native scheduler's worker thread) runs every op through ONE C-ABI entry point
on the communicator's stream:

  CentralizedLowPrecisionSynchronous   -> bagua_centralized_low_precision_synchronous
  CentralizedFullPrecisionSynchronous  -> bagua_centralized_full_precision_synchronous
  DecentralizedLowPrecisionSynchronous -> bagua_decentralized_low_precision_synchronous
  PythonOp                             -> a ctypes callback (python_ffi_op.rs)

The communication tensor follows get_communication_tensor
(datatypes/mod.rs:963-1070): in place when the tensors are back to back in
memory, otherwise packed into a pool buffer on the stream and copied back.
The dataclasses below are the Python view of the ops (ops(), print_ops()).
"""
from __future__ import annotations

import ctypes
import weakref
from dataclasses import dataclass, field
from typing import Callable, Optional

from . import _native as N
from .communicator import BaguaSingleCommunicatorPy
from .tensor import _DTYPES, BaguaTensorPy, compression_code

CALLBACK = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_char_p)


def _handle(c: Optional[BaguaSingleCommunicatorPy]):
    return c.handle.value if c is not None else None


@dataclass
class CentralizedLowPrecisionSynchronous:
    communicator: Optional[BaguaSingleCommunicatorPy]  # internode (None on a hierarchical node worker)
    average: bool
    compression: str
    fused: bool = True
    intranode: Optional[BaguaSingleCommunicatorPy] = None  # hierarchical mode

    def native(self) -> N.bagua_bucket_op_t:
        return N.bagua_bucket_op_t(kind=N.BUCKET_OP_CENTRALIZED_LOW_PRECISION, average=int(self.average),
                                   compression=compression_code(self.compression), fused=int(self.fused),
                                   comm=_handle(self.communicator), intranode=_handle(self.intranode))


@dataclass
class CentralizedFullPrecisionSynchronous:
    communicator: Optional[BaguaSingleCommunicatorPy]
    average: bool
    intranode: Optional[BaguaSingleCommunicatorPy] = None

    def native(self) -> N.bagua_bucket_op_t:
        return N.bagua_bucket_op_t(kind=N.BUCKET_OP_CENTRALIZED_FULL_PRECISION, average=int(self.average),
                                   comm=_handle(self.communicator), intranode=_handle(self.intranode))


@dataclass
class DecentralizedLowPrecisionSynchronous:
    communicator: Optional[BaguaSingleCommunicatorPy]
    compression: str
    weight: BaguaTensorPy
    left_peer_weight: BaguaTensorPy
    right_peer_weight: BaguaTensorPy
    intranode: Optional[BaguaSingleCommunicatorPy] = None

    def native(self) -> N.bagua_bucket_op_t:
        return N.bagua_bucket_op_t(kind=N.BUCKET_OP_DECENTRALIZED_LOW_PRECISION,
                                   compression=compression_code(self.compression),
                                   comm=_handle(self.communicator), weight=self.weight.raw(),
                                   left_peer_weight=self.left_peer_weight.raw(),
                                   right_peer_weight=self.right_peer_weight.raw(), intranode=_handle(self.intranode))


@dataclass
class PythonOp:
    op: Callable
    _cb: object = field(default=None, repr=False)

    def native(self) -> N.bagua_bucket_op_t:
        if self._cb is None:
            def call(_user, bucket_name):  # python_ffi_op.rs: py_callable(bucket.name)
                self.op(bucket_name.decode())
            self._cb = CALLBACK(call)  # kept alive with the op
        return N.bagua_bucket_op_t(kind=N.BUCKET_OP_CALLBACK, callback=ctypes.cast(self._cb, ctypes.c_void_p).value)


_ERRORS = {N.STATUS_INVALID_ARG: "BucketError: tensors in the same bucket should be of the same dtype and device, "
                                 "and num_elem_allocated should always be greater than num_elem"}


class BaguaBucketPy:
    def __init__(self, name: str, tensors: list):
        if not tensors:
            raise RuntimeError("BucketError: bucket is empty")
        raws = [t.raw() for t in tensors]
        first = raws[0]
        for r in raws:
            if r.dtype != first.dtype:
                raise RuntimeError("BucketError: tensors in the same bucket should be of the same dtype")
            if r.device_id != first.device_id:
                raise RuntimeError("BucketError: tensors in the same bucket should be of the same device")
            if r.num_elem_allocated < r.num_elem:
                raise RuntimeError("TensorError: num_elem_allocated should always be greater than num_elem")
        arr = (N.bagua_tensor_t * len(raws))(*raws)
        names = (ctypes.c_char_p * len(raws))(*[t.name().encode() for t in tensors])
        st = ctypes.c_int(0)
        handle = N.C.bagua_bucket_create(name.encode(), arr, names, len(raws), ctypes.byref(st))
        if not handle:
            raise RuntimeError(_ERRORS.get(st.value, f"BucketError: {N.STATUS.get(st.value, st.value)}"))
        self._handle = ctypes.c_void_p(handle)
        self.name = name
        self._tensors = list(tensors)
        self._by_name = {t.name(): t for t in tensors}
        self._ops: list = []
        # ops removed by clear_ops while a scheduled execution of this bucket may still
        # hold their native copies (callback thunks, communicator handles): kept alive
        # until the scheduler has run everything it scheduled (the reference's Arc
        # clones, lib.rs:143-146) -- released by BaguaCommBackendPy.wait_pending_comm_ops.
        # Only a bucket registered with a scheduler can have such executions: execute_ops
        # has enqueued everything (and run every callback) by the time it returns.
        self._retired: list = []
        self._schedulers = weakref.WeakSet()  # BaguaCommBackendPy instances this bucket is registered with

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            N.C.bagua_bucket_destroy(h)
            self._handle = None

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._handle

    # ---- bookkeeping (lib.rs:371-486) ------------------------------------------
    def tensors(self) -> list:
        return list(self._tensors)

    def _append(self, op) -> None:
        N.check(N.C.bagua_bucket_append_op(self._handle, ctypes.byref(op.native())), "append op")
        self._ops.append(op)

    def clear_ops(self) -> None:
        N.check(N.C.bagua_bucket_clear_ops(self._handle), "clear ops")
        if any(b._holds(self) for b in list(self._schedulers)):
            self._retired.extend(self._ops)
        self._ops.clear()

    def _release_retired(self) -> None:
        """every scheduled execution has run: the cleared ops can go"""
        self._retired.clear()

    def print_ops(self) -> None:
        print(self._ops)

    def ops(self) -> list:
        return list(self._ops)

    def append_python_op(self, op: Callable) -> None:
        assert callable(op), "python op should be a callable"
        self._append(PythonOp(op))

    def append_centralized_synchronous_op(self, communicator_internode: Optional[BaguaSingleCommunicatorPy],
                                          communicator_intranode: Optional[BaguaSingleCommunicatorPy] = None,
                                          hierarchical: bool = False, average: bool = True,
                                          scattergather: bool = False, compression: Optional[str] = None) -> None:
        comm, intra = self._communicators(communicator_internode, communicator_intranode, hierarchical)
        if compression is None:
            if scattergather:
                raise NotImplementedError("scattergather full-precision op is outside the compressed-gradient path")
            self._append(CentralizedFullPrecisionSynchronous(comm, average, intranode=intra))
        else:
            compression_code(compression)
            self._append(CentralizedLowPrecisionSynchronous(comm, average, compression, intranode=intra))

    def append_low_precision_decentralized_synchronous_op(
            self, communicator_internode: Optional[BaguaSingleCommunicatorPy],
            communicator_intranode: Optional[BaguaSingleCommunicatorPy], hierarchical: bool = False,
            peer_selection_mode: str = "ring", compression: str = "MinMaxUInt8", weight: BaguaTensorPy = None,
            left_peer_weight: BaguaTensorPy = None, right_peer_weight: BaguaTensorPy = None) -> None:
        comm, intra = self._communicators(communicator_internode, communicator_intranode, hierarchical)
        if peer_selection_mode != "ring":
            # datatypes/mod.rs:1170-1174
            raise NotImplementedError("unsupported peer_selection_mode for low precision decentralized algorithm "
                                      "(should be `ring`)")
        compression_code(compression)
        self._append(DecentralizedLowPrecisionSynchronous(comm, compression, weight, left_peer_weight,
                                                          right_peer_weight, intranode=intra))

    # The full-precision decentralized ops (decentralized_full_precision_synchronous.rs,
    # decentralized_full_precision_asynchronous.rs) carry no compression: outside the
    # compressed-gradient path this package rebuilds.  Same signatures as
    # bagua-core-py/src/lib.rs:408-426 and :453-467, so callers get a clear error.
    def append_decentralized_synchronous_op(self, communicator_internode, communicator_intranode,
                                            hierarchical: bool = False, peer_selection_mode: str = "all",
                                            peer_weight: BaguaTensorPy = None) -> None:
        raise NotImplementedError("append_decentralized_synchronous_op (full-precision decentralized op) is outside "
                                  "the compressed-gradient path; use append_low_precision_decentralized_synchronous_op")

    def append_decentralized_asynchronous_op(self, communicator_internode, communicator_intranode,
                                             peer_selection_mode: str = "all", torch_stream: int = 0) -> None:
        raise NotImplementedError("append_decentralized_asynchronous_op (full-precision asynchronous model "
                                  "averaging) is outside the compressed-gradient path")

    @staticmethod
    def _communicators(internode, intranode, hierarchical):
        """BaguaCommunicator::new (communicators/mod.rs:348-383): (internode, None), or in
        hierarchical mode (internode on the node leader, None on its workers, intranode)."""
        if not hierarchical:
            if internode is None:
                raise RuntimeError("inter node communicator must be given in non-hierarchical mode")
            return internode, None
        if intranode is None:
            raise RuntimeError("intra node communicator must be given in hierarchical mode")
        if intranode.rank() != 0:
            return None, intranode  # a node worker: reduce + broadcast only
        if internode is None:
            raise RuntimeError("inter node communicator must be given on the node leader in hierarchical mode")
        if internode.stream_ptr() != intranode.stream_ptr():
            raise RuntimeError("intra node communicator should use the same stream as the inter node communicator")
        return internode, intranode

    # ---- readiness (datatypes/mod.rs:1256-1266, 793-813), by tensor name --------
    def mark_tensor_ready(self, tensor: BaguaTensorPy, ready_cuda_event_ptr: int = 0) -> None:
        # the tensor's CURRENT storage (data_ptr read at run time, datatypes/mod.rs:775-791)
        t = tensor._torch
        if t is not None:
            ptr = t.data_ptr()
            dev = tensor._mark_dev if ptr == tensor._mark_ptr else tensor._mark_device(ptr)
            spec = _DTYPES.get(t.dtype)
            rc = N.FAST.bucket_mark(self._handle.value, tensor._name_b, int(ready_cuda_event_ptr or 0), ptr,
                                    t.numel(), spec[0] if spec else -1, dev)
        else:
            rc = N.C.bagua_bucket_mark_tensor_ready_desc(self._handle, tensor._name_b, int(ready_cuda_event_ptr or 0),
                                                         ctypes.byref(tensor._raw))
        N.check(rc, f"tensor {tensor.name()} is not in bucket {self.name} (or changed dtype/device)")

    def _refresh(self) -> None:
        """re-read every tensor's storage (a .data / set_ swap after the bucket was built)"""
        for t in self._tensors:
            N.check(N.C.bagua_bucket_refresh_tensor(self._handle, t.name().encode(), ctypes.byref(t._current())),
                    f"tensor {t.name()} changed dtype or device")

    def ready_for_comm(self) -> bool:
        return bool(N.C.bagua_bucket_ready_for_comm(self._handle))

    def reset_comm_ready(self) -> None:
        N.check(N.C.bagua_bucket_reset_comm_ready(self._handle), "reset comm ready")

    # ---- execution ---------------------------------------------------------------
    def execute_ops(self, stream_ptr: Optional[int] = None) -> None:
        """Run every op now on the bucket's communication tensor (the worker loop body,
        bagua-core-internal/src/lib.rs:241-246); synchronous like the reference
        (datatypes/mod.rs:1062-1066) unless an op's communicator is async (then it
        returns once the work is queued).  stream_ptr: the stream the pack / copy-back
        run on (None: the first op's communicator stream); the ops run on their
        communicator's stream, ordered against it by events."""
        self._refresh()
        N.check(N.C.bagua_bucket_execute(self._handle, int(stream_ptr or 0)), f"ops of bucket {self.name}")
