"""BaguaCommBackendPy — ordered-bucket scheduler (bagua-core-internal/src/lib.rs:125-338,
bagua-core-py/src/lib.rs:301-350).

A thin handle on the native scheduler (`BaguaCommBackendC`,
csrc/runtime/backend.cpp): `register_ordered_buckets(buckets)` fixes the order;
`mark_communication_ready(tensor, ready_event_ptr)` marks a tensor (by name),
and while the FRONT bucket is fully ready it is rotated to the back and
scheduled on a bounded channel to one native worker thread, which makes the
communicator stream wait for the tensors' ready events and runs the bucket's
ops; `wait_pending_comm_ops()` blocks until every scheduled bucket finished and
returns how many.  A native monitor fails an op still running 300 s after the
worker picked it up (lib.rs:255-265): it aborts the op's communicators and
wait_pending_comm_ops raises with the monitor's message, where the reference
panics the process.  Every
call releases the GIL (ctypes), so buckets communicate while Python computes.
"""
from __future__ import annotations

import ctypes

from . import _native as N
from .bucket import BaguaBucketPy
from .tensor import _DTYPES, BaguaTensorPy

_backend_mark = N.FAST.backend_mark

# Buckets of a backend destroyed while an aborted op's worker call never returned: the
# native side leaves that worker (and the backend) running, so what it may still touch
# -- the buckets, their ops, tensors and communicators -- is kept here for good.
_ABANDONED: list = []


class BaguaCommBackendPy:
    def __init__(self, schedule_channel_cap: int, device_id: int):
        self.device_id = int(device_id)
        handle = N.C.bagua_comm_backend_create(max(1, int(schedule_channel_cap)), self.device_id)
        if not handle:
            raise RuntimeError(f"cannot create the comm backend on device {device_id}")
        self._handle = ctypes.c_void_p(handle)
        self._h = int(handle)  # for the fast-path mark
        self._ordered: list[BaguaBucketPy] = []  # keeps the native buckets alive while registered
        self._names: set[str] = set()
        self._reported = 0  # monitor messages already raised by wait_pending_comm_ops

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            if N.C.bagua_comm_backend_stuck(h) != 0:
                _ABANDONED.append(self._ordered)
            self._h = 0
            N.C.bagua_comm_backend_destroy(h)
            self._handle = None

    # ---- API ---------------------------------------------------------------------
    def register_ordered_buckets(self, buckets: list) -> None:
        """lib.rs:270-298: calling again replaces the previous buckets."""
        handles = (ctypes.c_void_p * max(1, len(buckets)))(*[b.handle.value for b in buckets])
        rc = N.C.bagua_comm_backend_register_ordered_buckets(self._handle, handles, len(buckets))
        if rc == N.STATUS_INVALID_ARG:
            seen, ptrs = set(), set()
            for b in buckets:
                for t in b.tensors():
                    if t.name() in seen or t.data_ptr() in ptrs:
                        raise RuntimeError(f"TensorError: duplicated tensor detected, name {t.name()}, "
                                           f"ptr {t.data_ptr()}")
                    seen.add(t.name())
                    ptrs.add(t.data_ptr())
        N.check(rc, "register_ordered_buckets")
        keep = N.C.bagua_comm_backend_stuck(self._handle) != 0  # see wait_pending_comm_ops
        for b in self._ordered:  # the native call waited for everything scheduled
            if not keep:
                b._release_retired()
            b._schedulers.discard(self)
        self._ordered = list(buckets)
        for b in self._ordered:
            b._schedulers.add(self)
        self._names = {t.name() for b in buckets for t in b.tensors()}

    def mark_communication_ready(self, tensor: BaguaTensorPy, ready_cuda_event_ptr: int) -> None:
        """lib.rs:300-319.  The tensor's current storage goes with it (the reference reads
        data_ptr / numel at run time, datatypes/mod.rs:775-791).  One call per gradient
        tensor per step: the torch-backed case goes through the CPython fast path
        (csrc/pyext/fastpath.c) with plain ints; errors are explained after the fact."""
        t = tensor._torch
        if t is not None:
            ptr = t.data_ptr()
            dev = tensor._mark_dev if ptr == tensor._mark_ptr else tensor._mark_device(ptr)
            spec = _DTYPES.get(t.dtype)
            rc = _backend_mark(self._h, tensor._name_b, ready_cuda_event_ptr or 0, ptr, t.numel(),
                               spec[0] if spec else -1, dev)
        else:
            rc = N.C.bagua_comm_backend_mark_communication_ready_desc(
                self._handle, tensor._name_b, int(ready_cuda_event_ptr or 0), ctypes.byref(tensor._raw))
        if rc:
            self._mark_failed(tensor, rc)

    def _mark_failed(self, tensor: BaguaTensorPy, rc: int) -> None:
        if not self._ordered:
            raise RuntimeError("BackendError: ordered buckets not yet set in comm backend")
        name = tensor.name()
        if name not in self._names:
            raise RuntimeError(f"TensorError: tensor {name} is not registered in any bucket")
        N.check(rc, "mark_communication_ready")

    def wait_pending_comm_ops(self) -> int:
        """lib.rs:321-337: wait for every scheduled op; returns how many finished."""
        n = ctypes.c_int(0)
        rc = N.C.bagua_comm_backend_wait_pending_comm_ops(self._handle, ctypes.byref(n))
        # Nothing scheduled is left to run, so cleared ops may go now -- unless an op was
        # abandoned (aborted, its worker call never returned): that call may still touch
        # its tensors and communicators, so every retired op stays referenced for good.
        if N.C.bagua_comm_backend_stuck(self._handle) == 0:
            for b in self._ordered:
                b._release_retired()
        if rc:
            msgs = self.failures()
            why = "; ".join(msgs[self._reported:])  # only failures not raised before
            self._reported = len(msgs)
            raise RuntimeError(f"comm op failed: {N.STATUS.get(rc, rc)} ({n.value} ops waited for)"
                               + (f": {why}" if why else ""))
        return n.value

    def _holds(self, bucket: BaguaBucketPy) -> bool:
        """the scheduler may still run `bucket` (it is registered here)"""
        return any(b is bucket for b in self._ordered)

    def set_lanes(self, lanes: int) -> None:
        """cross-bucket pipelining: bucket i runs on lane 1 + i % lanes of its communicator
        (1 = every bucket on the communicator's stream); waits for everything scheduled"""
        N.check(N.C.bagua_comm_backend_set_lanes(self._handle, int(lanes)), "set_lanes")

    def lanes(self) -> int:
        return int(N.C.bagua_comm_backend_lanes(self._handle))

    def set_op_timeout(self, seconds: float) -> None:
        """the monitor's limit (default 300 s, lib.rs:255-265; BAGUA_COMM_OP_TIMEOUT_S): an op
        still running that long after the worker picked it up is failed and its
        communicators are aborted, so wait_pending_comm_ops raises instead of hanging"""
        N.check(N.C.bagua_comm_backend_set_op_timeout_ms(self._handle, max(1, int(seconds * 1000))),
                "set_op_timeout")

    def failures(self) -> list[str]:
        """the monitor's messages, one per op it failed"""
        out = []
        buf = ctypes.create_string_buffer(512)
        for i in range(max(0, N.C.bagua_comm_backend_failures(self._handle))):
            if N.C.bagua_comm_backend_failure_message(self._handle, i, buf, len(buf)) >= 0:
                out.append(buf.value.decode(errors="replace"))
        return out
