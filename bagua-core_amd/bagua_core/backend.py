"""BaguaCommBackendPy — ordered-bucket scheduler (bagua-core-internal/src/lib.rs:176-338,
bagua-core-py/src/lib.rs:301-350).

Same contract as the reference: `register_ordered_buckets(buckets)` fixes the
order; `mark_communication_ready(tensor, ready_event_ptr)` marks a tensor,
and while the FRONT bucket is fully ready it is rotated to the back and
scheduled on a bounded channel to one worker thread that runs its ops;
`wait_pending_comm_ops()` blocks until every scheduled bucket finished and
returns how many.  A monitor flags an op running longer than 300 s
(lib.rs:255-265; here it logs and records the failure instead of panicking
the process).  The worker's op calls release the GIL (ctypes), so buckets
communicate while Python keeps computing.
"""
from __future__ import annotations

import queue
import threading
import time
from typing import Optional

import torch

from . import _native as N
from .bucket import BaguaBucketPy
from .tensor import BaguaTensorPy

WATCHDOG_SECONDS = 300.0


class _Scheduled:
    def __init__(self, bucket: BaguaBucketPy, events: list[int]):
        self.bucket = bucket
        self.events = events
        self.done = threading.Event()
        self.error: Optional[BaseException] = None


class BaguaCommBackendPy:
    def __init__(self, schedule_channel_cap: int, device_id: int):
        self.device_id = int(device_id)
        self._channel: "queue.Queue[Optional[_Scheduled]]" = queue.Queue(maxsize=max(1, int(schedule_channel_cap)))
        self._pending: "queue.Queue[_Scheduled]" = queue.Queue()
        self._ordered: list[BaguaBucketPy] = []
        self._mapping: dict[str, BaguaBucketPy] = {}
        self._events: dict[str, int] = {}  # ready event per tensor name
        self._current: Optional[tuple[_Scheduled, float]] = None
        self._failures: list[str] = []
        self._worker = threading.Thread(target=self._work, name="bagua-comm-worker", daemon=True)
        self._worker.start()
        self._monitor = threading.Thread(target=self._watch, name="bagua-comm-monitor", daemon=True)
        self._monitor.start()

    # ---- API ---------------------------------------------------------------------
    def register_ordered_buckets(self, buckets: list) -> None:
        """lib.rs:270-298: calling again replaces the previous buckets."""
        self.wait_pending_comm_ops()
        self._ordered, self._mapping, ptrs = [], {}, set()
        for b in buckets:
            for t in b.tensors():
                if t.name() in self._mapping or t.data_ptr() in ptrs:
                    raise RuntimeError(f"TensorError: duplicated tensor detected, name {t.name()}, "
                                       f"ptr {t.data_ptr()}")
                self._mapping[t.name()] = b
                ptrs.add(t.data_ptr())
            self._ordered.append(b)

    def mark_communication_ready(self, tensor: BaguaTensorPy, ready_cuda_event_ptr: int) -> None:
        """lib.rs:300-319"""
        if not self._ordered:
            raise RuntimeError("BackendError: ordered buckets not yet set in comm backend")
        bucket = self._mapping.get(tensor.name())
        if bucket is None:
            raise RuntimeError(f"TensorError: tensor {tensor.name()} is not registered in any bucket")
        bucket.mark_tensor_ready(tensor)
        if ready_cuda_event_ptr:
            self._events[tensor.name()] = int(ready_cuda_event_ptr)
        while self._ordered[0].ready_for_comm():
            b = self._ordered.pop(0)
            b.reset_comm_ready()
            self._ordered.append(b)
            evs = [self._events.pop(t.name(), 0) for t in b.tensors()]
            item = _Scheduled(b, [e for e in evs if e])
            self._channel.put(item)
            self._pending.put(item)

    def wait_pending_comm_ops(self) -> int:
        """lib.rs:321-337: wait for every scheduled op; returns how many finished."""
        n = 0
        while True:
            try:
                item = self._pending.get_nowait()
            except queue.Empty:
                return n
            item.done.wait()
            n += 1
            if item.error is not None:
                raise RuntimeError(f"comm op on bucket {item.bucket.name} failed: {item.error}") from item.error

    # ---- worker / monitor ----------------------------------------------------------
    def _work(self) -> None:
        torch.cuda.set_device(self.device_id)
        while True:
            item = self._channel.get()
            if item is None:
                return
            self._current = (item, time.monotonic())
            try:
                stream = _bucket_stream(item.bucket)
                for ev in item.events:
                    N.check(N.C.bagua_stream_wait_event(stream, ev), "stream wait on tensor ready event")
                item.bucket.execute_ops(stream)
            except BaseException as e:  # surfaced by wait_pending_comm_ops
                item.error = e
            finally:
                self._current = None
                item.done.set()

    def _watch(self) -> None:
        while True:
            time.sleep(5.0)
            cur = self._current
            if cur is not None and time.monotonic() - cur[1] > WATCHDOG_SECONDS:
                msg = f"comm op on bucket {cur[0].bucket.name} has not finished for 5 min"
                if msg not in self._failures:
                    self._failures.append(msg)
                    print(f"[bagua-core] {msg}", flush=True)

    def failures(self) -> list[str]:
        return list(self._failures)


def _bucket_stream(bucket: BaguaBucketPy) -> int:
    for op in bucket.ops():
        comm = getattr(op, "communicator", None)
        if comm is not None:
            return comm.stream_ptr()
    return 0
