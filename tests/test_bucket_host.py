"""Host-side bucket bookkeeping (no GPU): BaguaBucketPy over descriptors of
fake device pointers -- the native bucket never dereferences them unless it
executes.  Mirrors the reference's bucket lifecycle (datatypes/mod.rs:1072-1267,
bagua-core-py/src/lib.rs:352-487)."""
import gc
import weakref

import pytest

pytest.importorskip("torch")


def _tensor(bc, N, name, ptr, n=1024):
    raw = N.bagua_tensor_t(ptr, n, n, N.DTYPE_F32, 0)
    return bc.BaguaTensorPy._from_raw(raw, name, owned=False)


def test_clear_ops_without_scheduler_keeps_nothing():
    """clear_ops on a bucket that only runs through execute_ops must not
    accumulate the cleared ops (their ctypes thunks and communicator handles)."""
    import bagua_core as bc
    from bagua_core import _native as N
    ts = [_tensor(bc, N, f"t{i}", 0x7f0000000000 + i * 4096) for i in range(3)]
    b = bc.BaguaBucketPy("b", ts)
    cbs = []
    for _ in range(50):
        op = lambda name: None  # noqa: E731
        cbs.append(weakref.ref(op))
        b.append_python_op(op)
        assert N.C.bagua_bucket_num_ops(b.handle) == 1
        b.clear_ops()
        assert N.C.bagua_bucket_num_ops(b.handle) == 0
    assert b._retired == []
    del op
    gc.collect()
    assert all(r() is None for r in cbs), "cleared ops are still referenced"


def test_clear_ops_while_scheduled_keeps_ops_until_released():
    """A bucket registered with a scheduler keeps its cleared ops until the scheduler
    releases them (wait_pending_comm_ops / re-registration)."""
    import bagua_core as bc
    from bagua_core import _native as N

    class FakeScheduler:  # the part of BaguaCommBackendPy the bucket consults
        def __init__(self, buckets):
            self._ordered = list(buckets)

        def _holds(self, bucket):
            return any(x is bucket for x in self._ordered)

    b = bc.BaguaBucketPy("b", [_tensor(bc, N, "x", 0x7f0000100000)])
    sched = FakeScheduler([b])
    b._schedulers.add(sched)
    b.append_python_op(lambda name: None)
    b.clear_ops()
    assert len(b._retired) == 1
    b._release_retired()
    assert b._retired == []
    sched._ordered = []  # deregistered: nothing can run the bucket any more
    b.append_python_op(lambda name: None)
    b.clear_ops()
    assert b._retired == []
