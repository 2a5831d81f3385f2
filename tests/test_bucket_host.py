"""Host-side bucket bookkeeping (no GPU): BaguaBucketPy over descriptors of
fake device pointers -- the native bucket never dereferences them unless it
executes.  Mirrors the reference's bucket lifecycle (datatypes/mod.rs:1072-1267,
bagua-core-py/src/lib.rs:352-487)."""
import ctypes
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


def test_readiness_by_flags_through_the_fast_path():
    """The native bucket's readiness (datatypes/mod.rs:1256-1266) through the CPython
    fast path (csrc/pyext/fastpath.c): every non-padding tensor marked once makes the
    bucket ready, repeated marks count once, padding tensors count as ready, an unknown
    name or a dtype change is refused, and a reset starts over."""
    import bagua_core as bc
    from bagua_core import _native as N
    names = ["w0", "bagua_padding_tensor_x", "w1", "w2"]
    ts = [_tensor(bc, N, nm, 0x7f0000200000 + i * 8192) for i, nm in enumerate(names)]
    b = bc.BaguaBucketPy("flags", ts)
    h = b.handle.value

    def mark(name, ev=0, dtype=N.DTYPE_F32, ptr=0x7f0000300000):
        return N.FAST.bucket_mark(h, name.encode(), ev, ptr, 1024, dtype, 0)

    for _ in range(2):
        assert not b.ready_for_comm()
        assert mark("w0", 11) == 0 and mark("w0", 12) == 0  # repeated: counted once
        assert mark("w2") == 0
        assert not b.ready_for_comm()
        assert mark("nope") == N.STATUS_INVALID_ARG
        assert mark("w1", dtype=N.DTYPE_F16) == N.STATUS_INVALID_ARG  # dtype may not change
        assert not b.ready_for_comm()
        assert mark("w1", 11) == 0
        assert b.ready_for_comm()  # the padding tensor was never marked
        b.reset_comm_ready()
    # a refresh by an unknown name is refused too
    assert N.C.bagua_bucket_refresh_tensor(b.handle, b"missing", ctypes.byref(ts[0]._raw)) == N.STATUS_INVALID_ARG
    with pytest.raises(TypeError):
        N.FAST.bucket_mark(h, b"w0", 0)


def test_backend_mark_error_messages_without_a_gpu():
    """mark_communication_ready's error path keeps the reference's messages
    (lib.rs:300-319) while the call itself goes through the fast path."""
    import bagua_core as bc
    from bagua_core import _native as N
    from bagua_core.backend import BaguaCommBackendPy
    be = BaguaCommBackendPy.__new__(BaguaCommBackendPy)  # no native handle: the call returns an error
    be._handle, be._h, be._ordered, be._names = ctypes.c_void_p(0), 0, [], set()
    t = _tensor(bc, N, "g0", 0x7f0000400000)
    with pytest.raises(RuntimeError, match="ordered buckets not yet set"):
        be.mark_communication_ready(t, 0)
    be._ordered = [object()]
    with pytest.raises(RuntimeError, match="not registered in any bucket"):
        be.mark_communication_ready(t, 0)
    assert N.FAST.backend_mark(0, b"g0", 0, 1, 1, 0, 0) == N.STATUS_INVALID_ARG


def test_bucket_mark_tensor_ready_api_without_a_gpu():
    """BaguaBucketPy.mark_tensor_ready (datatypes/mod.rs:793-813): marking every tensor
    makes the bucket ready, a tensor of another bucket is refused with the bucket's name
    in the message, and reset_comm_ready starts over."""
    import bagua_core as bc
    from bagua_core import _native as N
    ts = [_tensor(bc, N, f"m{i}", 0x7f0000500000 + i * 8192) for i in range(3)]
    b = bc.BaguaBucketPy("api", ts)
    stranger = _tensor(bc, N, "elsewhere", 0x7f0000600000)
    for _ in range(2):
        for t in ts[:2]:
            b.mark_tensor_ready(t)
        assert not b.ready_for_comm()
        with pytest.raises(RuntimeError, match="not in bucket api"):
            b.mark_tensor_ready(stranger)
        b.mark_tensor_ready(ts[2], 0)
        assert b.ready_for_comm()
        b.reset_comm_ready()


def test_python_surface_names_every_reference_method():
    """Every method of the reference's Python classes (bagua-core-py/src/lib.rs:19-487) exists
    on the mirror; the collective wrappers that no compressed op uses (alltoall_v, gather,
    scatter, reduce_scatter) raise NotImplementedError, not AttributeError."""
    import bagua_core as bc
    surface = {
        bc.BaguaSingleCommunicatorPy: "nranks rank device_id abort check_abort allreduce allreduce_inplace broadcast "
                                      "reduce reduce_inplace send recv alltoall alltoall_inplace alltoall_v allgather "
                                      "allgather_inplace gather gather_inplace scatter scatter_inplace reduce_scatter "
                                      "reduce_scatter_inplace barrier generate_nccl_unique_id_str",
        bc.BaguaTensorPy: "compress to_numpy_f32 to_numpy_u8 decompress_from data_ptr device_id num_elements "
                          "num_elements_allocated dtype",
        bc.BaguaCommBackendPy: "register_ordered_buckets mark_communication_ready wait_pending_comm_ops",
        bc.BaguaBucketPy: "tensors append_python_op append_centralized_synchronous_op "
                          "append_decentralized_synchronous_op append_low_precision_decentralized_synchronous_op "
                          "append_decentralized_asynchronous_op print_ops clear_ops ready_for_comm reset_comm_ready",
    }
    for cls, names in surface.items():
        for name in names.split():
            assert callable(getattr(cls, name, None)), f"{cls.__name__}.{name}"
    c = bc.BaguaSingleCommunicatorPy.__new__(bc.BaguaSingleCommunicatorPy)  # no RCCL communicator needed
    for name, args in (("alltoall_v", (None, [], [], None, [], [])), ("gather", (None, None, 0)),
                       ("gather_inplace", (None, 0, 0)), ("scatter", (None, None, 0)), ("scatter_inplace", (None, 0, 0)),
                       ("reduce_scatter", (None, None, 0)), ("reduce_scatter_inplace", (None, 0))):
        with pytest.raises(NotImplementedError):
            getattr(c, name)(*args)
