"""GPU tests of the per-stream state behind the codec (round-2 advisor items).

* The one-launch encode's slot (ticket counter + exchange granules) and the
  per-stream workspace are keyed per REAL stream: the hipStreamPerThread
  sentinel names a different stream on every host thread, so two threads
  encoding on it concurrently get separate slots (they would otherwise fold
  each other's min/max silently).
* Slots are released with the stream (bagua_release_stream_resources,
  communicator teardown) and, once all 64 are owned, the least recently used
  one is reclaimed only after its last launch completed: more than 64 streams
  keep the one-launch encode and stay bit-exact.
* A compressed tensor dropped while queued work still reads it goes back to
  the pool behind an event (bagua_pool_free_after), not immediately.
* The scheduler keys readiness and ready events by tensor name, so any
  wrapper of a registered tensor marks it ready.
Every payload is compared byte-for-byte with the C oracle (K:533-571).
"""
import ctypes
import os
import threading

import numpy as np
import pytest
import torch

from test_gpu_codec import F32, to_dev
from test_gpu_resident import make_input

pytestmark = pytest.mark.gpu

PER_THREAD = 2  # hipStreamPerThread


@pytest.fixture(scope="module")
def N():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from bagua_core import _native
    return _native


@pytest.fixture(autouse=True)
def small_threshold():
    old = os.environ.get("BAGUA_RESIDENT_MIN_ELEMS")
    os.environ["BAGUA_RESIDENT_MIN_ELEMS"] = str(1 << 22)
    yield
    if old is None:
        os.environ.pop("BAGUA_RESIDENT_MIN_ELEMS", None)
    else:
        os.environ["BAGUA_RESIDENT_MIN_ELEMS"] = old


def _buffers(K, n, p):
    cs = n // p
    S = K.bagua_minmax_u8_compressed_bytes(F32, cs, p)
    out = torch.full((S,), 0xA5, dtype=torch.uint8, device="cuda")
    wsb = K.bagua_minmax_u8_workspace_bytes(cs, p)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    return out, ws, S, wsb


def test_per_thread_stream_two_threads(N, oracle_c):
    """Two host threads each run back-to-back one-launch encodes on
    hipStreamPerThread at the same time: every payload exact."""
    K = N.K
    n, p, rounds = 1 << 22, 2, 6
    xs = [[make_input(n, F32, seed=500 + 10 * t + i) for i in range(rounds)] for t in range(2)]
    xts = [[to_dev(x, F32) for x in row] for row in xs]
    bufs = [[_buffers(K, n, p) for _ in range(rounds)] for _ in range(2)]
    torch.cuda.synchronize()
    sp = ctypes.c_void_p(PER_THREAD)
    for xt, (out, ws, S, wsb) in zip(xts[0][:1], bufs[0][:1]):  # the path is the one-launch encode
        assert K.bagua_minmax_u8_resident_path(F32, xt.data_ptr(), n, n // p, p, out.data_ptr(), S, -1, sp) == 1
    errors = []
    start = threading.Barrier(2)

    def worker(t):
        try:
            start.wait()
            for xt, (out, ws, S, wsb) in zip(xts[t], bufs[t]):
                rc = K.bagua_minmax_u8_compress(F32, xt.data_ptr(), n, n // p, p, out.data_ptr(), S, ws.data_ptr(),
                                                wsb, -1, sp)
                if rc:
                    errors.append(rc)
        except BaseException as e:  # pragma: no cover - surfaced below
            errors.append(e)

    before = K.bagua_minmax_u8_resident_slots_in_use(0)
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    torch.cuda.synchronize()  # device-wide: drains both threads' per-thread streams
    assert not errors, errors
    # one slot per (sentinel, thread)
    assert K.bagua_minmax_u8_resident_slots_in_use(0) >= before + 2
    for t in range(2):
        for x, (out, *_rest) in zip(xs[t], bufs[t]):
            assert np.array_equal(out.cpu().numpy(), oracle_c.compress_minmax_u8(x, F32, p))


def test_more_streams_than_slots(N, oracle_c):
    """70 streams (> 64 slots), encodes queued on all of them without host
    waits: reclaimed slots are handed over only after their last launch."""
    K = N.K
    n, p = 1 << 22, 1
    x = make_input(n, F32, seed=77)
    xt = to_dev(x, F32)
    want = oracle_c.compress_minmax_u8(x, F32, p)
    streams = [torch.cuda.Stream() for _ in range(70)]
    bufs = [_buffers(K, n, p) for _ in streams]
    torch.cuda.synchronize()
    for st, (out, ws, S, wsb) in zip(streams, bufs):
        sp = ctypes.c_void_p(st.cuda_stream)
        assert K.bagua_minmax_u8_resident_path(F32, xt.data_ptr(), n, n, p, out.data_ptr(), S, -1, sp) == 1
        assert K.bagua_minmax_u8_compress(F32, xt.data_ptr(), n, n, p, out.data_ptr(), S, ws.data_ptr(), wsb, -1,
                                          sp) == 0
    torch.cuda.synchronize()
    assert K.bagua_minmax_u8_resident_slots_in_use(0) <= 64
    for out, *_rest in bufs:
        assert np.array_equal(out.cpu().numpy(), want)
    for st in streams:
        assert K.bagua_minmax_u8_release_stream(ctypes.c_void_p(st.cuda_stream)) == 0
    # a released stream takes a slot again on its next encode
    out, ws, S, wsb = bufs[0]
    sp = ctypes.c_void_p(streams[0].cuda_stream)
    used = K.bagua_minmax_u8_resident_slots_in_use(0)
    assert K.bagua_minmax_u8_compress(F32, xt.data_ptr(), n, n, p, out.data_ptr(), S, ws.data_ptr(), wsb, -1, sp) == 0
    assert K.bagua_minmax_u8_resident_slots_in_use(0) == used + 1
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), want)
    assert K.bagua_minmax_u8_release_stream(sp) == 0
    assert K.bagua_minmax_u8_resident_slots_in_use(0) == used


def test_release_stream_resources(N):
    """A stream's workspace and slot go away with bagua_release_stream_resources."""
    import bagua_core
    st = torch.cuda.Stream()
    xt = torch.randn(1 << 22, device="cuda")
    count0 = N.C.bagua_stream_workspace_count()
    slots0 = N.K.bagua_minmax_u8_resident_slots_in_use(0)
    with torch.cuda.stream(st):
        comp = bagua_core.BaguaTensorPy(xt, "x").compress("MinMaxUInt8", 1, -1)
    assert N.C.bagua_stream_workspace_count() == count0 + 1
    assert N.K.bagua_minmax_u8_resident_slots_in_use(0) == slots0 + 1
    assert N.C.bagua_release_stream_resources(0, st.cuda_stream) == 0
    assert N.C.bagua_stream_workspace_count() == count0
    assert N.K.bagua_minmax_u8_resident_slots_in_use(0) == slots0
    del comp


def test_communicator_teardown_releases_streams(N):
    """Destroying a communicator drops the workspaces/slots of its streams."""
    from bagua_core.communicator import loopback_communicators
    import bagua_core
    count0 = N.C.bagua_stream_workspace_count()
    comms = loopback_communicators(1, 0)
    t = torch.randn(1 << 22, device="cuda")
    b = bagua_core.BaguaBucketPy("b", [bagua_core.BaguaTensorPy(t, "t")])
    b.append_centralized_synchronous_op(comms[0], None, False, True, False, "MinMaxUInt8")
    b.execute_ops()
    assert N.C.bagua_stream_workspace_count() > count0
    del b, comms
    import gc
    gc.collect()
    assert N.C.bagua_stream_workspace_count() == count0


def test_pool_free_after_waits_for_the_stream(N):
    """A block freed behind queued work is not handed out again until the
    stream has passed that point."""
    C = N.C
    st = torch.cuda.Stream()
    size = 3 << 20
    a = ctypes.c_uint64()
    assert C.bagua_pool_alloc(0, size, ctypes.byref(a)) == 0
    with torch.cuda.stream(st):
        torch.cuda._sleep(200_000_000)  # ~0.1 s of queued work on `st`
    arr = (ctypes.c_uint64 * 1)(st.cuda_stream)
    assert C.bagua_pool_free_after(a.value, arr, 1) == 0
    assert C.bagua_pool_bytes_pending(0) >= size
    b = ctypes.c_uint64()
    assert C.bagua_pool_alloc(0, size, ctypes.byref(b)) == 0
    assert b.value != a.value  # still pending behind the sleep
    st.synchronize()
    c = ctypes.c_uint64()
    assert C.bagua_pool_alloc(0, size, ctypes.byref(c)) == 0
    assert c.value == a.value  # reaped once the stream passed the event
    assert C.bagua_pool_bytes_pending(0) == 0
    assert C.bagua_pool_free(b.value) == 0 and C.bagua_pool_free(c.value) == 0


def test_compressed_tensor_release_is_stream_ordered(N, oracle_c):
    """Dropping a compressed tensor right after decompress_from queues the
    release behind that stream; the decode still reads intact bytes."""
    import bagua_core
    n = 1 << 20
    x = make_input(n, F32, seed=91)
    xt = to_dev(x, F32)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        comp = bagua_core.BaguaTensorPy(xt, "x").compress("MinMaxUInt8", 1, -1)
        torch.cuda._sleep(100_000_000)  # the decode below is queued behind this
        y = torch.empty_like(xt)
        bagua_core.BaguaTensorPy(y, "y").decompress_from("MinMaxUInt8", 1, comp)
        del comp  # stream-ordered release
    # another stream allocates the same size class right away: it must not get
    # the pending block (it would overwrite it before the queued decode ran)
    s2 = torch.cuda.Stream()
    with torch.cuda.stream(s2):
        z = torch.zeros_like(xt)
        comp2 = bagua_core.BaguaTensorPy(z, "z").compress("MinMaxUInt8", 1, -1)
    st.synchronize()
    s2.synchronize()
    want = oracle_c.compress_minmax_u8(x, F32, 1)
    dw = np.empty_like(x)
    oracle_c.decompress_minmax_u8(want, 1, dw, F32)
    assert np.array_equal(y.cpu().numpy().view(np.uint32), dw.view(np.uint32))
    del comp2


def test_backend_readiness_by_name(N):
    """Marking readiness through a different wrapper of a registered tensor
    (same name) makes the bucket ready (lib.rs:300-319)."""
    import bagua_core
    from bagua_core.communicator import loopback_communicators
    comms = loopback_communicators(1, 0)
    t = torch.randn(4096, device="cuda")
    reg = bagua_core.BaguaTensorPy(t, "grad0")
    bucket = bagua_core.BaguaBucketPy("bucket0", [reg])
    bucket.append_centralized_synchronous_op(comms[0], None, False, True, False, "MinMaxUInt8")
    backend = bagua_core.BaguaCommBackendPy(4, 0)
    backend.register_ordered_buckets([bucket])
    other = bagua_core.BaguaTensorPy(t, "grad0")  # a second wrapper, same name
    ev = torch.cuda.Event()
    ev.record()
    backend.mark_communication_ready(other, ev.cuda_event)
    assert backend.wait_pending_comm_ops() == 1


def test_resident_encode_replayed_from_a_graph(N, oracle_c):
    """The one-launch encode captured into a HIP graph: every replay draws fresh
    tickets (tags advance without the host) and stays bit-exact on new data; the
    captured slot is never handed to another stream, even after a release."""
    K = N.K
    n, p = 1 << 22, 2
    xs = [make_input(n, F32, seed=300 + i) for i in range(3)]
    xt = to_dev(xs[0], F32)
    out, ws, S, wsb = _buffers(K, n, p)
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    assert K.bagua_minmax_u8_resident_path(F32, xt.data_ptr(), n, n // p, p, out.data_ptr(), S, -1, sp) == 1
    # warm up outside capture (one-time attribute/occupancy setup)
    assert K.bagua_minmax_u8_compress(F32, xt.data_ptr(), n, n // p, p, out.data_ptr(), S, ws.data_ptr(), wsb, -1,
                                      sp) == 0
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        rc = K.bagua_minmax_u8_compress(F32, xt.data_ptr(), n, n // p, p, out.data_ptr(), S, ws.data_ptr(), wsb, -1,
                                        sp)
    assert rc == 0
    for x in xs:
        xt.copy_(torch.from_numpy(x).cuda())
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), oracle_c.compress_minmax_u8(x, F32, p))
    used = K.bagua_minmax_u8_resident_slots_in_use(0)
    assert K.bagua_minmax_u8_release_stream(sp) == 0
    assert K.bagua_minmax_u8_resident_slots_in_use(0) == used - 1
    # the graph still owns its slot: a replay after the release is still exact
    xt.copy_(torch.from_numpy(xs[1]).cuda())
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), oracle_c.compress_minmax_u8(xs[1], F32, p))
