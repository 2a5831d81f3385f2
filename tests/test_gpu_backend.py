"""GPU tests of the native bucket + scheduler (csrc/runtime/backend.cpp), the
reference's BaguaCommBackend (bagua-core-internal/src/lib.rs:125-338) and
BaguaBucket (datatypes/mod.rs:1072-1267) semantics:

* buckets are scheduled in registration order, each as soon as it and every
  bucket before it are fully ready (lib.rs:300-319), and run on one worker;
* the worker waits for the tensors' ready events on the communicator stream;
* a Python op is called with the bucket's name (python_ffi_op.rs);
* a bounded channel (capacity 1) still schedules every bucket;
* an op failure surfaces from wait_pending_comm_ops;
* results equal the oracle simulation of the reference op sequence, for
  contiguous buckets (in place) and scattered ones (packed + copied back).
"""
import ctypes
import threading

import numpy as np
import pytest
import torch

from oracle import simulate

pytestmark = pytest.mark.gpu

F32 = 0


@pytest.fixture(scope="module")
def bc():
    import bagua_core
    return bagua_core


@pytest.fixture(scope="module")
def comm(bc):
    stream = torch.cuda.Stream()
    uid = bc.BaguaSingleCommunicatorPy.generate_nccl_unique_id_str()
    c = bc.BaguaSingleCommunicatorPy(0, 1, 0, stream.cuda_stream, uid)
    c._keep_stream = stream
    return c


def _grads(n_buckets, per, seed, scattered=False):
    rng = np.random.default_rng(seed)
    host = [(rng.standard_normal(per) * 1e-3).astype(np.float32) for _ in range(n_buckets)]
    if scattered:  # every tensor its own allocation, with gaps between them
        devs, keep = [], []
        for h in host:
            parts = []
            for q in np.array_split(h, 3):
                parts.append(torch.from_numpy(q.copy()).cuda())
                keep.append(torch.empty(4096, device="cuda"))
            devs.append(parts)
        return host, devs, keep
    flats = [torch.from_numpy(h.copy()).cuda() for h in host]
    return host, [list(f.view(3, -1).unbind(0)) if per % 3 == 0 else [f] for f in flats], flats


@pytest.mark.parametrize("lanes", [1, 2, 3])
@pytest.mark.parametrize("scattered", [False, True])
def test_scheduler_runs_buckets_in_order_and_matches_oracle(bc, comm, oracle_c, scattered, lanes):
    n_buckets, per = 6, 3 * 40000
    host, parts, _keep = _grads(n_buckets, per, 7 + scattered, scattered)
    log = []
    buckets, tensors = [], []
    for b in range(n_buckets):
        ts = [bc.BaguaTensorPy(t, f"g{b}.{i}") for i, t in enumerate(parts[b])]
        bk = bc.BaguaBucketPy(f"bucket{b}", ts)
        bk.append_centralized_synchronous_op(comm, None, False, True, False, "MinMaxUInt8")
        bk.append_python_op(lambda name: log.append(name))
        buckets.append(bk)
        tensors.append(ts)
    backend = bc.BaguaCommBackendPy(2, 0)
    backend.set_lanes(lanes)  # cross-bucket pipelining: bucket i on lane 1 + i % lanes
    assert backend.lanes() == lanes
    backend.register_ordered_buckets(buckets)
    ev = torch.cuda.Event()
    # mark the LAST bucket first: nothing may run until bucket 0 is ready
    for t in tensors[-1]:
        backend.mark_communication_ready(t, 0)
    assert backend.wait_pending_comm_ops() == 0
    for b in range(n_buckets - 1):
        ev.record()
        for t in tensors[b]:
            backend.mark_communication_ready(t, ev.cuda_event)
    assert backend.wait_pending_comm_ops() == n_buckets
    assert log == [f"bucket{b}" for b in range(n_buckets)], log  # registration order, bucket name passed
    for b in range(n_buckets):
        want = simulate.centralized_low_precision(oracle_c, [host[b]], F32, True)[0]
        got = torch.cat([t.reshape(-1) for t in parts[b]]).cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"bucket {b}"


def test_bounded_channel_capacity_one(bc, comm):
    """capacity 1: scheduling a bucket waits for channel space, never drops one"""
    n_buckets = 12
    flats = [torch.randn(3 * 4096, device="cuda") * 1e-3 for _ in range(n_buckets)]
    seen = []
    buckets = []
    for b, f in enumerate(flats):
        bk = bc.BaguaBucketPy(f"b{b}", [bc.BaguaTensorPy(f, f"t{b}")])
        bk.append_python_op(lambda name: seen.append(name))
        buckets.append(bk)
    backend = bc.BaguaCommBackendPy(1, 0)
    backend.register_ordered_buckets(buckets)
    for it in range(3):
        for b in range(n_buckets):
            backend.mark_communication_ready(buckets[b].tensors()[0], 0)
        assert backend.wait_pending_comm_ops() == n_buckets
    assert seen == [f"b{b}" for b in range(n_buckets)] * 3


def test_ready_event_orders_the_comm_stream(bc, comm, oracle_c):
    """The gradient is written on the compute stream AFTER a long sleep; the event
    recorded behind that write must hold the comm op back (datatypes/mod.rs:969-980)."""
    n = 3 * 50000
    rng = np.random.default_rng(3)
    x = (rng.standard_normal(n) * 1e-3).astype(np.float32)
    t = torch.zeros(n, device="cuda")
    bt = bc.BaguaTensorPy(t, "late")
    bk = bc.BaguaBucketPy("late_bucket", [bt])
    bk.append_centralized_synchronous_op(comm, None, False, True, False, "MinMaxUInt8")
    backend = bc.BaguaCommBackendPy(4, 0)
    backend.register_ordered_buckets([bk])
    src = torch.from_numpy(x).cuda()
    torch.cuda.synchronize()
    torch.cuda._sleep(100_000_000)
    t.copy_(src)
    ev = torch.cuda.Event()
    ev.record()
    backend.mark_communication_ready(bt, ev.cuda_event)
    assert backend.wait_pending_comm_ops() == 1
    want = simulate.centralized_low_precision(oracle_c, [x], F32, True)[0]
    assert np.array_equal(t.cpu().numpy().view(np.uint32), want.view(np.uint32))


def test_op_failure_surfaces(bc):
    """An op that fails (an aborted communicator) is reported by wait_pending_comm_ops."""
    from bagua_core.communicator import loopback_communicators
    comms = loopback_communicators(1, 0)
    comms[0].abort()
    f = torch.randn(3 * 1024, device="cuda")
    bk = bc.BaguaBucketPy("doomed", [bc.BaguaTensorPy(f, "d")])
    bk.append_centralized_synchronous_op(comms[0], None, False, True, False, "MinMaxUInt8")
    backend = bc.BaguaCommBackendPy(2, 0)
    backend.register_ordered_buckets([bk])
    backend.mark_communication_ready(bk.tensors()[0], 0)
    with pytest.raises(RuntimeError, match="comm op failed"):
        backend.wait_pending_comm_ops()


def test_registration_errors(bc, comm):
    f = torch.randn(4096, device="cuda")
    a = bc.BaguaTensorPy(f, "x")
    bk1 = bc.BaguaBucketPy("b1", [a])
    backend = bc.BaguaCommBackendPy(2, 0)
    with pytest.raises(RuntimeError, match="ordered buckets not yet set"):
        backend.mark_communication_ready(a, 0)
    with pytest.raises(RuntimeError, match="duplicated tensor"):
        backend.register_ordered_buckets([bk1, bc.BaguaBucketPy("b2", [bc.BaguaTensorPy(f, "x")])])
    backend.register_ordered_buckets([bk1])
    with pytest.raises(RuntimeError, match="not registered"):
        backend.mark_communication_ready(bc.BaguaTensorPy(torch.randn(8, device="cuda"), "y"), 0)
    with pytest.raises(RuntimeError):
        bc.BaguaBucketPy("mixed", [a, bc.BaguaTensorPy(torch.randn(8, device="cuda", dtype=torch.float16), "h")])


def test_bucket_readiness_api(bc, comm):
    """BaguaBucketPy.ready_for_comm / reset_comm_ready (lib.rs:479-486); padding tensors
    (name prefix bagua_padding_tensor) count as ready."""
    f = torch.randn(3 * 1024, device="cuda")
    ts = [bc.BaguaTensorPy(v, n) for v, n in zip(f.view(3, -1).unbind(0), ["a", "b", "bagua_padding_tensor_0"])]
    bk = bc.BaguaBucketPy("r", ts)
    assert not bk.ready_for_comm()
    bk.mark_tensor_ready(ts[0])
    assert not bk.ready_for_comm()
    bk.mark_tensor_ready(ts[1])
    assert bk.ready_for_comm()
    bk.reset_comm_ready()
    assert not bk.ready_for_comm()
    assert ctypes.c_int(bc._native.C.bagua_bucket_num_ops(bk.handle)).value == 0


def test_async_ops_on_a_communicator(bc, oracle_c):
    """bagua_comm_set_async: ops return once enqueued (their buffers go back to the
    pool behind the stream); many buckets queued back to back, one sync at the end,
    every result equal to the oracle's simulation."""
    N = bc._native
    stream = torch.cuda.Stream()
    uid = bc.BaguaSingleCommunicatorPy.generate_nccl_unique_id_str()
    comm = bc.BaguaSingleCommunicatorPy(0, 1, 0, stream.cuda_stream, uid)
    assert N.C.bagua_comm_set_async(comm.handle, 1) == 0
    rng = np.random.default_rng(11)
    xs = [(rng.standard_normal(3 * 20000 + 96 * i) * 1e-3).astype(np.float32) for i in range(8)]
    ts = [torch.from_numpy(x).cuda() for x in xs]
    torch.cuda.synchronize()
    for rep in range(2):
        for t in ts:
            raw = bc.BaguaTensorPy(t, "g").raw()
            N.check(N.C.bagua_centralized_low_precision_synchronous(comm.handle, ctypes.byref(raw), 1,
                                                                    N.COMPRESSION_MINMAX_UINT8), "op")
    comm.synchronize()
    for x, t in zip(xs, ts):
        want = simulate.centralized_low_precision(oracle_c, [x], F32, True)[0]
        want = simulate.centralized_low_precision(oracle_c, [want], F32, True)[0]
        assert np.array_equal(t.cpu().numpy().view(np.uint32), want.view(np.uint32))
    assert N.C.bagua_comm_set_async(comm.handle, 0) == 0


def test_backend_sync_mode_env(bc, comm, oracle_c, monkeypatch):
    """BAGUA_BACKEND_SYNC=1: the worker waits for every op (the reference's behaviour);
    same results."""
    monkeypatch.setenv("BAGUA_BACKEND_SYNC", "1")
    host, parts, _keep = _grads(3, 3 * 30000, 5, True)
    buckets = []
    for b in range(3):
        bk = bc.BaguaBucketPy(f"s{b}", [bc.BaguaTensorPy(t, f"s{b}.{i}") for i, t in enumerate(parts[b])])
        bk.append_centralized_synchronous_op(comm, None, False, True, False, "MinMaxUInt8")
        buckets.append(bk)
    backend = bc.BaguaCommBackendPy(4, 0)
    backend.register_ordered_buckets(buckets)
    for bk in buckets:
        for t in bk.tensors():
            backend.mark_communication_ready(t, 0)
    assert backend.wait_pending_comm_ops() == 3
    for b in range(3):
        want = simulate.centralized_low_precision(oracle_c, [host[b]], F32, True)[0]
        got = torch.cat([t.reshape(-1) for t in parts[b]]).cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("p,lanes", [(2, 1), (2, 2), (4, 2), (4, 3)])
def test_scheduler_multirank_loopback(bc, oracle_c, p, lanes):
    """p virtual ranks on the loopback transport, each with its own scheduler (worker
    thread, async ops, `lanes` streams per communicator for consecutive buckets) and the
    same ordered buckets: every rank's workers meet in the
    collectives, and every bucket on every rank equals the oracle's simulation of the
    reference op across the ranks (bit-for-bit).  Buckets are marked ready in reverse
    order, as backward produces them; the scheduler runs them in registration order."""
    from bagua_core.communicator import loopback_communicators
    comms = loopback_communicators(p, 0)
    n_buckets, per = 5, 3 * 4096 * p
    rng = np.random.default_rng(100 + p)
    host = [[(rng.standard_normal(per) * 1e-3).astype(np.float32) for _ in range(n_buckets)] for _ in range(p)]
    flats = [[torch.from_numpy(h.copy()).cuda() for h in host[r]] for r in range(p)]
    seen = [[] for _ in range(p)]
    backends, tensors = [], []
    for r in range(p):
        buckets, ts_r = [], []
        for b in range(n_buckets):
            ts = [bc.BaguaTensorPy(v, f"g{b}.{i}") for i, v in enumerate(flats[r][b].view(3, -1).unbind(0))]
            bk = bc.BaguaBucketPy(f"bucket{b}", ts)
            bk.append_centralized_synchronous_op(comms[r], None, False, True, False, "MinMaxUInt8")
            bk.append_python_op(lambda name, r=r: seen[r].append(name))
            buckets.append(bk)
            ts_r.append(ts)
        be = bc.BaguaCommBackendPy(2, 0)
        be.set_lanes(lanes)
        be.register_ordered_buckets(buckets)
        backends.append((be, buckets))
        tensors.append(ts_r)
    torch.cuda.synchronize()
    for it in range(2):
        done = [None] * p

        def rank(r):  # one host thread per rank, as one process per GPU would be
            for b in reversed(range(n_buckets)):
                for t in tensors[r][b]:
                    backends[r][0].mark_communication_ready(t, 0)
            done[r] = backends[r][0].wait_pending_comm_ops()
        ths = [threading.Thread(target=rank, args=(r,)) for r in range(p)]
        for th in ths:
            th.start()
        for th in ths:
            th.join(timeout=120)
        assert done == [n_buckets] * p, done
        for b in range(n_buckets):
            want = simulate.centralized_low_precision(oracle_c, [host[r][b] for r in range(p)], F32, True)
            for r in range(p):
                host[r][b] = want[r]
                got = flats[r][b].cpu().numpy()
                assert np.array_equal(got.view(np.uint32), want[r].view(np.uint32)), (it, b, r)
    assert all(s == [f"bucket{b}" for b in range(n_buckets)] * 2 for s in seen), seen
    del backends


def test_clear_ops_while_a_python_op_is_queued(bc):
    """clear_ops on a bucket that is scheduled but not yet run: the native item holds a
    copy of the op (its ctypes thunk); the Python op must stay alive until the scheduler
    has run it (the reference clones its ops into Arcs, lib.rs:143-146)."""
    import gc
    import time
    gate = threading.Event()
    seen = []
    first = bc.BaguaBucketPy("first", [bc.BaguaTensorPy(torch.zeros(64, device="cuda"), "f0")])
    first.append_python_op(lambda name: (gate.wait(10), seen.append(name)))  # holds the worker
    second = bc.BaguaBucketPy("second", [bc.BaguaTensorPy(torch.zeros(64, device="cuda"), "s0")])
    second.append_python_op(lambda name: seen.append(name))
    backend = bc.BaguaCommBackendPy(4, 0)
    backend.register_ordered_buckets([first, second])
    backend.mark_communication_ready(first.tensors()[0], 0)
    backend.mark_communication_ready(second.tensors()[0], 0)  # queued behind `first`
    time.sleep(0.05)
    second.clear_ops()  # the queued item still refers to the callback
    gc.collect()
    gate.set()
    assert backend.wait_pending_comm_ops() == 2
    assert seen == ["first", "second"], seen
    assert second._retired == []  # released once everything scheduled has run
    # the next iteration runs without the cleared op
    backend.mark_communication_ready(first.tensors()[0], 0)
    backend.mark_communication_ready(second.tensors()[0], 0)
    assert backend.wait_pending_comm_ops() == 2
    assert seen == ["first", "second", "first"], seen


@pytest.mark.parametrize("via", ["scheduler", "execute"])
def test_storage_swapped_after_bucket_creation(bc, comm, oracle_c, via):
    """`t.data = other` after the bucket was built: the op must run on the tensor's
    CURRENT storage (the reference reads data_ptr at run time, datatypes/mod.rs:775-791)
    and leave the old storage alone."""
    n = 3 * 40000
    rng = np.random.default_rng(21)
    x_old = (rng.standard_normal(n) * 1e-3).astype(np.float32)
    x_new = (rng.standard_normal(n) * 1e-3 + 0.25).astype(np.float32)
    t = torch.from_numpy(x_old.copy()).cuda()
    old_storage = t.data
    bt = bc.BaguaTensorPy(t, f"swap_{via}")
    bk = bc.BaguaBucketPy(f"swap_bucket_{via}", [bt])
    bk.append_centralized_synchronous_op(comm, None, False, True, False, "MinMaxUInt8")
    t.data = torch.from_numpy(x_new.copy()).cuda()  # new storage, same tensor object
    torch.cuda.synchronize()
    if via == "scheduler":
        backend = bc.BaguaCommBackendPy(2, 0)
        backend.register_ordered_buckets([bk])
        backend.mark_communication_ready(bt, 0)
        assert backend.wait_pending_comm_ops() == 1
    else:
        bk.execute_ops()
    torch.cuda.synchronize()
    want = simulate.centralized_low_precision(oracle_c, [x_new], F32, True)[0]
    assert np.array_equal(t.cpu().numpy().view(np.uint32), want.view(np.uint32))
    assert np.array_equal(old_storage.cpu().numpy().view(np.uint32), x_old.view(np.uint32))


def test_execute_on_a_foreign_stream_orders_the_pack(bc, comm, oracle_c):
    """execute_ops(stream) with a stream other than the communicator's: the pack (on
    `stream`, behind a long sleep there) must land before the op reads it, and the
    copy-back after the op (event ordering in execute_bucket)."""
    per = 3 * 30000
    rng = np.random.default_rng(22)
    h = (rng.standard_normal(per) * 1e-3).astype(np.float32)
    parts = [torch.from_numpy(q.copy()).cuda() for q in np.array_split(h, 3)]
    gaps = [torch.empty(4096, device="cuda") for _ in range(3)]  # noqa: F841 - scattered tensors
    bk = bc.BaguaBucketPy("foreign", [bc.BaguaTensorPy(p, f"fp{i}") for i, p in enumerate(parts)])
    bk.append_centralized_synchronous_op(comm, None, False, True, False, "MinMaxUInt8")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        torch.cuda._sleep(20_000_000)  # the pack waits behind this on `s`
    bk.execute_ops(s.cuda_stream)
    torch.cuda.synchronize()
    want = simulate.centralized_low_precision(oracle_c, [h], F32, True)[0]
    got = torch.cat(parts).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("lanes", [1, 2])
def test_lanes_pipelined_op_buckets(bc, oracle_c, lanes):
    """Cross-bucket lanes with the pipelined op at p = 2 (side stream per lane, pieces
    exchanged on the loopback transport) over buckets large enough to be pieced, two
    iterations without re-registration: every bucket equals the oracle simulation."""
    from bagua_core.communicator import loopback_communicators
    p, n_buckets, per = 2, 4, 2 * (1 << 21)
    comms = loopback_communicators(p, 0)
    rng = np.random.default_rng(300 + lanes)
    host = [[(rng.standard_normal(per) * 1e-3).astype(np.float32) for _ in range(n_buckets)] for _ in range(p)]
    flats = [[torch.from_numpy(h.copy()).cuda() for h in host[r]] for r in range(p)]
    backends, tensors = [], []
    for r in range(p):
        buckets, ts_r = [], []
        for b in range(n_buckets):
            t = bc.BaguaTensorPy(flats[r][b], f"g{b}")
            bk = bc.BaguaBucketPy(f"bucket{b}", [t])
            bk.append_centralized_synchronous_op(comms[r], None, False, True, False, "MinMaxUInt8")
            buckets.append(bk)
            ts_r.append(t)
        be = bc.BaguaCommBackendPy(4, 0)
        be.set_lanes(lanes)
        be.register_ordered_buckets(buckets)
        backends.append((be, buckets))
        tensors.append(ts_r)
    torch.cuda.synchronize()
    for it in range(2):
        done = [None] * p

        def rank(r):
            for b in reversed(range(n_buckets)):
                backends[r][0].mark_communication_ready(tensors[r][b], 0)
            done[r] = backends[r][0].wait_pending_comm_ops()
        ths = [threading.Thread(target=rank, args=(r,)) for r in range(p)]
        for th in ths:
            th.start()
        for th in ths:
            th.join(timeout=120)
        assert done == [n_buckets] * p, done
        for b in range(n_buckets):
            want = simulate.centralized_low_precision(oracle_c, [host[r][b] for r in range(p)], F32, True)
            for r in range(p):
                host[r][b] = want[r]
                assert np.array_equal(flats[r][b].cpu().numpy().view(np.uint32), want[r].view(np.uint32)), (it, b, r)
    del backends


@pytest.mark.parametrize("p,lanes", [(2, 2), (1, 3)])
def test_lanes_mixed_ops_multirank(bc, oracle_c, p, lanes):
    """Lanes on the loopback transport, buckets alternating between the 1-bit centralized op
    and the decentralized ring op (its weight/peer tensors per bucket): every bucket on every
    rank equals the oracle's simulation, two iterations.  p = 1 runs both ops' one-rank forms
    (two passes each) on three lane streams."""
    from bagua_core.communicator import loopback_communicators
    nb, n = 4, 3 * 16384
    comms = loopback_communicators(p, 0)
    rng = np.random.default_rng(4711)
    host = {(r, b, k): (rng.standard_normal(n) * 1e-3).astype(np.float32) for r in range(p) for b in range(nb)
            for k in "twlr"}
    dev = {key: torch.from_numpy(v.copy()).cuda() for key, v in host.items()}
    backends, tensors = [], []
    for r in range(p):
        buckets, ts_r = [], []
        for b in range(nb):
            t = bc.BaguaTensorPy(dev[(r, b, "t")], f"g{b}")
            bk = bc.BaguaBucketPy(f"bucket{b}", [t])
            if b % 2 == 0:
                bk.append_centralized_synchronous_op(comms[r], None, False, True, False, "OneBitSignScale")
            else:
                w, lft, rgt = (bc.BaguaTensorPy(dev[(r, b, k)], f"{k}{b}") for k in "wlr")
                bk.append_low_precision_decentralized_synchronous_op(comms[r], None, False, "ring", "MinMaxUInt8",
                                                                     w, lft, rgt)
            buckets.append(bk)
            ts_r.append(t)
        be = bc.BaguaCommBackendPy(4, 0)
        be.set_lanes(lanes)
        be.register_ordered_buckets(buckets)
        backends.append((be, buckets))
        tensors.append(ts_r)
    torch.cuda.synchronize()
    for it in range(2):
        want = {}
        for b in range(nb):
            if b % 2 == 0:
                w = simulate.centralized_low_precision(oracle_c, [host[(r, b, "t")].copy() for r in range(p)], F32,
                                                       True, method="OneBitSignScale")
                for r in range(p):
                    want[(r, b, "t")] = w[r]
            else:
                res = simulate.decentralized_low_precision(oracle_c, *[[host[(r, b, k)].copy() for r in range(p)]
                                                                       for k in "twlr"], F32)
                for k, wk in zip("twlr", res):
                    for r in range(p):
                        want[(r, b, k)] = wk[r]
        done = [None] * p

        def rank(r):
            for b in reversed(range(nb)):
                backends[r][0].mark_communication_ready(tensors[r][b], 0)
            done[r] = backends[r][0].wait_pending_comm_ops()
        ths = [threading.Thread(target=rank, args=(r,)) for r in range(p)]
        for th in ths:
            th.start()
        for th in ths:
            th.join(timeout=120)
        assert done == [nb] * p, done
        for key, w in want.items():
            got = dev[key].cpu().numpy()
            assert np.array_equal(got.view(np.uint32), w.view(np.uint32)), (it, key)
            host[key] = w
    del backends


@pytest.mark.parametrize("lanes", [1, 2])
def test_completion_covers_every_bucket_of_a_burst(bc, comm, oracle_c, lanes):
    """Buckets the worker enqueues in one burst share one completion event per lane
    (backend.cpp cover_uncovered).  wait_pending_comm_ops must still return only after
    every bucket's work finished: the ready event trails a long GPU sleep, so every lane
    runs late, and the results are read right after the wait with no other
    synchronisation.  A second burst (on the first one's output) works the same way."""
    n_buckets, per = 5, 3 * 30000
    host, parts, _keep = _grads(n_buckets, per, 11)
    buckets, tensors = [], []
    for b in range(n_buckets):
        ts = [bc.BaguaTensorPy(t, f"c{b}.{i}") for i, t in enumerate(parts[b])]
        bk = bc.BaguaBucketPy(f"cover{b}", ts)
        bk.append_centralized_synchronous_op(comm, None, False, True, False, "MinMaxUInt8")
        buckets.append(bk)
        tensors.append(ts)
    backend = bc.BaguaCommBackendPy(8, 0)
    backend.set_lanes(lanes)
    backend.register_ordered_buckets(buckets)
    want = host
    for it in range(2):
        want = [simulate.centralized_low_precision(oracle_c, [w], F32, True)[0] for w in want]
        torch.cuda._sleep(50_000_000)  # the "backward pass" still running on the default stream
        ev = torch.cuda.Event()
        ev.record()
        for b in range(n_buckets):
            for t in tensors[b]:
                backend.mark_communication_ready(t, ev.cuda_event)
        assert backend.wait_pending_comm_ops() == n_buckets
        for b in range(n_buckets):
            got = torch.cat([t.reshape(-1) for t in parts[b]]).cpu().numpy()
            assert np.array_equal(got.view(np.uint32), want[b].view(np.uint32)), f"iteration {it} bucket {b}"


@pytest.mark.parametrize("dtype", [1, 2])  # F16 (a reference dtype), BF16 (extension)
def test_scheduler_16bit_buckets_match_oracle(bc, comm, oracle_c, dtype):
    """16-bit gradient buckets through the scheduler at the default lanes: every tensor
    is marked through the fast path (csrc/pyext/fastpath.c) with its dtype code, and each
    bucket ends bit-identical to the oracle's simulation of the reference op sequence
    (centralized_low_precision_synchronous.rs:30-71 at one rank)."""
    from oracle import oracle_np as NP
    from test_gpu_multirank import dev, host
    n_buckets, per = 4, 3 * 20000
    rng = np.random.default_rng(40 + dtype)
    xs = [NP.from_f32((rng.standard_normal(per) * 1e-2).astype(np.float32), dtype) for _ in range(n_buckets)]
    flats = [dev(x, dtype) for x in xs]
    buckets, tensors = [], []
    for b, f in enumerate(flats):
        ts = [bc.BaguaTensorPy(t, f"h{dtype}.{b}.{i}") for i, t in enumerate(f.view(3, -1).unbind(0))]
        bk = bc.BaguaBucketPy(f"half{b}", ts)
        bk.append_centralized_synchronous_op(comm, None, False, True, False, "MinMaxUInt8")
        buckets.append(bk)
        tensors.append(ts)
    backend = bc.BaguaCommBackendPy(4, 0)
    backend.register_ordered_buckets(buckets)
    ev = torch.cuda.Event()
    ev.record()
    for ts in tensors:
        for t in ts:
            backend.mark_communication_ready(t, ev.cuda_event)
    assert backend.wait_pending_comm_ops() == n_buckets
    for b in range(n_buckets):
        want = simulate.centralized_low_precision(oracle_c, [xs[b].copy()], dtype, True)[0]
        assert np.array_equal(host(flats[b], dtype).view(np.uint8), want.view(np.uint8)), f"bucket {b}"
