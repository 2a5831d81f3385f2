"""Ranks that post different collectives fail instead of crashing or hanging.

The comm ops are correct only while every rank posts the same collectives in the
same order (centralized_low_precision_synchronous.rs:30-71 is the sequence every
rank runs).  Three layers guard that here, tested on the in-process loopback
transport (csrc/runtime/loopback.cpp; the RCCL side is in test_gpu_rccl_procs.py):

  * the loopback transport compares every rank's collective (kind, bytes, root,
    op, sequence number) and every send/recv pair's sizes after its barrier: a
    mismatch is BAGUA_ERR_COMM on every rank, not an out-of-bounds copy;
  * the schedule switches (BAGUA_PIPELINE_*, BAGUA_RING_MULTIPATH,
    BAGUA_CHECK_SCHEDULE) are read once, when the communicators are created;
  * BAGUA_CHECK_SCHEDULE=1 makes the ranks allgather an op descriptor before the
    op's first collective: any difference is BAGUA_ERR_INVALID_ARG on every rank,
    before any data moves.

And a stuck op (a peer that never arrives) is failed by the scheduler's monitor
(lib.rs:255-265) after its limit, instead of blocking wait_pending_comm_ops."""
import ctypes
import time

import numpy as np
import pytest
import torch

from oracle import simulate
from test_gpu_multirank import host, run_ranks

pytestmark = pytest.mark.gpu

F32 = 0
ERR_INVALID_ARG, ERR_COMM = 1, 16


@pytest.fixture(scope="module")
def bc():
    import bagua_core
    return bagua_core


def _inputs(p, n, seed):
    rng = np.random.default_rng(seed)
    return [(rng.standard_normal(n) * 1e-3 + 1e-4 * r).astype(np.float32) for r in range(p)]


def _run_each(p, fn):
    """fn(r) -> status on every rank (threads), the statuses in rank order"""
    rcs = [None] * p

    def rank(r):
        rcs[r] = fn(r)

    run_ranks(rank, p)
    return rcs


@pytest.mark.parametrize("check", [False, True])
def test_different_piece_counts(bc, oracle_c, monkeypatch, check):
    """rank 0 pipelines with 4 pieces, rank 1 with 2: every rank fails (transport check:
    the first grouped send/recv sizes differ; descriptor check: the schedules differ,
    nothing is posted), the process lives, tensors are untouched (the pipelined op writes
    them only after the exchange), and the same communicators then run a matching op that
    equals the oracle."""
    if check:
        monkeypatch.setenv("BAGUA_CHECK_SCHEDULE", "1")
    from bagua_core.communicator import loopback_communicators
    p, cs = 2, 4 * 16384
    xs = _inputs(p, p * cs, 11)
    comms = loopback_communicators(p, 0)
    ts = [torch.from_numpy(x.copy()).cuda() for x in xs]
    torch.cuda.synchronize()
    N = bc._native
    raws = [bc.BaguaTensorPy(t, "g").raw() for t in ts]
    op = N.C.bagua_centralized_low_precision_pipelined
    rcs = _run_each(p, lambda r: op(comms[r].handle, ctypes.byref(raws[r]), 1, N.COMPRESSION_MINMAX_UINT8,
                                    4 if r == 0 else 2))
    assert rcs == [ERR_INVALID_ARG if check else ERR_COMM] * p, rcs
    for r in range(p):
        assert np.array_equal(host(ts[r], F32), xs[r]), f"rank {r} changed"
    rcs = _run_each(p, lambda r: op(comms[r].handle, ctypes.byref(raws[r]), 1, N.COMPRESSION_MINMAX_UINT8, 3))
    assert rcs == [0] * p, rcs
    want = simulate.centralized_low_precision(oracle_c, xs, F32, True)
    for r in range(p):
        assert np.array_equal(host(ts[r], F32).view(np.uint8), want[r].view(np.uint8)), f"rank {r}"


@pytest.mark.parametrize("check", [False, True])
def test_ring_op_against_centralized_op(bc, monkeypatch, check):
    """rank 0 runs the ring (decentralized) op, rank 1 the centralized one: every rank fails
    (grouped send/recv against an alltoall; with the check, the op field differs)."""
    if check:
        monkeypatch.setenv("BAGUA_CHECK_SCHEDULE", "1")
    from bagua_core.communicator import loopback_communicators
    p, n = 2, 2 * 30000
    xs = _inputs(p, n, 12)
    comms = loopback_communicators(p, 0)
    ts = {k: [torch.from_numpy(x.copy()).cuda() for x in xs] for k in "twlr"}
    torch.cuda.synchronize()
    N = bc._native

    def fn(r):
        raws = [bc.BaguaTensorPy(ts[k][r], k).raw() for k in "twlr"]
        if r == 0:
            return N.C.bagua_decentralized_low_precision_synchronous(comms[r].handle, *[ctypes.byref(x) for x in raws],
                                                                     N.COMPRESSION_MINMAX_UINT8)
        return N.C.bagua_centralized_low_precision_synchronous(comms[r].handle, ctypes.byref(raws[0]), 1,
                                                               N.COMPRESSION_MINMAX_UINT8)

    rcs = _run_each(p, fn)
    assert rcs == [ERR_INVALID_ARG if check else ERR_COMM] * p, rcs
    if check:  # nothing ran: every tensor is untouched
        for k in "twlr":
            for r in range(p):
                assert np.array_equal(host(ts[k][r], F32), xs[r]), (k, r)


def test_check_on_matching_ops_is_transparent(bc, oracle_c, monkeypatch):
    """With the descriptor check on, matching ops of every kind still equal the oracle."""
    monkeypatch.setenv("BAGUA_CHECK_SCHEDULE", "1")
    from bagua_core.communicator import loopback_communicators
    p, cs = 4, 8192
    xs = _inputs(p, p * cs, 13)
    want = simulate.centralized_low_precision(oracle_c, xs, F32, True)
    want1 = simulate.centralized_low_precision(oracle_c, xs, F32, True, method="OneBitSignScale")
    comms = loopback_communicators(p, 0)
    N = bc._native
    for method, fn, w in ((N.COMPRESSION_MINMAX_UINT8, N.C.bagua_centralized_low_precision_synchronous, want),
                          (N.COMPRESSION_MINMAX_UINT8, N.C.bagua_centralized_low_precision_synchronous_unfused, want),
                          (N.COMPRESSION_ONEBIT, N.C.bagua_centralized_low_precision_synchronous, want1)):
        ts = [torch.from_numpy(x.copy()).cuda() for x in xs]
        torch.cuda.synchronize()
        raws = [bc.BaguaTensorPy(t, "g").raw() for t in ts]
        rcs = _run_each(p, lambda r: fn(comms[r].handle, ctypes.byref(raws[r]), 1, method))
        assert rcs == [0] * p, rcs
        for r in range(p):
            assert np.array_equal(host(ts[r], F32).view(np.uint8), w[r].view(np.uint8)), (fn, r)


def test_schedule_env_is_read_at_creation(bc, oracle_c, monkeypatch):
    """The schedule switches are fixed when a communicator is created: changing the
    environment afterwards changes nothing for existing communicators (an op that read it
    per rank per op could post a different schedule than its peers), while new ones see it;
    ops on the existing ones still equal the oracle."""
    from bagua_core.communicator import loopback_communicators
    for k in ("BAGUA_PIPELINE_TAPER", "BAGUA_PIPELINE_PIECES", "BAGUA_PIPELINE_MIN_PIECE", "BAGUA_RING_MULTIPATH",
              "BAGUA_CHECK_SCHEDULE"):
        monkeypatch.delenv(k, raising=False)
    p, cs = 2, 6 * 16384
    xs = _inputs(p, p * cs, 14)
    want = simulate.centralized_low_precision(oracle_c, xs, F32, True)
    comms = loopback_communicators(p, 0)
    # taper -1: the op's automatic piece schedules are tapered (round 6 default)
    default = {"pieces_cap": 4, "min_piece": 1 << 20, "taper": -1, "multipath": 0, "check": 0}
    assert [c.schedule_config() for c in comms] == [default] * p
    monkeypatch.setenv("BAGUA_PIPELINE_TAPER", "1")
    monkeypatch.setenv("BAGUA_PIPELINE_PIECES", "8")
    monkeypatch.setenv("BAGUA_RING_MULTIPATH", "1")
    monkeypatch.setenv("BAGUA_CHECK_SCHEDULE", "1")
    assert [c.schedule_config() for c in comms] == [default] * p
    fresh = loopback_communicators(p, 0)
    assert fresh[1].schedule_config() == {"pieces_cap": 8, "min_piece": 1 << 20, "taper": 1, "multipath": 1,
                                          "check": 1}
    ts = [torch.from_numpy(x.copy()).cuda() for x in xs]
    torch.cuda.synchronize()
    N = bc._native
    raws = [bc.BaguaTensorPy(t, "g").raw() for t in ts]
    rcs = _run_each(p, lambda r: N.C.bagua_centralized_low_precision_pipelined(
        comms[r].handle, ctypes.byref(raws[r]), 1, N.COMPRESSION_MINMAX_UINT8, 5))
    assert rcs == [0] * p
    for r in range(p):
        assert np.array_equal(host(ts[r], F32).view(np.uint8), want[r].view(np.uint8)), r


def test_stuck_op_fails_within_limit(bc):
    """lib.rs:255-265: a scheduler whose op waits for a peer that never comes (rank 1 of the
    loopback group never posts) fails it after the limit: the monitor aborts the
    communicator, wait_pending_comm_ops raises with the monitor's message within the limit
    plus a margin, and the backend is destroyed without hanging."""
    from bagua_core.communicator import loopback_communicators
    comms = loopback_communicators(2, 0)
    x = torch.randn(2 * 65536, device="cuda") * 1e-3
    torch.cuda.synchronize()
    bk = bc.BaguaBucketPy("lonely", [bc.BaguaTensorPy(x, "x")])
    bk.append_centralized_synchronous_op(comms[0], None, False, True, False, "MinMaxUInt8")
    backend = bc.BaguaCommBackendPy(1, 0)
    limit = 2.0
    backend.set_op_timeout(limit)
    backend.register_ordered_buckets([bk])
    ev = torch.cuda.Event()
    ev.record()
    t0 = time.time()
    backend.mark_communication_ready(bk.tensors()[0], ev.cuda_event)
    with pytest.raises(RuntimeError, match="has not finished for 2 s"):
        backend.wait_pending_comm_ops()
    elapsed = time.time() - t0
    assert limit <= elapsed < limit + 10, elapsed
    assert len(backend.failures()) == 1 and "lonely" in backend.failures()[0]
    assert comms[0].check_abort()
    t1 = time.time()
    del backend
    assert time.time() - t1 < 10


def test_stuck_op_never_released(bc, monkeypatch):
    """a transport whose blocked call never returns after the abort
    (BAGUA_LOOPBACK_ABORT_HOLD_S: the loopback rank keeps waiting 20 s).  The op is failed
    at the limit, wait_pending_comm_ops raises once the op is abandoned (10 s after the
    abort), the backend reports it stuck and keeps the retired ops' references, and
    destroying the backend leaves the stuck worker behind instead of joining it.  The
    communicators outlive the hold, so the worker returns into live objects."""
    from bagua_core import backend as backend_mod
    from bagua_core.communicator import loopback_communicators
    monkeypatch.setenv("BAGUA_LOOPBACK_ABORT_HOLD_S", "20")
    comms = loopback_communicators(2, 0)
    x = torch.randn(2 * 65536, device="cuda") * 1e-3
    torch.cuda.synchronize()
    bk = bc.BaguaBucketPy("held", [bc.BaguaTensorPy(x, "x")])
    bk.append_centralized_synchronous_op(comms[0], None, False, True, False, "MinMaxUInt8")
    backend = bc.BaguaCommBackendPy(1, 0)
    backend.set_op_timeout(1.0)
    backend.register_ordered_buckets([bk])
    bk.clear_ops()  # its op is retired while scheduled: must stay referenced while stuck
    bk.append_centralized_synchronous_op(comms[0], None, False, True, False, "MinMaxUInt8")
    ev = torch.cuda.Event()
    ev.record()
    t0 = time.time()
    backend.mark_communication_ready(bk.tensors()[0], ev.cuda_event)
    with pytest.raises(RuntimeError, match="has not finished for 1 s"):
        backend.wait_pending_comm_ops()
    assert 1.0 + 10.0 <= time.time() - t0 < 20.0
    N = bc._native
    assert N.C.bagua_comm_backend_stuck(backend._handle) == 1
    assert bk._retired, "the retired op must stay referenced while its call is stuck"
    t1 = time.time()
    del backend
    assert time.time() - t1 < 5
    assert backend_mod._ABANDONED and backend_mod._ABANDONED[-1][0] is bk
    time.sleep(max(0.0, 20.0 + 3.0 - (time.time() - t0)))  # the held call has returned
    backend_mod._ABANDONED.clear()
