"""GPU tests of the comm ops through RCCL on a single-rank communicator
(the GPU box has one MI355X; multi-rank semantics are covered on CPU with
gloo in tests/test_distributed_sim.py and by construction), and of the
bucket / scheduler surface.  Results are compared bit-exact with the oracle
simulation of the reference op sequence (oracle/simulate.py)."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import oracle_np as NP
from oracle import simulate

pytestmark = pytest.mark.gpu

F32, F16, BF16 = 0, 1, 2
TORCH = {F32: torch.float32, F16: torch.float16, BF16: torch.bfloat16}
STORAGE = {F32: np.float32, F16: np.float16, BF16: np.uint16}


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


def dev(x, dtype):
    if dtype == BF16:
        return torch.from_numpy(x.view(np.int16).copy()).view(torch.bfloat16).cuda()
    return torch.from_numpy(x.copy()).cuda()


def host(t, dtype):
    torch.cuda.synchronize()
    if dtype == BF16:
        return t.view(torch.int16).cpu().numpy().view(np.uint16)
    return t.cpu().numpy()


def test_communicator_basics(bc, comm):
    assert comm.nranks() == 1 and comm.rank() == 0
    assert not comm.check_abort()
    uid = bc.BaguaSingleCommunicatorPy.generate_nccl_unique_id_str()
    import base64
    assert len(base64.b64decode(uid)) == 128  # communicators/mod.rs:226-240
    t = torch.arange(16, dtype=torch.float32, device="cuda")
    bt = bc.BaguaTensorPy(t, "t")
    comm.allreduce_inplace(bt, 0)
    comm.allgather_inplace(bt)
    comm.alltoall_inplace(bt)
    comm.barrier()
    assert torch.equal(t.cpu(), torch.arange(16, dtype=torch.float32))


@pytest.mark.parametrize("dtype", [F32, BF16, F16])
@pytest.mark.parametrize("fused", [True, False])
def test_centralized_low_precision_p1(bc, comm, oracle_c, dtype, fused):
    """Config 1 (loopback, p = 1) on the GPU through RCCL: bit-exact with the reference sequence."""
    rng = np.random.default_rng(21 + dtype)
    x = NP.from_f32((rng.standard_normal(1 << 18) * 1e-3).astype(np.float32), dtype)
    want = simulate.centralized_low_precision(oracle_c, [x], dtype, True)[0]
    t = dev(x, dtype)
    b = bc.BaguaBucketPy("b", [bc.BaguaTensorPy(t, "t")])
    from bagua_core.bucket import CentralizedLowPrecisionSynchronous
    b._append(CentralizedLowPrecisionSynchronous(comm, True, "MinMaxUInt8", fused))
    b.execute_ops()
    assert np.array_equal(host(t, dtype).view(np.uint8), want.view(np.uint8))


def test_full_precision_p1(bc, comm):
    t = torch.randn(4096, device="cuda")
    ref = t.clone()
    b = bc.BaguaBucketPy("b", [bc.BaguaTensorPy(t, "t")])
    b.append_centralized_synchronous_op(comm, None, False, True, False, None)
    b.execute_ops()
    assert torch.equal(t, ref)


@pytest.mark.parametrize("dtype", [F32, BF16])
def test_decentralized_low_precision_p1(bc, comm, oracle_c, dtype):
    rng = np.random.default_rng(31 + dtype)
    n = 100003
    arrs = [NP.from_f32((rng.standard_normal(n) * 1e-3).astype(np.float32), dtype) for _ in range(4)]
    want = simulate.decentralized_low_precision(oracle_c, [arrs[0]], [arrs[1]], [arrs[2]], [arrs[3]], dtype)
    ts = [dev(a, dtype) for a in arrs]
    bt = [bc.BaguaTensorPy(x, nm) for x, nm in zip(ts, ["t", "w", "l", "r"])]
    b = bc.BaguaBucketPy("b", [bt[0]])
    b.append_low_precision_decentralized_synchronous_op(comm, None, False, "ring", "MinMaxUInt8", bt[1], bt[2], bt[3])
    b.execute_ops()
    for got, w in zip(ts, want):
        assert np.array_equal(host(got, dtype).view(np.uint8), w[0].view(np.uint8))


def test_backend_schedules_noncontiguous_bucket(bc, comm, oracle_c):
    """Two non-adjacent tensors in one bucket: flattened, reduced, copied back
    (datatypes/mod.rs:963-1070), driven by BaguaCommBackendPy readiness."""
    rng = np.random.default_rng(41)
    a = (rng.standard_normal(3000) * 1e-3).astype(np.float32)
    c = (rng.standard_normal(5000) * 1e-3).astype(np.float32)
    want = simulate.centralized_low_precision(oracle_c, [np.concatenate([a, c])], F32, True)[0]
    ta, tc = dev(a, F32), dev(c, F32)
    _gap = torch.empty(1000, device="cuda")  # keep the two allocations apart
    ba, bc_ = bc.BaguaTensorPy(ta, "a"), bc.BaguaTensorPy(tc, "c")
    bucket = bc.BaguaBucketPy("bucket0", [ba, bc_])
    bucket.append_centralized_synchronous_op(comm, None, False, True, False, "MinMaxUInt8")
    backend = bc.BaguaCommBackendPy(10, 0)
    backend.register_ordered_buckets([bucket])
    ev = torch.cuda.Event()
    ev.record()
    backend.mark_communication_ready(ba, ev.cuda_event)
    assert backend.wait_pending_comm_ops() == 0  # not ready until every tensor is
    backend.mark_communication_ready(bc_, 0)
    assert backend.wait_pending_comm_ops() == 1
    got = np.concatenate([host(ta, F32), host(tc, F32)])
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    with pytest.raises(RuntimeError):
        backend.register_ordered_buckets([bucket, bc.BaguaBucketPy("dup", [ba])])
    del _gap


def test_pool_reuse(bc):
    N = bc._native
    import ctypes
    p1 = ctypes.c_uint64()
    assert N.C.bagua_pool_alloc(0, 1 << 20, ctypes.byref(p1)) == 0
    assert N.C.bagua_pool_free(p1.value) == 0
    p2 = ctypes.c_uint64()
    assert N.C.bagua_pool_alloc(0, (1 << 20) - 100, ctypes.byref(p2)) == 0
    assert p2.value == p1.value  # same size class -> block reused
    assert N.C.bagua_pool_free(p2.value) == 0
    assert N.C.bagua_pool_free(12345) != 0


@pytest.mark.parametrize("method", ["MinMaxUInt8", "OneBit"])
def test_op_captured_into_a_hip_graph(bc, comm, oracle_c, method):
    """The compressed centralized op (async mode) captured into a HIP graph between
    bagua_pool_capture_begin/end: the graph owns the op's pool blocks, every replay
    on new data equals the eager op bit-for-bit, and the arena gives the blocks back
    once the graph is gone."""
    N = bc._native
    code = N.COMPRESSION_MINMAX_UINT8 if method == "MinMaxUInt8" else N.COMPRESSION_ONEBIT
    assert N.C.bagua_comm_set_async(comm.handle, 1) == 0
    try:
        n = 3 * 65536
        rng = np.random.default_rng(77)
        xs = [(rng.standard_normal(n) * 1e-3).astype(np.float32) for _ in range(3)]
        t = torch.zeros(n, device="cuda")
        raw = bc.BaguaTensorPy(t, "g").raw()

        def op():
            N.check(N.C.bagua_centralized_low_precision_synchronous(comm.handle, ctypes.byref(raw), 1, code), "op")

        want = []
        for x in xs:  # eager results (and a warm pool)
            t.copy_(torch.from_numpy(x))
            op()
            comm.synchronize()
            want.append(t.cpu().numpy().copy())
        stream = comm._keep_stream
        in_use = N.C.bagua_pool_bytes_in_use(0)
        g = torch.cuda.CUDAGraph()
        arena = N.C.bagua_pool_capture_begin()
        assert arena
        try:
            with torch.cuda.graph(g, stream=stream, capture_error_mode="relaxed"):
                op()
        finally:
            assert N.C.bagua_pool_capture_end(arena) == 0
        held = N.C.bagua_pool_bytes_in_use(0) - in_use
        # compressed buffers would stay with the graph; the op at one rank has none (MinMax:
        # the min/max pass + one table pass over the tensor, bagua_minmax_u8_centralized_one_rank;
        # 1-bit: encode, scales, +-scale2 pass on the stream's workspace,
        # bagua_onebit_centralized_one_rank)
        assert held >= 0 and (held > 0 or comm.nranks() == 1)
        for x, w in zip(reversed(xs), reversed(want)):
            t.copy_(torch.from_numpy(x))
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            assert np.array_equal(t.cpu().numpy().view(np.uint32), w.view(np.uint32))
        del g
        torch.cuda.synchronize()
        assert N.C.bagua_pool_capture_release(arena) == 0
        assert N.C.bagua_pool_bytes_in_use(0) == in_use
    finally:
        assert N.C.bagua_comm_set_async(comm.handle, 0) == 0


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("unfused", [False, True])
def test_decentralized_p1_reads_its_own_bytes(bc, comm, oracle_c, dtype, unfused):
    """One rank is its own left and right peer: the op reads its own payload in
    place of the self send/recv (decentralized_low_precision_synchronous.rs:98-115
    would deliver exactly those bytes), fused and reference sequence alike."""
    N = bc._native
    rng = np.random.default_rng(57 + dtype + 2 * unfused)
    n = 1 << 16
    arrs = [NP.from_f32((rng.standard_normal(n) * 1e-3).astype(np.float32), dtype) for _ in range(4)]
    want = simulate.decentralized_low_precision(oracle_c, [arrs[0]], [arrs[1]], [arrs[2]], [arrs[3]], dtype)
    ts = [dev(a, dtype) for a in arrs]
    raws = [bc.BaguaTensorPy(x, nm).raw() for x, nm in zip(ts, "twlr")]
    torch.cuda.synchronize()
    fn = (N.C.bagua_decentralized_low_precision_synchronous_unfused if unfused
          else N.C.bagua_decentralized_low_precision_synchronous)
    N.check(fn(comm.handle, *[ctypes.byref(r) for r in raws], N.COMPRESSION_MINMAX_UINT8), "ring op")
    comm.synchronize()
    for got, w in zip(ts, want):
        assert np.array_equal(host(got, dtype).view(np.uint8), w[0].view(np.uint8))
