"""GPU tests of hierarchical mode (communicators/mod.rs:243-427): every rank of a
node reduces (AVG, or SUM for a summing centralized op) into the node leader
(intranode rank 0), the leaders run the op on the internode communicator, and
the leader broadcasts the result over its node.  This is how upstream Bagua's
ByteGrad drives the compressed op by default.

Nodes are emulated with the loopback transport on one device: 2 nodes x 2 ranks
(and 1 node x 4 ranks), one host thread per rank; the leader's intranode and
internode communicators share its stream, as the reference requires
(:250-256).  The loopback reduce sums in rank order, so the node average is
((x0 + x1) + ...) / n in f32 and every rank's result is checked bit-for-bit
against the oracle's simulation of the leaders' op on those averages."""
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


class _Group:
    def __init__(self, N, p):
        self.N = N
        self.h = N.C.bagua_loopback_group_create(p, 0)
        assert self.h

    def __del__(self):
        self.N.C.bagua_loopback_group_destroy(self.h)


def _comm(bc, group, rank, p, stream):
    h = bc._native.C.bagua_loopback_communicator_create(group.h, rank, stream.cuda_stream)
    assert h
    return bc.BaguaSingleCommunicatorPy._from_handle(h, rank, p, 0, stream.cuda_stream, keep=(group, stream))


def _topology(bc, nodes, per_node):
    """(intranode, internode or None) communicators per global rank; ranks of node k are
    k * per_node + i, the leader is i = 0."""
    N = bc._native
    streams = [torch.cuda.Stream() for _ in range(nodes * per_node)]
    intra_groups = [_Group(N, per_node) for _ in range(nodes)]
    inter_group = _Group(N, nodes)
    out = []
    for g in range(nodes * per_node):
        k, i = divmod(g, per_node)
        intra = _comm(bc, intra_groups[k], i, per_node, streams[g])
        inter = _comm(bc, inter_group, k, nodes, streams[g]) if i == 0 else None
        out.append((intra, inter))
    return out


def _run(p, fn):
    errs = [None] * p

    def wrap(r):
        try:
            fn(r)
        except BaseException as e:  # noqa: BLE001
            errs[r] = e
    ths = [threading.Thread(target=wrap, args=(r,)) for r in range(p)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    for e in errs:
        if e is not None:
            raise e


def _node_reduce(xs, average):
    acc = xs[0].copy()
    for x in xs[1:]:
        acc = (acc + x).astype(np.float32)
    if average:
        acc = (acc / np.float32(len(xs))).astype(np.float32)
    return acc


@pytest.mark.parametrize("nodes,per_node", [(2, 2), (1, 4), (2, 3)])
@pytest.mark.parametrize("average", [True, False])
@pytest.mark.parametrize("method", ["MinMaxUInt8", "OneBitSignScale"])
def test_centralized_hierarchical(bc, oracle_c, nodes, per_node, average, method):
    N = bc._native
    code = N.COMPRESSION_MINMAX_UINT8 if method == "MinMaxUInt8" else N.COMPRESSION_ONEBIT
    p = nodes * per_node
    n = 3 * 4096 * nodes
    rng = np.random.default_rng(11 * p + average)
    xs = [(rng.standard_normal(n) * 1e-3).astype(np.float32) for _ in range(p)]
    comms = _topology(bc, nodes, per_node)
    ts = [torch.from_numpy(x.copy()).cuda() for x in xs]
    torch.cuda.synchronize()

    def rank(g):
        intra, inter = comms[g]
        raw = bc.BaguaTensorPy(ts[g], "g").raw()
        N.check(N.C.bagua_centralized_low_precision_hierarchical(
            intra.handle, inter.handle if inter is not None else None, ctypes.byref(raw), int(average), code),
            "hierarchical op")
    _run(p, rank)
    node_vals = [_node_reduce(xs[k * per_node:(k + 1) * per_node], average) for k in range(nodes)]
    want = simulate.centralized_low_precision(oracle_c, node_vals, F32, average,
                                              method="MinMaxUInt8" if method == "MinMaxUInt8" else "OneBit")
    for g in range(p):
        got = ts[g].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want[g // per_node].view(np.uint32)), g


def test_decentralized_hierarchical(bc, oracle_c):
    """The ring op among the node leaders on the node averages (the node always
    averages, decentralized_low_precision_synchronous.rs:37-41); the workers receive
    their leader's t."""
    N = bc._native
    nodes, per_node = 3, 2
    p = nodes * per_node
    n = 8 * 1000
    rng = np.random.default_rng(5)
    xs = [(rng.standard_normal(n) * 1e-3).astype(np.float32) for _ in range(p)]
    w, l, r = ([(rng.standard_normal(n) * 1e-3).astype(np.float32) for _ in range(nodes)] for _ in range(3))
    comms = _topology(bc, nodes, per_node)
    ts = [torch.from_numpy(x.copy()).cuda() for x in xs]
    st = {k: [torch.from_numpy(a[k].copy()).cuda() for a in (w, l, r)] for k in range(nodes)}
    torch.cuda.synchronize()

    def rank(g):
        intra, inter = comms[g]
        k, i = divmod(g, per_node)
        raws = [bc.BaguaTensorPy(ts[g], "t").raw()]
        # the node's ring state: only its leader runs the ring op and updates it
        raws += [bc.BaguaTensorPy(v, nm).raw() for v, nm in zip(st[k], "wlr")]
        N.check(N.C.bagua_decentralized_low_precision_hierarchical(
            intra.handle, inter.handle if inter is not None else None, *[ctypes.byref(x) for x in raws],
            N.COMPRESSION_MINMAX_UINT8), "hierarchical ring op")
    _run(p, rank)
    node_vals = [_node_reduce(xs[k * per_node:(k + 1) * per_node], True) for k in range(nodes)]
    t2, w2, l2, r2 = simulate.decentralized_low_precision(oracle_c, node_vals, w, l, r, F32)
    for g in range(p):
        k = g // per_node
        assert np.array_equal(ts[g].cpu().numpy().view(np.uint32), t2[k].view(np.uint32)), g
    for k in range(nodes):
        for got, want in zip(st[k], (w2[k], l2[k], r2[k])):
            assert np.array_equal(got.cpu().numpy().view(np.uint32), want.view(np.uint32)), k


def test_bucket_api_hierarchical(bc, oracle_c):
    """BaguaBucketPy.append_centralized_synchronous_op(..., hierarchical=True) as
    ByteGrad calls it (scattergather=True, compression="MinMaxUInt8"), executed on
    every rank: a worker passes no internode communicator."""
    nodes, per_node = 2, 2
    p = nodes * per_node
    n = 3 * 8192
    rng = np.random.default_rng(21)
    xs = [(rng.standard_normal(n) * 1e-3).astype(np.float32) for _ in range(p)]
    comms = _topology(bc, nodes, per_node)
    flats = [torch.from_numpy(x.copy()).cuda() for x in xs]
    buckets = []
    for g in range(p):
        intra, inter = comms[g]
        ts = [bc.BaguaTensorPy(v, f"t{i}") for i, v in enumerate(flats[g].view(3, -1).unbind(0))]
        bk = bc.BaguaBucketPy("b", ts)
        bk.append_centralized_synchronous_op(inter, intra, True, True, True, "MinMaxUInt8")
        buckets.append(bk)
    torch.cuda.synchronize()
    _run(p, lambda g: buckets[g].execute_ops())
    node_vals = [_node_reduce(xs[k * per_node:(k + 1) * per_node], True) for k in range(nodes)]
    want = simulate.centralized_low_precision(oracle_c, node_vals, F32, True)
    for g in range(p):
        assert np.array_equal(flats[g].cpu().numpy().view(np.uint32), want[g // per_node].view(np.uint32)), g
    with pytest.raises(RuntimeError, match="intra node communicator must be given"):
        bc.BaguaBucketPy("c", [bc.BaguaTensorPy(flats[0], "z")]).append_centralized_synchronous_op(
            comms[0][1], None, True, True, False, "MinMaxUInt8")


def test_hierarchical_single_rank_rccl(bc, oracle_c):
    """One node of one rank over RCCL: intranode and internode communicators on one
    stream; the reduce and broadcast are identities and the result is the op's."""
    N = bc._native
    stream = torch.cuda.Stream()
    mk = lambda: bc.BaguaSingleCommunicatorPy(0, 1, 0, stream.cuda_stream,  # noqa: E731
                                               bc.BaguaSingleCommunicatorPy.generate_nccl_unique_id_str())
    intra, inter = mk(), mk()
    n = 3 * 65536
    x = (np.random.default_rng(3).standard_normal(n) * 1e-3).astype(np.float32)
    t = torch.from_numpy(x.copy()).cuda()
    raw = bc.BaguaTensorPy(t, "g").raw()
    torch.cuda.synchronize()
    N.check(N.C.bagua_centralized_low_precision_hierarchical(intra.handle, inter.handle, ctypes.byref(raw), 1,
                                                             N.COMPRESSION_MINMAX_UINT8), "op")
    want = simulate.centralized_low_precision(oracle_c, [x], F32, True)[0]
    assert np.array_equal(t.cpu().numpy().view(np.uint32), want.view(np.uint32))
    # a leader whose communicators do not share a stream is refused (:356-360)
    other = bc.BaguaSingleCommunicatorPy(0, 1, 0, torch.cuda.Stream().cuda_stream,
                                         bc.BaguaSingleCommunicatorPy.generate_nccl_unique_id_str())
    assert N.C.bagua_centralized_low_precision_hierarchical(intra.handle, other.handle, ctypes.byref(raw), 1,
                                                            N.COMPRESSION_MINMAX_UINT8) != 0
