"""GPU tests of the comm ops at p > 1 on a single MI355X.

The C++ comm ops (csrc/runtime/comm_ops.cpp) run unchanged on the in-process
loopback transport: p virtual ranks, one host thread each, on one device,
collectives as device-to-device copies (csrc/runtime/loopback.cpp).  Every
rank's result must equal the oracle simulation of the reference op sequence
bit-for-bit (and, for the centralized op, all ranks must agree)."""
import ctypes
import threading

import numpy as np
import pytest
import torch

from oracle import oracle_np as NP
from oracle import simulate

pytestmark = pytest.mark.gpu

F32, F16, BF16 = 0, 1, 2
TORCH = {F32: torch.float32, F16: torch.float16, BF16: torch.bfloat16}


@pytest.fixture(scope="module")
def bc():
    import bagua_core
    return bagua_core


def dev(x, dtype):
    if dtype == BF16:
        return torch.from_numpy(x.view(np.int16).copy()).view(torch.bfloat16).cuda()
    return torch.from_numpy(x.copy()).cuda()


def host(t, dtype):
    torch.cuda.synchronize()
    if dtype == BF16:
        return t.view(torch.int16).cpu().numpy().view(np.uint16)
    return t.cpu().numpy()


def run_ranks(fn, p):
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
        t.join(timeout=300)
    for e in errs:
        if e is not None:
            raise e


@pytest.mark.parametrize("p,dtype,cs,fused", [(2, F32, 40000, True), (4, F32, 65536, True), (8, F32, 12345 * 4, True),
                                              (8, BF16, 20000, True), (4, F16, 8192, True), (4, F32, 10000, False),
                                              (3, F32, 3 * 1024, True), (16, F32, 4096, True)])
def test_centralized_low_precision_multirank(bc, oracle_c, p, dtype, cs, fused):
    from bagua_core.communicator import loopback_communicators
    if oracle_c.minmax_compressed_size(p, cs, dtype) % p:
        pytest.skip("reference alltoall requires S % nranks == 0")
    rng = np.random.default_rng(p * 100 + dtype)
    xs = [NP.from_f32((rng.standard_normal(p * cs) * 1e-3 + 0.01 * r).astype(np.float32), dtype) for r in range(p)]
    want = simulate.centralized_low_precision(oracle_c, xs, dtype, True)
    comms = loopback_communicators(p, 0)
    ts = [dev(x, dtype) for x in xs]
    torch.cuda.synchronize()
    N = bc._native
    fn = (N.C.bagua_centralized_low_precision_synchronous if fused
          else N.C.bagua_centralized_low_precision_synchronous_unfused)

    def rank(r):
        raw = bc.BaguaTensorPy(ts[r], f"g{r}").raw()
        N.check(fn(comms[r].handle, ctypes.byref(raw), 1, N.COMPRESSION_MINMAX_UINT8), f"rank {r}")

    run_ranks(rank, p)
    outs = [host(t, dtype) for t in ts]
    for r in range(p):
        assert np.array_equal(outs[r].view(np.uint8), want[r].view(np.uint8)), f"rank {r}"
        assert np.array_equal(outs[r].view(np.uint8), outs[0].view(np.uint8))


@pytest.mark.parametrize("p,dtype,cs,pieces", [(2, F32, 40000, 3), (4, F32, 65536, 4), (8, F32, 12345 * 4, 2),
                                               (8, BF16, 20000, 5), (4, F16, 8192, 2), (4, F32, 1536, 4),
                                               (1, F32, 70000, 3), (16, F32, 4096 * 3, 3), (3, F32, 3 * 1024, 4),
                                               (2, F32, (1 << 21) + 1024, 0)])
@pytest.mark.parametrize("taper", ["0", "1", None])
def test_centralized_pipelined_multirank(bc, oracle_c, p, dtype, cs, pieces, taper, monkeypatch):
    """Pieced op (side-stream exchange per piece) == the reference sequence, bit-for-bit.
    (4, F32, 1536, 4) has an empty trailing piece (pieces are 512-element aligned).
    taper: first and last piece half size (BAGUA_PIPELINE_TAPER: 0 never, 1 every count,
    unset -- the default -- the automatic schedules (pieces = 0) only)."""
    if taper is None:
        monkeypatch.delenv("BAGUA_PIPELINE_TAPER", raising=False)
    else:
        monkeypatch.setenv("BAGUA_PIPELINE_TAPER", taper)
    from bagua_core.communicator import loopback_communicators
    if oracle_c.minmax_compressed_size(p, cs, dtype) % p:
        pytest.skip("reference alltoall requires S % nranks == 0")
    rng = np.random.default_rng(p * 1000 + dtype + cs)
    xs = [NP.from_f32((rng.standard_normal(p * cs) * 1e-3 - 0.02 * r).astype(np.float32), dtype) for r in range(p)]
    want = simulate.centralized_low_precision(oracle_c, xs, dtype, True)
    comms = loopback_communicators(p, 0)
    ts = [dev(x, dtype) for x in xs]
    torch.cuda.synchronize()
    N = bc._native

    def rank(r):
        raw = bc.BaguaTensorPy(ts[r], f"g{r}").raw()
        N.check(N.C.bagua_centralized_low_precision_pipelined(comms[r].handle, ctypes.byref(raw), 1,
                                                              N.COMPRESSION_MINMAX_UINT8, pieces), f"rank {r}")

    run_ranks(rank, p)
    for r in range(p):
        assert np.array_equal(host(ts[r], dtype).view(np.uint8), want[r].view(np.uint8)), f"rank {r}"


@pytest.mark.parametrize("p,dtype,cs,pieces", [(2, F32, 40000, 3), (2, BF16, 30000, 4), (2, F16, 8192 + 512, 2),
                                               (4, F32, 65536, 4), (8, F32, 12345 * 4, 2)])
@pytest.mark.parametrize("recompute", ["0", "1"])
def test_centralized_pipelined_middle_variants(bc, oracle_c, p, dtype, cs, pieces, recompute, monkeypatch):
    """Both middle steps of the pieced op, forced (BAGUA_PIPE_RECOMPUTE): the storing pair
    (reduce pieces store the reduced chunk, the requantise reads it) and the recompute pair
    (partials-only reduce pieces, the requantise recomputes the values from the received
    segments; at p = 2 the kernels built with p known) -- every rank bit-for-bit the reference
    sequence, in every dtype."""
    monkeypatch.setenv("BAGUA_PIPE_RECOMPUTE", recompute)
    from bagua_core.communicator import loopback_communicators
    if oracle_c.minmax_compressed_size(p, cs, dtype) % p:
        pytest.skip("reference alltoall requires S % nranks == 0")
    rng = np.random.default_rng(p * 1300 + dtype + cs)
    xs = [NP.from_f32((rng.standard_normal(p * cs) * 1e-3 + 0.01 * r).astype(np.float32), dtype) for r in range(p)]
    want = simulate.centralized_low_precision(oracle_c, xs, dtype, True)
    comms = loopback_communicators(p, 0)
    ts = [dev(x, dtype) for x in xs]
    torch.cuda.synchronize()
    N = bc._native

    def rank(r):
        raw = bc.BaguaTensorPy(ts[r], f"g{r}").raw()
        N.check(N.C.bagua_centralized_low_precision_pipelined(comms[r].handle, ctypes.byref(raw), 1,
                                                              N.COMPRESSION_MINMAX_UINT8, pieces), f"rank {r}")

    run_ranks(rank, p)
    for r in range(p):
        assert np.array_equal(host(ts[r], dtype).view(np.uint8), want[r].view(np.uint8)), f"rank {r}"


@pytest.mark.parametrize("p,dtype,cs,pieces", [(2, F32, 4096 * 3, 3), (4, F32, 40000, 4), (8, BF16, 2500 * 4, 2),
                                               (8, F32, 5000 * 8, 5), (4, F16, 1024 * 7 + 3, 3), (1, F32, 70000, 3),
                                               (16, F32, 3000 * 2, 2), (3, F32, 2048, 4), (2, F32, 0, 2),
                                               (2, F32, (1 << 24) + 1000, 0)])
def test_centralized_onebit_pipelined_multirank(bc, oracle_c, p, dtype, cs, pieces):
    """Pieced 1-bit op (sign bits of piece q exchanged while piece q+1 encodes, headers with
    the last alltoall piece and the first allgather piece) == the reference op sequence with the
    1-bit codec, every rank bit-for-bit.  (3, F32, 2048, 4): 2 tiles, empty trailing pieces;
    cs = 0: headers only; pieces = 0: automatic (4 pieces of >= 1 MiB of bits per chunk)."""
    from bagua_core.communicator import loopback_communicators
    rng = np.random.default_rng(p * 77 + cs + dtype)
    xs = [NP.from_f32((rng.standard_normal(p * cs) * 1e-3 - 3e-4 * r).astype(np.float32), dtype) for r in range(p)]
    want = simulate.centralized_low_precision(oracle_c, xs, dtype, True, method="OneBitSignScale")
    comms = loopback_communicators(p, 0)
    ts = [dev(x, dtype) for x in xs]
    torch.cuda.synchronize()
    N = bc._native

    def rank(r):
        raw = bc.BaguaTensorPy(ts[r], "g").raw()
        N.check(N.C.bagua_centralized_low_precision_pipelined(comms[r].handle, ctypes.byref(raw), 1,
                                                              N.COMPRESSION_ONEBIT, pieces), f"rank {r}")

    run_ranks(rank, p)
    for r in range(p):
        assert np.array_equal(host(ts[r], dtype).view(np.uint8), want[r].view(np.uint8)), f"rank {r}"


@pytest.mark.parametrize("p,dtype,short", [(2, F32, 37), (4, BF16, 1000), (3, F32, 4096 + 5)])
def test_centralized_partially_valid_tensor(bc, oracle_c, p, dtype, short):
    """num_elem < num_elem_allocated: the reference compresses num_elements()
    (DT:339); the op must run the unfused sequence and match it bit-for-bit."""
    from bagua_core.communicator import loopback_communicators
    cs = 12288
    n = p * cs
    rng = np.random.default_rng(7 * p + short)
    xs = [NP.from_f32((rng.standard_normal(n) * 1e-3 + 0.5 * r).astype(np.float32), dtype) for r in range(p)]
    want = simulate.centralized_low_precision(oracle_c, xs, dtype, True, num_elem=n - short)
    comms = loopback_communicators(p, 0)
    ts = [dev(x, dtype) for x in xs]
    torch.cuda.synchronize()
    N = bc._native

    def rank(r):
        raw = bc.BaguaTensorPy(ts[r], f"g{r}").raw()
        raw.num_elem = n - short
        N.check(N.C.bagua_centralized_low_precision_synchronous(comms[r].handle, ctypes.byref(raw), 1,
                                                                N.COMPRESSION_MINMAX_UINT8), f"rank {r}")

    run_ranks(rank, p)
    for r in range(p):
        assert np.array_equal(host(ts[r], dtype).view(np.uint8), want[r].view(np.uint8)), f"rank {r}"


@pytest.mark.parametrize("p,dtype,cs,unfused", [(2, F32, 4096 * 3, False), (4, F32, 4096 * 3, False),
                                               (3, F32, 5000, False), (8, BF16, 2500, False), (4, F16, 1024, False),
                                               (16, F32, 3000, False), (4, F32, 4096 * 3, True),
                                               (8, BF16, 2500, True)])
def test_centralized_onebit_multirank(bc, oracle_c, p, dtype, cs, unfused):
    """1-bit centralized op: fused decode+reduce+re-encode (onebit_reduce_encode_kernel) and the
    unfused sequence against the oracle simulation, every rank bit-for-bit (ragged cs included)."""
    from bagua_core.communicator import loopback_communicators
    rng = np.random.default_rng(p * 31 + cs + dtype)
    xs = [NP.from_f32((rng.standard_normal(p * cs) * 1e-3 + 2e-4 * r).astype(np.float32), dtype) for r in range(p)]
    want = simulate.centralized_low_precision(oracle_c, xs, dtype, True, method="OneBitSignScale")
    comms = loopback_communicators(p, 0)
    ts = [dev(x, dtype) for x in xs]
    torch.cuda.synchronize()
    N = bc._native
    fn = (N.C.bagua_centralized_low_precision_synchronous_unfused if unfused
          else N.C.bagua_centralized_low_precision_synchronous)

    def rank(r):
        raw = bc.BaguaTensorPy(ts[r], "g").raw()
        N.check(fn(comms[r].handle, ctypes.byref(raw), 1, N.COMPRESSION_ONEBIT), f"rank {r}")

    run_ranks(rank, p)
    for r in range(p):
        assert np.array_equal(host(ts[r], dtype).view(np.uint8), want[r].view(np.uint8)), f"rank {r}"


@pytest.mark.parametrize("p,dtype,n,unfused,offset", [(2, F32, 30011, False, 0), (3, F32, 30011, False, 0),
                                                     (4, BF16, 30011, False, 0), (8, F32, 30011, False, 0),
                                                     (2, F16, 65536 + 7, False, 0), (2, BF16, (1 << 20) + 3, False, 0),
                                                     (4, BF16, 30011, True, 0), (2, F32, 4099, False, 1)])
def test_decentralized_low_precision_multirank(bc, oracle_c, p, dtype, n, unfused, offset):
    """Fused ring kernels (decentralized.hip) and the reference sequence (`unfused`, or a
    misaligned tensor: offset elements) against the oracle's op simulation, every tensor."""
    from bagua_core.communicator import loopback_communicators
    rng = np.random.default_rng(50 + p + n)
    arrs = {k: [NP.from_f32((rng.standard_normal(n) * 1e-3).astype(np.float32), dtype) for _ in range(p)]
            for k in "twlr"}
    want = simulate.decentralized_low_precision(oracle_c, arrs["t"], arrs["w"], arrs["l"], arrs["r"], dtype)
    comms = loopback_communicators(p, 0)

    def place(a):
        full = dev(np.concatenate([np.zeros(offset, a.dtype), a]), dtype)
        return full[offset:]

    dts = {k: [place(a) for a in arrs[k]] for k in "twlr"}
    torch.cuda.synchronize()
    N = bc._native
    fn = (N.C.bagua_decentralized_low_precision_synchronous_unfused if unfused
          else N.C.bagua_decentralized_low_precision_synchronous)

    def rank(r):
        raws = [bc.BaguaTensorPy(dts[k][r], k).raw() for k in "twlr"]
        N.check(fn(comms[r].handle, *[ctypes.byref(x) for x in raws], N.COMPRESSION_MINMAX_UINT8), f"rank {r}")

    run_ranks(rank, p)
    for k, wk in zip("twlr", want):
        for r in range(p):
            assert np.array_equal(host(dts[k][r], dtype).view(np.uint8), wk[r].view(np.uint8)), f"{k} rank {r}"


@pytest.mark.parametrize("p,dtype,n,pieces", [(2, F32, 30011, 3), (3, BF16, 70001, 4), (4, F16, 65536 + 7, 2),
                                             (8, F32, 30011, 5), (1, BF16, 40000, 3), (2, BF16, (1 << 21) + 3, 0),
                                             (3, F32, 1000, 4)])
@pytest.mark.parametrize("taper", ["0", "1", None])
def test_decentralized_pipelined_multirank(bc, oracle_c, p, dtype, n, pieces, taper, monkeypatch):
    """Pieced ring op (quantise piece q -> send/recv piece q on the side stream -> apply piece q;
    one header travelling with piece 0) == the oracle's op simulation, all four tensors.
    (3, F32, 1000, 4): a single 512-aligned piece plus empty ones; pieces = 0: automatic.
    taper: first and last piece half size (BAGUA_PIPELINE_TAPER: 0, 1, or unset = the
    automatic schedules only)."""
    if taper is None:
        monkeypatch.delenv("BAGUA_PIPELINE_TAPER", raising=False)
    else:
        monkeypatch.setenv("BAGUA_PIPELINE_TAPER", taper)
    from bagua_core.communicator import loopback_communicators
    rng = np.random.default_rng(900 + p + n + pieces)
    arrs = {k: [NP.from_f32((rng.standard_normal(n) * 1e-3).astype(np.float32), dtype) for _ in range(p)]
            for k in "twlr"}
    want = simulate.decentralized_low_precision(oracle_c, arrs["t"], arrs["w"], arrs["l"], arrs["r"], dtype)
    comms = loopback_communicators(p, 0)
    dts = {k: [dev(a, dtype) for a in arrs[k]] for k in "twlr"}
    torch.cuda.synchronize()
    N = bc._native

    def rank(r):
        raws = [bc.BaguaTensorPy(dts[k][r], k).raw() for k in "twlr"]
        N.check(N.C.bagua_decentralized_low_precision_pipelined(comms[r].handle, *[ctypes.byref(x) for x in raws],
                                                                N.COMPRESSION_MINMAX_UINT8, pieces), f"rank {r}")

    run_ranks(rank, p)
    for k, wk in zip("twlr", want):
        for r in range(p):
            assert np.array_equal(host(dts[k][r], dtype).view(np.uint8), wk[r].view(np.uint8)), f"{k} rank {r}"


@pytest.mark.parametrize("mix_env", [{"BAGUA_RING_MIX_TILES": "0"}, {"BAGUA_RING_MIX_NTS": "1"},
                                     {"BAGUA_RING_MIX_TILES": "0", "BAGUA_RING_MIX_CONTIG": "1"}])
@pytest.mark.parametrize("p,dtype,n,pieces", [(2, BF16, (1 << 20) + 37, 1), (4, F32, 70001, 3)])
def test_ring_mix_shapes_multirank(bc, oracle_c, p, dtype, n, pieces, mix_env, monkeypatch):
    """The mix pass's other shapes (vector-strided -- the shape before round 5's tile-strided
    default --, non-temporal stores of the mixed t, contiguous ranges) leave every tensor of
    the ring op as the oracle's simulation has it: the min/max partials fold to the same
    header whatever the workgroups' ranges."""
    for k, v in mix_env.items():
        monkeypatch.setenv(k, v)
    from bagua_core.communicator import loopback_communicators
    rng = np.random.default_rng(77 + p + n + pieces)
    arrs = {k: [NP.from_f32((rng.standard_normal(n) * 1e-3).astype(np.float32), dtype) for _ in range(p)]
            for k in "twlr"}
    want = simulate.decentralized_low_precision(oracle_c, arrs["t"], arrs["w"], arrs["l"], arrs["r"], dtype)
    comms = loopback_communicators(p, 0)
    dts = {k: [dev(a, dtype) for a in arrs[k]] for k in "twlr"}
    torch.cuda.synchronize()
    N = bc._native

    def rank(r):
        raws = [bc.BaguaTensorPy(dts[k][r], k).raw() for k in "twlr"]
        N.check(N.C.bagua_decentralized_low_precision_pipelined(comms[r].handle, *[ctypes.byref(x) for x in raws],
                                                                N.COMPRESSION_MINMAX_UINT8, pieces), f"rank {r}")

    run_ranks(rank, p)
    for k, wk in zip("twlr", want):
        for r in range(p):
            assert np.array_equal(host(dts[k][r], dtype).view(np.uint8), wk[r].view(np.uint8)), f"{k} rank {r}"


def test_pipelined_ops_back_to_back_fuzz(bc, oracle_c):
    """Random shapes, rank counts and piece counts, every pipelined op run twice in a row on
    the same loopback communicators (pool buffers, events and workspaces are reused across
    ops): each result equals the oracle's simulation of the reference op sequence."""
    from bagua_core.communicator import loopback_communicators
    rng = np.random.default_rng(4242)
    N = bc._native
    for case in range(6):
        p = int(rng.integers(2, 9))
        dtype = int(rng.choice([F32, F16, BF16]))
        pieces = int(rng.integers(0, 6))
        comms = loopback_communicators(p, 0)
        # centralized MinMax and 1-bit (chunk sizes keep S % p == 0 for MinMax: multiples of 32)
        cs = int(rng.integers(1, 40)) * 1024 + 32 * int(rng.integers(0, 8))
        for method, name in ((N.COMPRESSION_MINMAX_UINT8, "MinMaxUInt8"), (N.COMPRESSION_ONEBIT, "OneBitSignScale")):
            if method == N.COMPRESSION_MINMAX_UINT8 and oracle_c.minmax_compressed_size(p, cs, dtype) % p:
                continue
            xs = [NP.from_f32((rng.standard_normal(p * cs) * 1e-3).astype(np.float32), dtype) for _ in range(p)]
            want = simulate.centralized_low_precision(oracle_c, xs, dtype, True, method=name)
            want2 = simulate.centralized_low_precision(oracle_c, want, dtype, True, method=name)
            ts = [dev(x, dtype) for x in xs]
            torch.cuda.synchronize()

            def rank(r, ts=ts, method=method):
                raw = bc.BaguaTensorPy(ts[r], "g").raw()
                for _ in range(2):
                    N.check(N.C.bagua_centralized_low_precision_pipelined(comms[r].handle, ctypes.byref(raw), 1,
                                                                          method, pieces), f"rank {r}")

            run_ranks(rank, p)
            for r in range(p):
                assert np.array_equal(host(ts[r], dtype).view(np.uint8), want2[r].view(np.uint8)), \
                    f"case {case} {name} p={p} cs={cs} pieces={pieces} rank {r}"
        # decentralized ring
        n = int(rng.integers(1, 300)) * 512 + int(rng.integers(0, 512))
        arrs = {k: [NP.from_f32((rng.standard_normal(n) * 1e-3).astype(np.float32), dtype) for _ in range(p)]
                for k in "twlr"}
        w1 = simulate.decentralized_low_precision(oracle_c, arrs["t"], arrs["w"], arrs["l"], arrs["r"], dtype)
        w2 = simulate.decentralized_low_precision(oracle_c, *w1, dtype)
        dts = {k: [dev(a, dtype) for a in arrs[k]] for k in "twlr"}
        torch.cuda.synchronize()

        def drank(r):
            raws = [bc.BaguaTensorPy(dts[k][r], k).raw() for k in "twlr"]
            for _ in range(2):
                N.check(N.C.bagua_decentralized_low_precision_pipelined(
                    comms[r].handle, *[ctypes.byref(x) for x in raws], N.COMPRESSION_MINMAX_UINT8, pieces), f"rank {r}")

        run_ranks(drank, p)
        for k, wk in zip("twlr", w2):
            for r in range(p):
                assert np.array_equal(host(dts[k][r], dtype).view(np.uint8), wk[r].view(np.uint8)), \
                    f"case {case} ring p={p} n={n} pieces={pieces} {k} rank {r}"



@pytest.mark.parametrize("p,dtype,n,pieces,multipath", [(6, F32, 30011, 1, True), (8, BF16, 70001, 4, True),
                                                       (8, F32, 65536 + 7, 0, True), (7, F16, 40000, 3, True),
                                                       (12, BF16, 20000, 2, True), (8, BF16, 70001, 4, False),
                                                       (8, F32, (1 << 20) + 3, 4, True)])
def test_decentralized_multipath_multirank(bc, oracle_c, p, dtype, n, pieces, multipath, monkeypatch):
    """Ring op with the multipath exchange (from 6 ranks: 3/p of each piece straight to the
    peer, the other slices relayed through ranks r +- (k-1) one group later; comm_ops.cpp
    ring_ops) == the oracle's op simulation on every rank and tensor; multipath False
    (BAGUA_RING_MULTIPATH=0) is the reference's direct exchange."""
    from bagua_core.communicator import loopback_communicators
    rng = np.random.default_rng(700 + p + n + pieces)
    arrs = {k: [NP.from_f32((rng.standard_normal(n) * 1e-3).astype(np.float32), dtype) for _ in range(p)]
            for k in "twlr"}
    want = simulate.decentralized_low_precision(oracle_c, arrs["t"], arrs["w"], arrs["l"], arrs["r"], dtype)
    # read once, when the communicators are created (ScheduleConfig)
    monkeypatch.setenv("BAGUA_RING_MULTIPATH", "1" if multipath else "0")
    comms = loopback_communicators(p, 0)
    dts = {k: [dev(a, dtype) for a in arrs[k]] for k in "twlr"}
    torch.cuda.synchronize()
    N = bc._native

    def rank(r):
        raws = [bc.BaguaTensorPy(dts[k][r], k).raw() for k in "twlr"]
        N.check(N.C.bagua_decentralized_low_precision_pipelined(
            comms[r].handle, *[ctypes.byref(x) for x in raws], N.COMPRESSION_MINMAX_UINT8, pieces), f"rank {r}")

    run_ranks(rank, p)
    for k, wk in zip("twlr", want):
        for r in range(p):
            assert np.array_equal(host(dts[k][r], dtype).view(np.uint8), wk[r].view(np.uint8)), f"{k} rank {r}"


@pytest.mark.parametrize("p,cs,pieces,offsets", [(4, 4096, 3, [0, 1, 0, 2]), (4, 999, 2, [0, 0, 0, 0]),
                                                 (2, 40000, 2, [1, 0])])
def test_pipelined_choice_is_rank_independent(bc, oracle_c, p, cs, pieces, offsets):
    """Every rank must take the same op schedule (the collectives must match): the
    pipelined/unpieced choice uses only sizes, never a rank's pointer.  A rank whose tensor
    is misaligned (offsets, in elements) runs the pipelined schedule on an aligned copy;
    a chunk size whose chunks are not 16-B aligned (cs = 999 f32) is unpieced on every
    rank.  Centralized MinMax op with explicit pieces, every rank == the oracle."""
    from bagua_core.communicator import loopback_communicators
    rng = np.random.default_rng(cs + pieces)
    xs = [(rng.standard_normal(p * cs) * 1e-3 + 0.01 * r).astype(np.float32) for r in range(p)]
    want = simulate.centralized_low_precision(oracle_c, xs, F32, True)
    comms = loopback_communicators(p, 0)
    bufs = [torch.zeros(p * cs + off, device="cuda") for off in offsets]
    ts = [b[off:] for b, off in zip(bufs, offsets)]
    for t, x in zip(ts, xs):
        t.copy_(torch.from_numpy(x))
    torch.cuda.synchronize()
    N = bc._native

    def rank(r):
        raw = bc.BaguaTensorPy(ts[r], f"g{r}").raw()
        N.check(N.C.bagua_centralized_low_precision_pipelined(comms[r].handle, ctypes.byref(raw), 1,
                                                              N.COMPRESSION_MINMAX_UINT8, pieces), f"rank {r}")

    run_ranks(rank, p)
    for r in range(p):
        assert np.array_equal(host(ts[r], F32).view(np.uint8), want[r].view(np.uint8)), f"rank {r}"


@pytest.mark.parametrize("offsets", [[0, 1], [1, 0, 0]])
def test_ring_pipelined_with_a_misaligned_rank(bc, oracle_c, offsets):
    """The pipelined ring op with one rank's tensors misaligned: that rank runs the fused,
    pieced schedule on aligned copies, so every rank posts the same exchange groups."""
    from bagua_core.communicator import loopback_communicators
    p, n = len(offsets), 30011
    rng = np.random.default_rng(77 + p)
    arrs = {k: [(rng.standard_normal(n) * 1e-3).astype(np.float32) for _ in range(p)] for k in "twlr"}
    want = simulate.decentralized_low_precision(oracle_c, arrs["t"], arrs["w"], arrs["l"], arrs["r"], F32)
    comms = loopback_communicators(p, 0)

    def place(a, off):
        full = torch.zeros(n + off, device="cuda")
        full[off:].copy_(torch.from_numpy(a))
        return full[off:]

    dts = {k: [place(a, off) for a, off in zip(arrs[k], offsets)] for k in "twlr"}
    torch.cuda.synchronize()
    N = bc._native

    def rank(r):
        raws = [bc.BaguaTensorPy(dts[k][r], k).raw() for k in "twlr"]
        N.check(N.C.bagua_decentralized_low_precision_pipelined(comms[r].handle, *[ctypes.byref(x) for x in raws],
                                                                N.COMPRESSION_MINMAX_UINT8, 3), f"rank {r}")

    run_ranks(rank, p)
    for k, wk in zip("twlr", want):
        for r in range(p):
            assert np.array_equal(host(dts[k][r], F32).view(np.uint8), wk[r].view(np.uint8)), f"{k} rank {r}"
