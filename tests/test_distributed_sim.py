"""CPU multi-process tests (gloo, world_size 2, 3, 4 and 8) of the compressed
all-reduce and the ring exchange: real collectives carry the compressed
bytes between processes; the result must equal the single-process
simulation of the reference op sequence bit-for-bit on every rank, and all
ranks must end with identical gradients (centralized op)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import oracle_c, oracle_np as NP
from oracle import simulate

import dist_worker


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,dtype,cs", [(2, 0, 5000), (4, 0, 1031 * 8), (2, 2, 4096)])
def test_centralized_gloo(tmp_path, world, dtype, cs):
    oracle_c.build()
    rng = np.random.default_rng(world * 7 + dtype)
    xs = [NP.from_f32((rng.standard_normal(world * cs) * 1e-3).astype(np.float32), dtype) for _ in range(world)]
    if oracle_c.minmax_compressed_size(world, cs, dtype) % world:
        pytest.skip("reference alltoall requires S % nranks == 0")
    inputs = tmp_path / "in.npz"
    np.savez(inputs, **{f"x{r}": x for r, x in enumerate(xs)})
    mp.spawn(dist_worker.centralized_rank, args=(world, _free_port(), str(inputs), str(tmp_path), dtype),
             nprocs=world, join=True)
    want = simulate.centralized_low_precision(oracle_c, xs, dtype, True)
    outs = [np.load(tmp_path / f"out{r}.npy") for r in range(world)]
    for r in range(world):
        assert np.array_equal(outs[r], want[r].view(np.uint8)), f"rank {r}"
        assert np.array_equal(outs[r], outs[0])


@pytest.mark.parametrize("world,dtype,cs,pieces", [(2, 0, 5000, 3), (4, 0, 1031 * 8, 4), (2, 2, 1536, 4),
                                                   (8, 0, 1031 * 8, 4)])  # the driver's N = 8
def test_centralized_pieced_gloo(tmp_path, world, dtype, cs, pieces):
    """The pipelined op's per-piece byte ranges (real bagua_minmax_u8_piece_range) moved
    between gloo processes reproduce the unpieced op bit-for-bit."""
    oracle_c.build()
    rng = np.random.default_rng(world * 11 + dtype + pieces)
    xs = [NP.from_f32((rng.standard_normal(world * cs) * 1e-3).astype(np.float32), dtype) for _ in range(world)]
    if oracle_c.minmax_compressed_size(world, cs, dtype) % world:
        pytest.skip("reference alltoall requires S % nranks == 0")
    inputs = tmp_path / "in.npz"
    np.savez(inputs, **{f"x{r}": x for r, x in enumerate(xs)})
    mp.spawn(dist_worker.centralized_pieced_rank, args=(world, _free_port(), str(inputs), str(tmp_path), dtype,
                                                         pieces), nprocs=world, join=True)
    want = simulate.centralized_low_precision(oracle_c, xs, dtype, True)
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"out{r}.npy"), want[r].view(np.uint8)), f"rank {r}"


@pytest.mark.parametrize("world,dtype,cs,pieces", [(2, 0, 5000, 3), (4, 0, 1024 * 9 + 7, 4), (3, 2, 2048, 4),
                                                   (8, 0, 1024 * 5 + 3, 3)])
def test_centralized_onebit_pieced_gloo(tmp_path, world, dtype, cs, pieces):
    """The pipelined 1-bit op's per-piece byte ranges (real bagua_onebit_piece_range; headers
    after the last alltoall piece, with the first allgather piece) moved between gloo
    processes reproduce the reference op sequence with the 1-bit codec bit-for-bit."""
    oracle_c.build()
    rng = np.random.default_rng(world * 13 + dtype + pieces)
    xs = [NP.from_f32((rng.standard_normal(world * cs) * 1e-3).astype(np.float32), dtype) for _ in range(world)]
    inputs = tmp_path / "in.npz"
    np.savez(inputs, **{f"x{r}": x for r, x in enumerate(xs)})
    mp.spawn(dist_worker.centralized_onebit_pieced_rank, args=(world, _free_port(), str(inputs), str(tmp_path),
                                                               dtype, pieces), nprocs=world, join=True)
    want = simulate.centralized_low_precision(oracle_c, xs, dtype, True, method="OneBitSignScale")
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"out{r}.npy"), want[r].view(np.uint8)), f"rank {r}"


@pytest.mark.parametrize("world", [2, 3])
def test_decentralized_ring_gloo(tmp_path, world):
    oracle_c.build()
    dtype, n = 0, 7001
    rng = np.random.default_rng(world)
    arrs = {k: [(rng.standard_normal(n) * 1e-3).astype(np.float32) for _ in range(world)] for k in "twlr"}
    inputs = tmp_path / "in.npz"
    np.savez(inputs, **{f"{k}{r}": arrs[k][r] for k in "twlr" for r in range(world)})
    mp.spawn(dist_worker.decentralized_rank, args=(world, _free_port(), str(inputs), str(tmp_path), dtype),
             nprocs=world, join=True)
    want = simulate.decentralized_low_precision(oracle_c, arrs["t"], arrs["w"], arrs["l"], arrs["r"], dtype)
    for r in range(world):
        with np.load(tmp_path / f"dec{r}.npz", allow_pickle=False) as z:
            for k, wk in zip("twlr", want):
                assert np.array_equal(z[k], wk[r].view(np.uint8)), f"rank {r} {k}"


def _simulate_ring_exchange(p: int, n: int, pieces: int, multipath: bool, rng) -> dict:
    """Runs bagua_ring_exchange_ops' schedule for all p ranks on host byte arrays,
    matching grouped transfers per (sender, receiver) pair in posting order as
    NCCL does; returns per-rank buffers and per-link byte counts."""
    groups, relay = dist_worker.ring_plan(p, 0, n, pieces, multipath)
    S = ((n + 31) // 32) * 32 + 32
    bufs = [[rng.integers(0, 256, S, dtype=np.uint8), np.full(S, 0xAB, np.uint8), np.full(S, 0xAB, np.uint8),
             np.zeros(max(1, relay), np.uint8)] for _ in range(p)]
    link = {}
    for g in range(groups):
        ops = [dist_worker.ring_ops(p, r, n, pieces, multipath, g) for r in range(p)]
        sends, recvs = {}, {}
        for r in range(p):
            for peer, is_send, buf, key, off, nb in ops[r]:
                (sends if is_send else recvs).setdefault((r, peer) if is_send else (peer, r), []).append(
                    (buf, key, off, nb))
        assert sends.keys() == recvs.keys()
        moves = []
        for (src, dst), ss in sends.items():
            rr = recvs[(src, dst)]
            assert len(ss) == len(rr)
            for (sb, skey, soff, snb), (rb, rkey, roff, rnb) in zip(ss, rr):
                assert skey == rkey and snb == rnb, (g, src, dst)
                moves.append((dst, rb, roff, bufs[src][sb][soff:soff + snb].copy()))
                if src != dst:
                    link[(src, dst)] = link.get((src, dst), 0) + snb
        for dst, rb, roff, data in moves:  # a group's sends read what was there before it
            bufs[dst][rb][roff:roff + data.size] = data
    return {"bufs": bufs, "link": link, "S": S, "groups": groups}


@pytest.mark.parametrize("p", [1, 2, 3, 5, 6, 7, 8, 12, 16])
@pytest.mark.parametrize("pieces", [1, 3, 4])
@pytest.mark.parametrize("multipath", [False, True])
@pytest.mark.parametrize("n", [200_003, 100])  # 100: slices of a few bytes, most of them empty
def test_ring_exchange_schedule(p, pieces, multipath, n):
    """Host-only check of the ring exchange schedule (comm_ops.cpp ring_ops): every rank
    ends with its left and right peers' payload byte for byte, matched transfers agree
    on key and size, and with multipath from 6 ranks on no link carries more than
    4/p of a payload (8 ranks: half; direct: all of it) plus slice rounding."""
    rng = np.random.default_rng(p * 100 + pieces)
    sim = _simulate_ring_exchange(p, n, pieces, multipath, rng)
    bufs, S = sim["bufs"], sim["S"]
    for r in range(p):
        assert np.array_equal(bufs[r][1], bufs[(r - 1) % p][0]), f"rank {r} left"
        assert np.array_equal(bufs[r][2], bufs[(r + 1) % p][0]), f"rank {r} right"
    assert sim["groups"] == pieces + (1 if multipath and p >= 6 else 0)
    if p >= 3 and n > 100_000:
        worst = max(sim["link"].values())
        if multipath and p >= 6:
            assert worst <= 4 * S / p + 64 * pieces * 4, (worst, S)
        else:
            assert worst == S


@pytest.mark.parametrize("world,pieces,dtype", [(6, 3, 0), (8, 4, 0), (8, 1, 2)])  # the driver's N = 8
def test_decentralized_multipath_gloo(tmp_path, world, pieces, dtype):
    """The multipath ring exchange (relayed slices) between gloo processes reproduces the
    reference op sequence bit-for-bit on every rank and tensor."""
    oracle_c.build()
    n = 30_011
    rng = np.random.default_rng(world * 17 + pieces)
    arrs = {k: [NP.from_f32((rng.standard_normal(n) * 1e-3).astype(np.float32), dtype) for _ in range(world)]
            for k in "twlr"}
    inputs = tmp_path / "in.npz"
    np.savez(inputs, **{f"{k}{r}": arrs[k][r] for k in "twlr" for r in range(world)})
    mp.spawn(dist_worker.decentralized_multipath_rank, args=(world, _free_port(), str(inputs), str(tmp_path), dtype,
                                                             pieces), nprocs=world, join=True)
    want = simulate.decentralized_low_precision(oracle_c, arrs["t"], arrs["w"], arrs["l"], arrs["r"], dtype)
    for r in range(world):
        with np.load(tmp_path / f"dec{r}.npz", allow_pickle=False) as z:
            for k, wk in zip("twlr", want):
                assert np.array_equal(z[k], wk[r].view(np.uint8)), f"rank {r} {k}"


@pytest.mark.parametrize("nodes", [2, 4])
def test_hierarchical_gloo(tmp_path, nodes):
    """Hierarchical mode with real process groups: 2 ranks per node, node averages
    reduced into the leaders, the compressed op among the leaders, broadcast back;
    every rank equals the simulation of the leaders' op on the node averages."""
    oracle_c.build()
    per_node, cs = 2, 4096
    world = nodes * per_node
    rng = np.random.default_rng(40 + nodes)
    xs = [(rng.standard_normal(nodes * cs) * 1e-3).astype(np.float32) for _ in range(world)]
    inputs = tmp_path / "in.npz"
    np.savez(inputs, **{f"x{r}": x for r, x in enumerate(xs)})
    mp.spawn(dist_worker.hierarchical_rank, args=(world, _free_port(), str(inputs), str(tmp_path), per_node),
             nprocs=world, join=True)
    node_avg = [((xs[k * per_node] + xs[k * per_node + 1]).astype(np.float32) / np.float32(per_node)).astype(np.float32)
                for k in range(nodes)]
    want = simulate.centralized_low_precision(oracle_c, node_avg, 0, True)
    for r in range(world):
        out = np.load(tmp_path / f"out{r}.npy")
        assert np.array_equal(out, want[r // per_node].view(np.uint8)), f"rank {r}"
