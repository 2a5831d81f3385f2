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
