"""Worker of tests/test_distributed_sim.py: one rank of the compressed comm
ops over torch.distributed (gloo, CPU), computing with the C oracle.

This is the multi-rank rehearsal of the RCCL path: the same op order as
bagua-core_amd/csrc/runtime/comm_ops.cpp (compress -> out-of-place alltoall
-> dequantise+reduce -> requantise own chunk -> in-place allgather ->
decompress; ring send/recv for the decentralized op), with real collectives
moving the real compressed bytes between processes.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch
import torch.distributed as dist

from oracle import oracle_c as C


def centralized_rank(rank: int, world: int, port: int, inputs_path: str, out_dir: str, dtype: int) -> None:
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        with np.load(inputs_path, allow_pickle=False) as z:
            t = z[f"x{rank}"].copy()
        p = world
        send = C.compress_minmax_u8(t, dtype, p, -1)
        S = send.size
        assert S % p == 0
        recv = torch.empty(S, dtype=torch.uint8)
        dist.all_to_all_single(recv, torch.from_numpy(send))
        C.decompress_minmax_u8(recv.numpy(), p, t, dtype)
        C.reduce_chunks(t, dtype, p, rank, True)
        C.compress_minmax_u8(t, dtype, p, rank, out=send)
        cnt = S // p
        gathered = torch.empty(S, dtype=torch.uint8)
        dist.all_gather_into_tensor(gathered, torch.from_numpy(send[rank * cnt:(rank + 1) * cnt].copy()))
        C.decompress_minmax_u8(gathered.numpy(), p, t, dtype)
        np.save(os.path.join(out_dir, f"out{rank}.npy"), t.view(np.uint8))
    finally:
        dist.destroy_process_group()


def _piece_range(cs: int, pieces: int, q: int) -> tuple[int, int]:
    """bagua_minmax_u8_piece_range from the built kernel library (host-only function)."""
    import ctypes
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = ctypes.CDLL(os.path.join(root, "bagua-core_amd", "lib", "libbagua_kernels.so"))
    b, e = ctypes.c_int(), ctypes.c_int()
    assert lib.bagua_minmax_u8_piece_range(cs, pieces, q, ctypes.byref(b), ctypes.byref(e)) == 0
    return b.value, e.value


def _piece_bytes(cs: int, co: int, pieces: int, q: int) -> tuple[int, int]:
    # comm_ops.cpp piece_bytes: header with piece 0, slack with the last non-empty piece
    b, e = _piece_range(cs, pieces, q)
    if q > 0 and b == e:
        return 0, 0
    return (0 if q == 0 else 32 + b), (co if e == cs else 32 + e)


def centralized_pieced_rank(rank: int, world: int, port: int, inputs_path: str, out_dir: str, dtype: int,
                            pieces: int) -> None:
    """The pipelined op's exchange protocol (comm_ops.cpp centralized_pipelined): every
    alltoall / allgather moves one byte range of every segment per piece."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        with np.load(inputs_path, allow_pickle=False) as z:
            t = z[f"x{rank}"].copy()
        p = world
        cs = t.size // p
        send = C.compress_minmax_u8(t, dtype, p, -1)
        S = send.size
        co = S // p
        recv = np.full(S, 0xAB, np.uint8)  # poison: every byte must arrive through a piece
        for q in range(pieces):
            lo, hi = _piece_bytes(cs, co, pieces, q)
            if hi <= lo:
                continue
            part = torch.from_numpy(np.concatenate([send[j * co + lo:j * co + hi] for j in range(p)]))
            got = torch.empty_like(part)
            dist.all_to_all_single(got, part)
            g = got.numpy()
            for j in range(p):
                recv[j * co + lo:j * co + hi] = g[j * (hi - lo):(j + 1) * (hi - lo)]
        C.decompress_minmax_u8(recv, p, t, dtype)
        C.reduce_chunks(t, dtype, p, rank, True)
        C.compress_minmax_u8(t, dtype, p, rank, out=send)
        for q in range(pieces):
            lo, hi = _piece_bytes(cs, co, pieces, q)
            if hi <= lo:
                continue
            got = torch.empty(p * (hi - lo), dtype=torch.uint8)
            dist.all_gather_into_tensor(got, torch.from_numpy(send[rank * co + lo:rank * co + hi].copy()))
            g = got.numpy()
            for j in range(p):
                send[j * co + lo:j * co + hi] = g[j * (hi - lo):(j + 1) * (hi - lo)]
        C.decompress_minmax_u8(send, p, t, dtype)
        np.save(os.path.join(out_dir, f"out{rank}.npy"), t.view(np.uint8))
    finally:
        dist.destroy_process_group()


def _onebit_piece_bytes(cs: int, co: int, pieces: int, q: int, header: bool) -> tuple[int, int]:
    # comm_ops.cpp onebit_piece_bytes: tile range of bagua_onebit_piece_range, 128 B per tile
    import ctypes
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = ctypes.CDLL(os.path.join(root, "bagua-core_amd", "lib", "libbagua_kernels.so"))
    b, e = ctypes.c_int(), ctypes.c_int()
    assert lib.bagua_onebit_piece_range(cs, pieces, q, ctypes.byref(b), ctypes.byref(e)) == 0
    tiles = (cs + 1023) // 1024
    lo = 0 if header else 32 + 128 * b.value
    hi = co if e.value >= tiles else 32 + 128 * e.value
    if not header and b.value >= e.value:
        return 0, 0
    return lo, hi


def _alltoall_range(send: np.ndarray, recv: np.ndarray, p: int, co: int, lo: int, hi: int) -> None:
    if hi <= lo:
        return
    part = torch.from_numpy(np.concatenate([send[j * co + lo:j * co + hi] for j in range(p)]))
    got = torch.empty_like(part)
    dist.all_to_all_single(got, part)
    g = got.numpy()
    for j in range(p):
        recv[j * co + lo:j * co + hi] = g[j * (hi - lo):(j + 1) * (hi - lo)]


def _allgather_range(send: np.ndarray, rank: int, p: int, co: int, lo: int, hi: int) -> None:
    if hi <= lo:
        return
    got = torch.empty(p * (hi - lo), dtype=torch.uint8)
    dist.all_gather_into_tensor(got, torch.from_numpy(send[rank * co + lo:rank * co + hi].copy()))
    g = got.numpy()
    for j in range(p):
        send[j * co + lo:j * co + hi] = g[j * (hi - lo):(j + 1) * (hi - lo)]


def centralized_onebit_pieced_rank(rank: int, world: int, port: int, inputs_path: str, out_dir: str, dtype: int,
                                   pieces: int) -> None:
    """The pipelined 1-bit op's exchange protocol (comm_ops.cpp centralized_pipelined_onebit):
    sign bits piece by piece, headers after the last alltoall piece, headers with the first
    allgather piece."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        with np.load(inputs_path, allow_pickle=False) as z:
            t = z[f"x{rank}"].copy()
        p = world
        cs = t.size // p
        send = C.compress_onebit(t, dtype, p, -1)
        S = send.size
        co = S // p
        recv = np.full(S, 0xAB, np.uint8)  # poison: every byte must arrive through a piece
        for q in range(pieces):
            _alltoall_range(send, recv, p, co, *_onebit_piece_bytes(cs, co, pieces, q, False))
        _alltoall_range(send, recv, p, co, 0, 32)
        C.decompress_onebit(recv, p, t, dtype)
        C.reduce_chunks(t, dtype, p, rank, True)
        C.compress_onebit(t, dtype, p, rank, out=send)
        for q in range(pieces):
            _allgather_range(send, rank, p, co, *_onebit_piece_bytes(cs, co, pieces, q, q == 0))
        C.decompress_onebit(send, p, t, dtype)
        np.save(os.path.join(out_dir, f"out{rank}.npy"), t.view(np.uint8))
    finally:
        dist.destroy_process_group()


def decentralized_rank(rank: int, world: int, port: int, inputs_path: str, out_dir: str, dtype: int) -> None:
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        with np.load(inputs_path, allow_pickle=False) as z:
            t, w, l, r = (z[f"{k}{rank}"].copy() for k in "twlr")
        f13, f53 = float(np.float32(1.0 / 3.0)), float(np.float32(-5.0 / 3.0))
        C.addmul_inplace(t, l, dtype, f13)
        C.addmul_inplace(t, r, dtype, f13)
        C.addmul_inplace(t, w, dtype, f53)
        mine = C.compress_minmax_u8(t, dtype, 1, -1)
        lpeer, rpeer = (rank + world - 1) % world, (rank + 1) % world
        lbuf, rbuf = torch.empty(mine.size, dtype=torch.uint8), torch.empty(mine.size, dtype=torch.uint8)
        m = torch.from_numpy(mine)
        reqs = [dist.isend(m, lpeer, tag=1), dist.isend(m, rpeer, tag=2),
                dist.irecv(lbuf, lpeer, tag=2), dist.irecv(rbuf, rpeer, tag=1)]
        for q in reqs:
            q.wait()
        C.decompress_minmax_u8(lbuf.numpy(), 1, t, dtype)
        C.add_inplace(l, t, dtype)
        C.decompress_minmax_u8(rbuf.numpy(), 1, t, dtype)
        C.add_inplace(r, t, dtype)
        C.decompress_minmax_u8(mine, 1, t, dtype)
        C.add_inplace(t, w, dtype)
        w[...] = t
        np.savez(os.path.join(out_dir, f"dec{rank}.npz"), t=t.view(np.uint8), w=w.view(np.uint8),
                 l=l.view(np.uint8), r=r.view(np.uint8))
    finally:
        dist.destroy_process_group()


class P2POp(ctypes.Structure):
    """bagua_p2p_op_t (include/bagua_core.h)"""
    _fields_ = [("peer", ctypes.c_int32), ("is_send", ctypes.c_int32), ("buffer", ctypes.c_int32),
                ("key", ctypes.c_int32), ("offset", ctypes.c_uint64), ("bytes", ctypes.c_uint64)]


def _core_lib():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return ctypes.CDLL(os.path.join(root, "bagua-core_amd", "lib", "libbagua_core.so"))


def ring_plan(p: int, rank: int, n: int, pieces: int, multipath: bool) -> tuple[int, int]:
    """(groups, relay scratch bytes) of bagua_ring_exchange_plan (host-only)."""
    lib = _core_lib()
    g, rb = ctypes.c_int(), ctypes.c_size_t()
    assert lib.bagua_ring_exchange_plan(p, rank, n, pieces, int(multipath), ctypes.byref(g), ctypes.byref(rb)) == 0
    return g.value, rb.value


def ring_ops(p: int, rank: int, n: int, pieces: int, multipath: bool, group: int) -> list:
    """Group `group`'s transfers from bagua_ring_exchange_ops (host-only):
    [(peer, is_send, buffer, key, offset, bytes)] in posting order."""
    lib = _core_lib()
    cap = 8 * p + 16
    arr = (P2POp * cap)()
    cnt = lib.bagua_ring_exchange_ops(p, rank, n, pieces, int(multipath), group, arr, cap)
    assert cnt >= 0, cnt
    return [(o.peer, o.is_send, o.buffer, o.key, o.offset, o.bytes) for o in arr[:cnt]]


def decentralized_multipath_rank(rank: int, world: int, port: int, inputs_path: str, out_dir: str, dtype: int,
                                 pieces: int) -> None:
    """The fused ring op's exchange (comm_ops.cpp ring_ops: direct slices + relayed slices,
    relays forward one group later) executed with gloo point-to-point transfers; a
    transfer is matched by its (hop, flow, slice) key, so the test checks the routing
    itself.  Receive buffers are poisoned: every byte must arrive."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        with np.load(inputs_path, allow_pickle=False) as z:
            t, w, l, r = (z[f"{k}{rank}"].copy() for k in "twlr")
        n = t.size
        f13, f53 = float(np.float32(1.0 / 3.0)), float(np.float32(-5.0 / 3.0))
        C.addmul_inplace(t, l, dtype, f13)
        C.addmul_inplace(t, r, dtype, f13)
        C.addmul_inplace(t, w, dtype, f53)
        mine = C.compress_minmax_u8(t, dtype, 1, -1)
        groups, relay_bytes = ring_plan(world, rank, n, pieces, True)
        bufs = [torch.from_numpy(mine), torch.full((mine.size,), 0xAB, dtype=torch.uint8),
                torch.full((mine.size,), 0xAB, dtype=torch.uint8), torch.zeros(max(1, relay_bytes), dtype=torch.uint8)]
        for g in range(groups):
            reqs = []
            for peer, is_send, buf, key, off, nbytes in ring_ops(world, rank, n, pieces, True, g):
                view = bufs[buf][off:off + nbytes]
                tag = g * 65536 + key
                reqs.append(dist.isend(view.clone(), peer, tag=tag) if is_send else (dist.irecv(view, peer, tag=tag)))
            for q in reqs:
                q.wait()
            dist.barrier()  # the relay scratch of group g is read in group g + 1 only
        lbuf, rbuf = bufs[1].numpy(), bufs[2].numpy()
        C.decompress_minmax_u8(lbuf, 1, t, dtype)
        C.add_inplace(l, t, dtype)
        C.decompress_minmax_u8(rbuf, 1, t, dtype)
        C.add_inplace(r, t, dtype)
        C.decompress_minmax_u8(mine, 1, t, dtype)
        C.add_inplace(t, w, dtype)
        w[...] = t
        np.savez(os.path.join(out_dir, f"dec{rank}.npz"), t=t.view(np.uint8), w=w.view(np.uint8),
                 l=l.view(np.uint8), r=r.view(np.uint8))
    finally:
        dist.destroy_process_group()


def hierarchical_rank(rank: int, world: int, port: int, inputs_path: str, out_dir: str, per_node: int) -> None:
    """Hierarchical mode (communicators/mod.rs:243-427, comm_ops.cpp hierarchical):
    reduce (AVG) into the node leader over the node's group, the compressed op among
    the leaders over their own group, broadcast from the leader over the node."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nodes = world // per_node
        node, local = divmod(rank, per_node)
        # every process creates every group, in the same order (torch.distributed rule)
        intra = [dist.new_group(list(range(k * per_node, (k + 1) * per_node))) for k in range(nodes)]
        inter = dist.new_group([k * per_node for k in range(nodes)])
        with np.load(inputs_path, allow_pickle=False) as z:
            t = z[f"x{rank}"].copy()
        leader = node * per_node
        buf = torch.from_numpy(t)
        dist.reduce(buf, dst=leader, op=dist.ReduceOp.SUM, group=intra[node])  # 2 ranks: x0 + x1 either way
        if local == 0:
            t = (buf.numpy() / np.float32(per_node)).astype(np.float32)  # AVG
            p = nodes
            send = C.compress_minmax_u8(t, 0, p, -1)
            S = send.size
            recv = torch.empty(S, dtype=torch.uint8)
            dist.all_to_all_single(recv, torch.from_numpy(send), group=inter)
            C.decompress_minmax_u8(recv.numpy(), p, t, 0)
            C.reduce_chunks(t, 0, p, node, True)
            C.compress_minmax_u8(t, 0, p, node, out=send)
            cnt = S // p
            gathered = torch.empty(S, dtype=torch.uint8)
            dist.all_gather_into_tensor(gathered, torch.from_numpy(send[node * cnt:(node + 1) * cnt].copy()),
                                        group=inter)
            C.decompress_minmax_u8(gathered.numpy(), p, t, 0)
            buf = torch.from_numpy(t)
        dist.broadcast(buf, src=leader, group=intra[node])
        np.save(os.path.join(out_dir, f"out{rank}.npy"), buf.numpy().view(np.uint8))
    finally:
        dist.destroy_process_group()
