"""CPU simulation of the compressed comm ops over p ranks.

TEST INFRASTRUCTURE ONLY.  Composes the oracle codec primitives exactly in
the reference's op order, with the collectives replaced by array moves:

  centralized_low_precision  centralized_low_precision_synchronous.rs:30-71
  decentralized_low_precision decentralized_low_precision_synchronous.rs:42-152

`backend` is oracle.oracle_c or oracle.oracle_np (same function names).
Alltoall/allgather semantics (communicators/mod.rs:602-630, 760-787):
count = S/p bytes; after alltoall rank r's slot j holds rank j's segment r;
allgather fills slot j with rank j's slot j.
"""
from __future__ import annotations

import numpy as np


def centralized_low_precision(backend, inputs: list[np.ndarray], dtype: int, average: bool = True,
                              method: str = "MinMaxUInt8", num_elem: int | None = None) -> list[np.ndarray]:
    """`num_elem` < allocated size: the tensors' num_elements() (MinMax only; both backends)."""
    p = len(inputs)
    comp = backend.compress_minmax_u8 if method == "MinMaxUInt8" else backend.compress_onebit
    if num_elem is not None:
        base_comp = comp

        def comp(t, dtype, n_chunks, target, out=None):
            return base_comp(t, dtype, n_chunks, target, out=out, num_elem=num_elem)
    decomp = backend.decompress_minmax_u8 if method == "MinMaxUInt8" else backend.decompress_onebit
    ts = [x.copy() for x in inputs]
    send = [comp(t, dtype, p, -1) for t in ts]
    S = send[0].size
    assert S % p == 0, "tensors must be aligned before using allscatter"
    cnt = S // p
    recv = [np.concatenate([send[j][r * cnt:(r + 1) * cnt] for j in range(p)]) for r in range(p)]
    gathered_slots = []
    for r in range(p):
        decomp(recv[r], p, ts[r], dtype)
        backend.reduce_chunks(ts[r], dtype, p, r, average)
        buf = np.zeros(S, np.uint8)
        comp(ts[r], dtype, p, r, out=buf)
        gathered_slots.append(buf[r * cnt:(r + 1) * cnt].copy())
    gathered = np.concatenate(gathered_slots)
    for r in range(p):
        decomp(gathered, p, ts[r], dtype)
    return ts


def decentralized_low_precision(backend, ts: list[np.ndarray], weights: list[np.ndarray],
                                lefts: list[np.ndarray], rights: list[np.ndarray], dtype: int,
                                method: str = "MinMaxUInt8"):
    """Returns updated (t, weight, left, right) per rank (ring peers)."""
    p = len(ts)
    comp = backend.compress_minmax_u8 if method == "MinMaxUInt8" else backend.compress_onebit
    decomp = backend.decompress_minmax_u8 if method == "MinMaxUInt8" else backend.decompress_onebit
    ts = [t.copy() for t in ts]
    weights = [w.copy() for w in weights]
    lefts = [x.copy() for x in lefts]
    rights = [x.copy() for x in rights]
    f13 = float(np.float32(1.0 / 3.0))
    f53 = float(np.float32(-5.0 / 3.0))
    comps = []
    for r in range(p):
        backend.addmul_inplace(ts[r], lefts[r], dtype, f13)
        backend.addmul_inplace(ts[r], rights[r], dtype, f13)
        backend.addmul_inplace(ts[r], weights[r], dtype, f53)
        comps.append(comp(ts[r], dtype, 1, -1))
    for r in range(p):
        lpeer, rpeer = (r + p - 1) % p, (r + 1) % p
        decomp(comps[lpeer], 1, ts[r], dtype)
        backend.add_inplace(lefts[r], ts[r], dtype)
        decomp(comps[rpeer], 1, ts[r], dtype)
        backend.add_inplace(rights[r], ts[r], dtype)
        decomp(comps[r], 1, ts[r], dtype)
        backend.add_inplace(ts[r], weights[r], dtype)
        weights[r][...] = ts[r]
    return ts, weights, lefts, rights
