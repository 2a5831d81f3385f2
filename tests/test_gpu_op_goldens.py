"""The committed op fixtures through the HIP comm ops.

tests/golden/codec_v1.npz holds the oracle's simulations of the two comm ops
(generated and cross-checked by tests/golden/gen_golden.py, C and numpy
restatements agreeing byte for byte):
  cen_*   centralized_low_precision_synchronous.rs:16-73, every tensor fully valid;
  cenp_*  the same op on partially valid tensors (num_elements < allocated, DT:339);
  dec_*   decentralized_low_precision_synchronous.rs:23-154 (ring, all four tensors).
Here every variant of the op the library runs -- unpieced fused, pipelined with
automatic / explicit / tapered pieces, and the unfused reference sequence -- must
reproduce the STORED bytes on every rank (p virtual ranks on the loopback
transport, csrc/runtime/loopback.cpp), with no oracle call at test time."""
import ctypes

import numpy as np
import pytest
import torch

from test_gpu_multirank import BF16, dev, host, run_ranks

pytestmark = pytest.mark.gpu

STORAGE = {0: np.float32, 1: np.float16, 2: np.uint16}


@pytest.fixture(scope="module")
def bc():
    import bagua_core
    return bagua_core


def _cases(goldens, prefix, count_index):
    return range(int(goldens["counts"][count_index]))


def _arr(row, dtype):
    return row.view(STORAGE[dtype])


CENTRALIZED_VARIANTS = ["synchronous", "unfused", "pipelined_auto", "pipelined_2", "pipelined_3_tapered"]


def _centralized(bc, comm, raw, variant):
    N = bc._native
    if variant == "synchronous":
        return N.C.bagua_centralized_low_precision_synchronous(comm.handle, ctypes.byref(raw), 1,
                                                               N.COMPRESSION_MINMAX_UINT8)
    if variant == "unfused":
        return N.C.bagua_centralized_low_precision_synchronous_unfused(comm.handle, ctypes.byref(raw), 1,
                                                                       N.COMPRESSION_MINMAX_UINT8)
    pieces = {"pipelined_auto": 0, "pipelined_2": 2, "pipelined_3_tapered": 3 | N.PIECES_TAPERED}[variant]
    return N.C.bagua_centralized_low_precision_pipelined(comm.handle, ctypes.byref(raw), 1,
                                                         N.COMPRESSION_MINMAX_UINT8, pieces)


@pytest.mark.parametrize("variant", CENTRALIZED_VARIANTS)
def test_centralized_op_fixtures(bc, goldens, variant):
    from bagua_core.communicator import loopback_communicators
    for i in _cases(goldens, "cen", 3):
        dtype, p, cs = (int(v) for v in goldens[f"cen_meta_{i}"])
        print(f"cen case {i}: dtype {dtype} p {p} cs {cs} {variant}", flush=True)
        xs = [_arr(r, dtype) for r in goldens[f"cen_in_{i}"]]
        want = goldens[f"cen_out_{i}"]
        comms = loopback_communicators(p, 0)
        ts = [dev(x, dtype) for x in xs]
        torch.cuda.synchronize()

        def rank(r):
            raw = bc.BaguaTensorPy(ts[r], f"g{r}").raw()
            bc._native.check(_centralized(bc, comms[r], raw, variant), f"case {i} rank {r}")

        run_ranks(rank, p)
        for r in range(p):
            got = host(ts[r], dtype).view(np.uint8)
            assert np.array_equal(got, want), f"cen case {i} (dtype {dtype}, p {p}, cs {cs}) rank {r}, {variant}"
        del comms


@pytest.mark.parametrize("variant", ["synchronous", "unfused", "pipelined_auto"])
def test_centralized_partially_valid_op_fixtures(bc, goldens, variant):
    from bagua_core.communicator import loopback_communicators
    for i in _cases(goldens, "cenp", 6):
        dtype, p, cs, n_in = (int(v) for v in goldens[f"cenp_meta_{i}"])
        xs = [_arr(r, dtype) for r in goldens[f"cenp_in_{i}"]]
        comms = loopback_communicators(p, 0)
        ts = [dev(x, dtype) for x in xs]
        torch.cuda.synchronize()

        def rank(r):
            raw = bc.BaguaTensorPy(ts[r], f"g{r}").raw()
            raw.num_elem = n_in
            bc._native.check(_centralized(bc, comms[r], raw, variant), f"case {i} rank {r}")

        run_ranks(rank, p)
        for r in range(p):
            got = host(ts[r], dtype).view(np.uint8)
            assert np.array_equal(got, goldens[f"cenp_out_{i}"][r]), \
                f"cenp case {i} (dtype {dtype}, p {p}, cs {cs}, valid {n_in}) rank {r}, {variant}"
        del comms


@pytest.mark.parametrize("variant", ["synchronous", "unfused", "pipelined_2", "pipelined_3_tapered"])
def test_decentralized_op_fixtures(bc, goldens, variant):
    from bagua_core.communicator import loopback_communicators
    N = bc._native
    for i in _cases(goldens, "dec", 4):
        dtype, p, n = (int(v) for v in goldens[f"dec_meta_{i}"])
        arrs = {k: [_arr(row, dtype) for row in goldens[f"dec_in_{k}_{i}"]] for k in "twlr"}
        comms = loopback_communicators(p, 0)
        dts = {k: [dev(a, dtype) for a in arrs[k]] for k in "twlr"}
        torch.cuda.synchronize()

        def rank(r):
            raws = [bc.BaguaTensorPy(dts[k][r], k).raw() for k in "twlr"]
            refs = [ctypes.byref(x) for x in raws]
            if variant == "synchronous":
                rc = N.C.bagua_decentralized_low_precision_synchronous(comms[r].handle, *refs,
                                                                       N.COMPRESSION_MINMAX_UINT8)
            elif variant == "unfused":
                rc = N.C.bagua_decentralized_low_precision_synchronous_unfused(comms[r].handle, *refs,
                                                                               N.COMPRESSION_MINMAX_UINT8)
            else:
                pieces = 2 if variant == "pipelined_2" else 3 | N.PIECES_TAPERED
                rc = N.C.bagua_decentralized_low_precision_pipelined(comms[r].handle, *refs,
                                                                     N.COMPRESSION_MINMAX_UINT8, pieces)
            N.check(rc, f"case {i} rank {r}")

        run_ranks(rank, p)
        for k in "twlr":
            for r in range(p):
                got = host(dts[k][r], dtype).view(np.uint8)
                assert np.array_equal(got, goldens[f"dec_out_{k}_{i}"][r]), \
                    f"dec case {i} (dtype {dtype}, p {p}, n {n}) tensor {k} rank {r}, {variant}"
        del comms


def test_fixture_counts_cover_all_three_dtypes(goldens):
    """the committed op cases span f32 and bf16 (centralized) and f32 / bf16 / f16 (ring)"""
    cen = {int(goldens[f"cen_meta_{i}"][0]) for i in _cases(goldens, "cen", 3)}
    dec = {int(goldens[f"dec_meta_{i}"][0]) for i in _cases(goldens, "dec", 4)}
    assert cen >= {0, BF16} and dec == {0, 1, BF16}
