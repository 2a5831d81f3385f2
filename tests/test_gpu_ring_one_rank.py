"""The decentralized ring op at one rank in two passes (bagua_ring_one_rank_minmax:
the mix pass, then one pass applying d = dq(q(mixed)) to the four tensors) against
the oracle's op simulation (decentralized_low_precision_synchronous.rs:42-152 with
p = 1: both ring peers are the rank itself) and against the op's four-kernel sequence
(BAGUA_ONE_RANK_FUSED=0), bit for bit on all four tensors."""
import ctypes
import os

import numpy as np
import pytest
import torch

from test_gpu_codec import F16, F32, BF16, assert_float_bits_equal, to_dev, to_host

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bc():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import bagua_core
    return bagua_core


CASES = ["normal", "offset", "nan_mixed", "pos_inf", "both_inf", "all_nan", "zeros", "neg_zeros", "constant",
         "huge", "w_inf"]


def inputs(case: str, n: int, dtype: int, seed: int):
    from oracle import oracle_np as NP
    rng = np.random.default_rng(seed)
    v = {k: (rng.standard_normal(n) * 1e-3).astype(np.float32) for k in "twlr"}
    big = {F32: 3e38, F16: 6e4, BF16: 3e38}[dtype]
    t = v["t"]
    if case == "offset":
        t += 7.5
    elif case == "nan_mixed":
        t[::7] = np.nan
    elif case == "pos_inf":
        t[min(5, n - 1)] = np.inf
    elif case == "both_inf":
        t[min(3, n - 1)], t[min(4, n - 1)] = np.inf, -np.inf
    elif case == "all_nan":
        t[:] = np.nan
    elif case == "zeros":
        for k in "twlr":
            v[k][:] = 0.0
    elif case == "neg_zeros":
        for k in "twlr":
            v[k][:] = -0.0
        t[::3] = 0.0
    elif case == "constant":
        for k in "twlr":
            v[k][:] = -0.25
    elif case == "huge":  # max - min overflows: the scale is +0
        t[:] = big
        t[1::2] = -big
    elif case == "w_inf":
        v["w"][min(2, n - 1)] = -np.inf
    return {k: NP.from_f32(a, dtype) for k, a in v.items()}


@pytest.mark.parametrize("dtype", [F32, F16, BF16])
@pytest.mark.parametrize("case", CASES)
def test_ring_one_rank_matches_oracle(bc, oracle_c, dtype, case):
    """Every launch shape of both passes (BAGUA_RING_ONE_RANK_CFG 0-8, _MIX_CFG 0-4, the stored
    mix, a cache-kept tail) on a regular,
    a ragged and a tiny bucket, the edge regimes of the header (NaN, +-inf, all NaN,
    +-0, constant, overflowing max - min) included."""
    from oracle import simulate
    K = bc._native.K
    for n in (5, (1 << 18) + 37, 1 << 20):
        a = inputs(case, n, dtype, seed=n + 3 * dtype + len(case))
        want = simulate.decentralized_low_precision(oracle_c, [a["t"]], [a["w"]], [a["l"]], [a["r"]], dtype)
        wsb = K.bagua_minmax_u8_workspace_bytes(n, 1)
        ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
        shapes = [{"BAGUA_RING_ONE_RANK_CFG": str(c)} for c in range(9)]
        shapes += [{"BAGUA_RING_ONE_RANK_MIX_CFG": str(c)} for c in range(5)]
        shapes += [{"BAGUA_RING_ONE_RANK_RECOMPUTE": "0"}, {"BAGUA_RING_ONE_RANK_KEEP_MIB": "1"}]
        for cfg in shapes:
            os.environ.update(cfg)
            try:
                d = {k: to_dev(a[k], dtype) for k in "twlr"}
                rc = K.bagua_ring_one_rank_minmax(dtype, d["t"].data_ptr(), d["w"].data_ptr(), d["l"].data_ptr(),
                                                  d["r"].data_ptr(), n, ws.data_ptr(), wsb, None)
                assert rc == 0
                for k, wk in zip("twlr", want):
                    assert_float_bits_equal(to_host(d[k], dtype), wk[0], dtype, f"{k} n={n} cfg={cfg} {case}")
            finally:
                for e in cfg:
                    del os.environ[e]


@pytest.mark.parametrize("dtype,n,offset", [(BF16, (1 << 25) + 13, 0), (F32, (1 << 22) + 3, 0), (F16, 30011, 1),
                                            (F32, 1, 0)])
def test_ring_one_rank_through_the_op(bc, dtype, n, offset, monkeypatch):
    """The op at one rank (loopback communicator, p = 1): two-pass path (default) ==
    the four-kernel sequence (BAGUA_ONE_RANK_FUSED=0) on all four tensors, a bucket
    large enough for every workgroup to sweep several batches included; a misaligned
    tensor runs on aligned copies."""
    from bagua_core.communicator import loopback_communicators
    N = bc._native
    comm = loopback_communicators(1, 0)[0]
    a = inputs("normal", max(n, 1), dtype, seed=77 + dtype)
    a = {k: v[:n] for k, v in a.items()}
    out = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("BAGUA_ONE_RANK_FUSED", fused)
        d = {k: to_dev(a[k], dtype, offset) for k in "twlr"}
        torch.cuda.synchronize()
        raws = [bc.BaguaTensorPy(d[k], k).raw() for k in "twlr"]
        N.check(N.C.bagua_decentralized_low_precision_synchronous(comm.handle, *[ctypes.byref(x) for x in raws],
                                                                  N.COMPRESSION_MINMAX_UINT8), "ring op")
        comm.synchronize()
        out[fused] = {k: to_host(d[k], dtype) for k in "twlr"}
    for k in "twlr":
        assert_float_bits_equal(out["1"][k], out["0"][k], dtype, f"{k} n={n}")
