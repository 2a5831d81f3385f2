"""GPU parity of the one-launch MinMax-UInt8 encode (minmax_resident.hip).

bagua_minmax_u8_compress takes this path for whole, fully valid chunks of
>= 12 Mi elements in total (BAGUA_RESIDENT_MIN_ELEMS; lowered to 4 Mi here so
the cases stay small); every case here first asserts that it does
(bagua_minmax_u8_resident_path), then compares every byte of the compressed
buffer with the C oracle (the reference's compress, K:533-571).  Covered:
every dtype, p = 1 / 3 (idle workgroups: the CU count is not a multiple of
3) / 8, a target chunk, ragged chunk sizes (scalar heads and tails), NaN / Inf / signed zeros, every kernel
configuration, the give-up path (timeout 0: workgroups that see an
incomplete exchange re-read the missing slices themselves),
back-to-back launches on one stream (tags advance) and launches on two
streams (separate slots).
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from test_gpu_codec import BF16, F16, F32, STORAGE, TORCH, to_dev

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from bagua_core import _native
    return _native.K


@pytest.fixture
def env():
    saved = {k: os.environ.get(k) for k in ("BAGUA_RESIDENT_CFG", "BAGUA_RESIDENT_TIMEOUT_US", "BAGUA_RESIDENT")}
    yield os.environ
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.fixture(autouse=True)
def small_threshold():
    old = os.environ.get("BAGUA_RESIDENT_MIN_ELEMS")
    os.environ["BAGUA_RESIDENT_MIN_ELEMS"] = str(1 << 22)
    yield
    if old is None:
        os.environ.pop("BAGUA_RESIDENT_MIN_ELEMS", None)
    else:
        os.environ["BAGUA_RESIDENT_MIN_ELEMS"] = old


def make_input(n: int, dtype: int, seed: int, specials: bool = False) -> np.ndarray:
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) * 1e-3).astype(np.float32)
    x[rng.integers(0, n, 64)] = rng.standard_normal(64).astype(np.float32) * 3.0  # outliers set the range
    if specials:
        idx = rng.integers(0, n, 12)
        x[idx[:3]] = np.nan
        x[idx[3:5]] = np.float32(-0.0)
        x[idx[5:7]] = np.float32(0.0)
        x[idx[7]] = np.float32(1e-40)  # denormal
    if dtype == F16:
        return x.astype(np.float16)
    if dtype == BF16:
        return (x.view(np.uint32) >> 16).astype(np.uint16)
    return x


def gpu_compress(K, xt: torch.Tensor, dtype: int, p: int, target: int, stream=None, expect_resident=True):
    n = xt.numel()
    cs = n // p
    S = K.bagua_minmax_u8_compressed_bytes(dtype, cs, p)
    out = torch.full((S,), 0xA5, dtype=torch.uint8, device="cuda")  # poison: every defined byte is written
    wsb = K.bagua_minmax_u8_workspace_bytes(cs, p)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    st = stream or torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    path = K.bagua_minmax_u8_resident_path(dtype, xt.data_ptr(), n, cs, p, out.data_ptr(), S, target, sp)
    assert path == (1 if expect_resident else 0)
    rc = K.bagua_minmax_u8_compress(dtype, xt.data_ptr(), n, cs, p, out.data_ptr(), S, ws.data_ptr(), wsb, target, sp)
    assert rc == 0, rc
    return out, (ws, st)


def check(K, oracle_c, x: np.ndarray, dtype: int, p: int, target: int = -1, offset: int = 0):
    xt = to_dev(x, dtype, offset)
    got_t, _ = gpu_compress(K, xt, dtype, p, target)
    torch.cuda.synchronize()
    got = got_t.cpu().numpy()
    want = oracle_c.compress_minmax_u8(x, dtype, p, target)
    if target >= 0:
        co = got.size // p
        got, want = got[target * co:(target + 1) * co], want[target * co:(target + 1) * co]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"


@pytest.mark.parametrize("dtype", [F32, F16, BF16])
@pytest.mark.parametrize("p,target,cs", [(1, -1, 1 << 22), (3, -1, (1 << 21) + 77), (8, -1, 1 << 19),
                                         (4, 2, (1 << 22) + 4)])
def test_resident_matches_oracle(K, oracle_c, dtype, p, target, cs):
    x = make_input(p * cs, dtype, seed=1000 + 10 * p + dtype)
    check(K, oracle_c, x, dtype, p, target)


@pytest.mark.parametrize("dtype", [F32, BF16])
def test_resident_ragged_chunks_and_specials(K, oracle_c, dtype):
    # chunk c starts at c * cs elements: with this cs every chunk has a scalar
    # head before its 128-B aligned payload line and a scalar tail
    x = make_input(3 * ((1 << 21) + 77), dtype, seed=7, specials=True)
    check(K, oracle_c, x, dtype, 3, -1)


@pytest.mark.parametrize("cfg", range(12))
def test_resident_every_configuration(K, oracle_c, env, cfg):
    env["BAGUA_RESIDENT_CFG"] = str(cfg)
    x = make_input(1 << 23, F32, seed=cfg)
    check(K, oracle_c, x, F32, 2)


@pytest.mark.parametrize("dtype", [F32, F16])
def test_resident_give_up_path(K, oracle_c, env, dtype):
    """timeout 0: a workgroup that does not find every partial on its first
    sweep gives up and folds the missing slices from memory: same bytes."""
    env["BAGUA_RESIDENT_TIMEOUT_US"] = "0"
    for p in (1, 3):
        x = make_input(p * (1 << 22), dtype, seed=40 + p)
        check(K, oracle_c, x, dtype, p)


def test_resident_back_to_back_and_two_streams(K, oracle_c):
    """Tags advance per launch on one stream's slot (every result exact, no
    stale partial is taken), and two streams use separate slots concurrently."""
    xs = [make_input(1 << 22, F32, seed=70 + i) for i in range(4)]
    xts = [to_dev(x, F32) for x in xs]
    s2 = torch.cuda.Stream()
    outs = []
    for i, xt in enumerate(xts):  # mixed shapes on the same slot: p=1 then p=4
        p = 1 if i % 2 == 0 else 4
        st = torch.cuda.current_stream() if i < 2 else s2
        out, keep = gpu_compress(K, xt, F32, p, -1, stream=st)
        outs.append((out, keep, p))
    torch.cuda.synchronize()
    for x, (out, _, p) in zip(xs, outs):
        assert np.array_equal(out.cpu().numpy(), oracle_c.compress_minmax_u8(x, F32, p))


def test_small_and_partial_tensors_take_the_two_pass_encode(K):
    xt = torch.randn(1 << 20, device="cuda")
    gpu_compress(K, xt, F32, 1, -1, expect_resident=False)  # below the size threshold
    n, p = 1 << 23, 2
    xt = torch.randn(n, device="cuda")
    S = K.bagua_minmax_u8_compressed_bytes(F32, n // p, p)
    out = torch.empty(S, dtype=torch.uint8, device="cuda")
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    # num_elements < p * chunk_size (a partially valid last chunk): two-pass encode
    assert K.bagua_minmax_u8_resident_path(F32, xt.data_ptr(), n - 3, n // p, p, out.data_ptr(), S, -1, sp) == 0


def test_resident_decode_round_trip_256mib(K, oracle_c):
    """config 2 shape through the resident encode, then the decode: exact vs the oracle."""
    n = 1 << 26
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    xt = torch.randn(n, device="cuda", generator=g) * 1e-3
    comp, _ = gpu_compress(K, xt, F32, 1, -1)
    y = torch.empty_like(xt)
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert K.bagua_minmax_u8_decompress(F32, comp.data_ptr(), comp.numel(), n, 1, y.data_ptr(), sp) == 0
    xh = xt.cpu().numpy()
    want = oracle_c.compress_minmax_u8(xh, F32, 1)
    assert np.array_equal(comp.cpu().numpy(), want)
    dw = np.empty_like(xh)
    oracle_c.decompress_minmax_u8(want, 1, dw, F32)
    assert np.array_equal(y.cpu().numpy().view(np.uint32), dw.view(np.uint32))


def test_default_size_threshold(K):
    """Default: the two-kernel encode below 12 Mi elements (it is faster there), the
    one-launch encode from 12 Mi on."""
    os.environ.pop("BAGUA_RESIDENT_MIN_ELEMS", None)
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    xt = torch.empty(16 << 20, device="cuda")
    for n, want in ((8 << 20, 0), ((12 << 20) - 1024, 0), (12 << 20, 1), (16 << 20, 1)):
        S = K.bagua_minmax_u8_compressed_bytes(F32, n, 1)
        out = torch.empty(S, dtype=torch.uint8, device="cuda")
        assert K.bagua_minmax_u8_resident_path(F32, xt.data_ptr(), n, n, 1, out.data_ptr(), S, -1, sp) == want, n

