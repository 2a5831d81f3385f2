"""GPU parity of the MinMax-UInt8 codec at the C ABI on the shapes the tensor
API can hand it (DT:313-446): partially valid buckets (input_num_element <
num_chunks * chunk_size, so the last chunks are ragged or hold no valid
element at all), many chunks per call, a target chunk, and chunk sizes that
are not multiples of the vector width.  The output buffer is poisoned, so
every byte the format defines (header, zero gap, payload, slack) must be
written and must equal the C oracle's; the decode must match it bit for bit.
"""
import ctypes

import numpy as np
import pytest
import torch

from test_gpu_codec import BF16, F16, F32, STORAGE, assert_float_bits_equal, bc, to_dev, to_host  # noqa: F401

pytestmark = pytest.mark.gpu


def sample(dtype, n, seed):
    from oracle import oracle_np as NP
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) * 1e-3).astype(np.float32)
    x[rng.integers(0, n, size=max(1, n // 997))] *= 50.0
    return NP.from_f32(x, dtype)


@pytest.mark.parametrize("dtype", [F32, F16, BF16])
@pytest.mark.parametrize("p,cs,n_in,target", [
    (4, 100_003, 3 * 100_003 + 4_321, -1),   # last chunk ragged
    (4, 100_003, 2 * 100_003, -1),           # last two chunks empty
    (3, 65_536 + 7, 5, -1),                  # only the first chunk holds (5) elements
    (64, 1_031, None, -1),                   # many chunks per call
    (5, 200_000 + 3, 4 * 200_003 - 10, 3),   # ragged target chunk
    (5, 200_000 + 3, 4 * 200_003 - 10, 4),   # empty target chunk
    (6, 777, None, 2),                       # small target chunk
    (1, (12 << 20) + 5, None, -1),           # one-launch encode eligible size, odd length
])
def test_minmax_partial_buckets_vs_oracle(bc, oracle_c, dtype, p, cs, n_in, target):
    K = bc._native.K
    n_in = p * cs if n_in is None else n_in
    x = sample(dtype, p * cs, p * 131 + cs)
    want = oracle_c.compress_minmax_u8(x, dtype, p, target, num_elem=n_in)
    S = K.bagua_minmax_u8_compressed_bytes(dtype, cs, p)
    assert S == want.size
    wsb = K.bagua_minmax_u8_workspace_bytes(cs, p)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    out = torch.full((S,), 0xA5, dtype=torch.uint8, device="cuda")
    xd = to_dev(x, dtype)
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert K.bagua_minmax_u8_compress(dtype, xd.data_ptr(), n_in, cs, p, out.data_ptr(), S, ws.data_ptr(), wsb,
                                      target, sp) == 0
    got = out.cpu().numpy()
    if target >= 0:
        co = S // p
        got, want = got[target * co:(target + 1) * co], want[target * co:(target + 1) * co]
        assert np.array_equal(got, want)
        return
    assert np.array_equal(got, want)
    # decode of the whole buffer: every element, valid or not, as the oracle decodes it
    y = torch.empty(p * cs, dtype=xd.dtype, device="cuda")
    assert K.bagua_minmax_u8_decompress(dtype, out.data_ptr(), S, cs, p, y.data_ptr(), sp) == 0
    dw = np.empty(p * cs, dtype=STORAGE[dtype])
    oracle_c.decompress_minmax_u8(want, p, dw, dtype)
    assert_float_bits_equal(to_host(y, dtype), dw, dtype, "decode")


def test_minmax_partial_goldens(bc, goldens):
    """The committed partially valid cases (tests/golden/gen_golden.py, both
    oracles agree): elements past input_num_element are outside the chunk's
    min/max (K:538-545) but quantised with it (K:468-472); an empty chunk
    carries the init header and bytes 255."""
    K = bc._native.K
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for i in range(int(goldens["counts"][5])):
        dtype, p, cs, target, n_in = (int(v) for v in goldens[f"mmp_meta_{i}"])
        x = goldens[f"mmp_in_{i}"].view(STORAGE[dtype])
        want = goldens[f"mmp_comp_{i}"]
        S = K.bagua_minmax_u8_compressed_bytes(dtype, cs, p)
        assert S == want.size
        wsb = K.bagua_minmax_u8_workspace_bytes(cs, p)
        ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
        out = torch.full((S,), 0xA5, dtype=torch.uint8, device="cuda")
        xd = to_dev(x, dtype)
        assert K.bagua_minmax_u8_compress(dtype, xd.data_ptr(), n_in, cs, p, out.data_ptr(), S, ws.data_ptr(), wsb,
                                          target, sp) == 0
        got = out.cpu().numpy()
        if target >= 0:
            co = S // p
            assert np.array_equal(got[target * co:(target + 1) * co], want[target * co:(target + 1) * co]), f"case {i}"
            continue
        assert np.array_equal(got, want), f"case {i}"
        y = torch.empty(p * cs, dtype=xd.dtype, device="cuda")
        assert K.bagua_minmax_u8_decompress(dtype, out.data_ptr(), S, cs, p, y.data_ptr(), sp) == 0
        assert_float_bits_equal(to_host(y, dtype), goldens[f"mmp_dec_{i}"].view(STORAGE[dtype]), dtype,
                                f"case {i} decode")
