"""GPU parity tests of the 1-bit encode (onebit_encode_kernel + onebit_finalize_kernel,
the scale tree of DESIGN.md §4) against the C oracle, bit-exact on every byte.

The cases aim at the tree and the tile bookkeeping: level-1 groups (1024
tiles) that end ragged, chunks whose valid tiles end inside a group (explicit
input_num_element < p * chunk_size), chunks with no valid element, level-2 and
level-3 trees (a single 2^31 - 32 element chunk), target chunks, many chunks
per launch, and back-to-back launches of different shapes on one stream and
on two streams.  The output buffer is poisoned: every defined byte must be
written.  (A one-launch variant that folded the finalize into the encode with
arrival counters was bit-identical on these cases but no faster:
profiles/r01_onebit_fused_finalize_ab.jsonl.)
"""
import ctypes

import numpy as np
import pytest
import torch

from test_gpu_codec import BF16, F32, bc, to_dev  # noqa: F401  (fixture re-export)

pytestmark = pytest.mark.gpu


def oracle_compress(oracle_c, x, dtype, n_in, cs, p, target=-1):
    """orc_compress_onebit with an explicit valid-element count (ragged input)."""
    size = oracle_c.onebit_compressed_size(p, cs)
    out = np.zeros(size, dtype=np.uint8)
    rc = oracle_c.lib().orc_compress_onebit(oracle_c._ptr(x), dtype, n_in, cs, p, oracle_c._ptr(out), size, target)
    assert rc == 0, rc
    return out


def gpu_compress(bc, xd, dtype, n_in, cs, p, target=-1, stream=None, out=None):
    K = bc._native.K
    S = K.bagua_onebit_compressed_bytes(cs, p)
    wsb = K.bagua_onebit_workspace_bytes(cs, p)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    if out is None:
        out = torch.full((S,), 0xA5, dtype=torch.uint8, device="cuda")  # poisoned: every byte must be written
    s = None if stream is None else ctypes.c_void_p(stream.cuda_stream)
    rc = K.bagua_onebit_compress(dtype, xd.data_ptr(), n_in, cs, p, out.data_ptr(), S, ws.data_ptr(), wsb, target, s)
    assert rc == 0, rc
    return out, ws


def sample(dtype, n, seed):
    from oracle import oracle_np as NP
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) * 1e-3).astype(np.float32)
    x[rng.integers(0, n, size=max(1, n // 1000))] *= -1e3  # a few large magnitudes
    return NP.from_f32(x, dtype)


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("p,cs,n_in,target", [
    (1, 1024 * 1024 * 3 + 517, None, -1),   # 3 full groups + a ragged fourth
    (1, 1024 * 1024 + 1024 * 7, None, -1),  # range shapes that straddle group edges
    (3, 1024 * 1500 + 3, None, -1),         # several chunks per launch
    (4, 1024 * 2100, 1024 * 2100 * 3 + 1024 * 900 + 5, -1),  # ragged: the last chunk ends inside group 0
    (4, 1024 * 2100, 1024 * 2100 * 2, -1),  # the last two chunks hold no valid element
    (5, 1024 * 1300 + 11, None, 3),         # target chunk
    (2, 700, None, -1),                     # less than one tile per chunk
    (64, 1024 * 33 + 1, None, -1),          # many chunks, ranges of a few tiles
])
def test_fused_encode_vs_oracle(bc, oracle_c, dtype, p, cs, n_in, target):
    n_in = p * cs if n_in is None else n_in
    x = sample(dtype, p * cs, cs + p)
    want = oracle_compress(oracle_c, x, dtype, n_in, cs, p, target)
    got, _ = gpu_compress(bc, to_dev(x, dtype), dtype, n_in, cs, p, target)
    torch.cuda.synchronize()
    g = got.cpu().numpy()
    if target >= 0:  # only the target segment (and nothing else) is defined
        co = g.size // p
        g, want = g[target * co:(target + 1) * co], want[target * co:(target + 1) * co]
    assert np.array_equal(g, want)


def test_back_to_back_shapes_one_stream(bc, oracle_c):
    """Launches of different shapes queued on one stream without a host sync."""
    shapes = [(1, 1024 * 2048 + 99), (3, 1024 * 1025), (1, 5000), (2, 1024 * 3000 + 1), (1, 1024 * 2048 + 99)]
    xs, outs = [], []
    for i, (p, cs) in enumerate(shapes):
        x = sample(F32, p * cs, 100 + i)
        xd = to_dev(x, F32)
        xs.append((x, p, cs))
        outs.append(gpu_compress(bc, xd, F32, p * cs, cs, p) + (xd,))
    torch.cuda.synchronize()
    for (x, p, cs), (got, _, _) in zip(xs, outs):
        assert np.array_equal(got.cpu().numpy(), oracle_compress(oracle_c, x, F32, p * cs, cs, p))


def test_two_streams_concurrently(bc, oracle_c):
    """Two streams encode different buckets at the same time (separate workspaces)."""
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    cases = [(1, 1024 * 4096 + 3, s1), (2, 1024 * 2049, s2), (1, 1024 * 1024 * 2, s1), (4, 1024 * 700, s2)]
    xs = [sample(F32, p * cs, 200 + i) for i, (p, cs, _) in enumerate(cases)]
    xds = [to_dev(x, F32) for x in xs]
    torch.cuda.synchronize()
    res = []
    for x, xd, (p, cs, st) in zip(xs, xds, cases):
        with torch.cuda.stream(st):
            res.append(gpu_compress(bc, xd, F32, p * cs, cs, p, stream=st))
    torch.cuda.synchronize()
    for x, (p, cs, _), (got, _) in zip(xs, cases, res):
        assert np.array_equal(got.cpu().numpy(), oracle_compress(oracle_c, x, F32, p * cs, cs, p))


def test_level3_tree_maximum_chunk(bc, oracle_c):
    """A single chunk of 2^31 - 32 fp32 elements: 2^21 tiles in 2048 level-1
    groups, so the scale takes the level-2 AND level-3 nodes of the tree."""
    n = (1 << 31) - 32
    g = torch.Generator(device="cuda").manual_seed(77)
    x = torch.randn(n, device="cuda", generator=g)
    got, _ = gpu_compress(bc, x, F32, n, n, 1)
    torch.cuda.synchronize()
    xh = x.cpu().numpy()
    del x
    want = oracle_compress(oracle_c, xh, F32, n, n, 1)
    assert np.array_equal(got.cpu().numpy(), want)


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("average", [1, 0])
@pytest.mark.parametrize("p", list(range(1, 17)))
def test_reduce_requantize_every_p(bc, oracle_c, dtype, average, p):
    """The 1-bit fused middle step (onebit_reduce_encode_lut_kernel: p <= 2 direct
    index, p <= 8 one 2^p table, 9 <= p <= 16 two half-tree tables) for every p and
    both reductions: the re-encoded target segment equals the oracle's
    decompress -> reduce_{mean,sum} -> compress(target), and the stored reduced
    chunk equals the oracle's reduced chunk.  cs is ragged (last tile partial)."""
    from oracle import oracle_np as NP
    K = bc._native.K
    cs = 1024 * 37 + 300
    target = p // 2
    rng = np.random.default_rng(1000 + 10 * p + average + dtype)
    x = NP.from_f32((rng.standard_normal(p * cs) * 1e-3 * (1 + rng.random(p * cs))).astype(np.float32), dtype)
    recv = oracle_compress(oracle_c, x, dtype, p * cs, cs, p)  # p segments, one scale each
    t = np.zeros_like(x)
    oracle_c.decompress_onebit(recv, p, t, dtype)
    oracle_c.reduce_chunks(t, dtype, p, target, bool(average))
    want = oracle_c.compress_onebit(t, dtype, p, target)
    S = recv.size
    co = S // p
    rd = torch.from_numpy(recv.copy()).cuda()
    out = torch.full((S,), 0xA5, dtype=torch.uint8, device="cuda")
    td = torch.zeros(p * cs, dtype=torch.float32 if dtype == F32 else torch.bfloat16, device="cuda")
    wsb = K.bagua_onebit_workspace_bytes(cs, 1)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    rc = K.bagua_onebit_reduce_requantize(dtype, rd.data_ptr(), S, cs, p, td.data_ptr(), average, out.data_ptr(), S,
                                          target, ws.data_ptr(), wsb, None)
    assert rc == 0, rc
    torch.cuda.synchronize()
    g = out.cpu().numpy()
    assert np.array_equal(g[target * co:(target + 1) * co], want[target * co:(target + 1) * co])
    got_chunk = td.view(torch.int32 if dtype == F32 else torch.int16).cpu().numpy()[target * cs:(target + 1) * cs]
    assert np.array_equal(got_chunk.view(np.uint8), t[target * cs:(target + 1) * cs].view(np.uint8))
