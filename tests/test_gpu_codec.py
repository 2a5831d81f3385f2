"""GPU parity tests: the HIP codec (through the C ABI and the BaguaTensorPy
surface) against the oracle, bit-exact on every defined byte.

Tolerance policy: uint8 payloads, headers and every decoded/reduced float are
compared BIT-EXACT (NaN compared as NaN-ness).  The float tolerance stated
in DESIGN.md §3 is a property of the format, checked on the oracle
(tests/test_oracle.py::test_dequantisation_error_bound) and again at full
size here.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

F32, F16, BF16 = 0, 1, 2
PIECES_FOLDED = 0x40000  # bagua_kernels.h BAGUA_PIECES_FOLDED
PIECES_TABLES = 0x80000  # bagua_kernels.h BAGUA_PIECES_TABLES
STORAGE = {F32: np.float32, F16: np.float16, BF16: np.uint16}
TORCH = {F32: torch.float32, F16: torch.float16, BF16: torch.bfloat16}


@pytest.fixture(scope="module")
def bc():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    import bagua_core
    return bagua_core


def to_dev(x: np.ndarray, dtype: int, offset: int = 0) -> torch.Tensor:
    """Copy a host array to the GPU; `offset` elements of padding in front
    make the tensor's data pointer deliberately misaligned."""
    if dtype == BF16:
        h = torch.from_numpy(x.view(np.int16).copy()).view(torch.bfloat16)
    else:
        h = torch.from_numpy(x.copy())
    buf = torch.zeros(x.size + offset, dtype=TORCH[dtype], device="cuda")
    buf[offset:].copy_(h.to("cuda"))
    return buf[offset:]


def to_host(t: torch.Tensor, dtype: int) -> np.ndarray:
    torch.cuda.synchronize()
    if dtype == BF16:
        return t.view(torch.int16).cpu().numpy().view(np.uint16)
    return t.cpu().numpy()


def assert_float_bits_equal(got: np.ndarray, want: np.ndarray, dtype: int, what: str):
    g = got.view(STORAGE[dtype])
    w = want.view(STORAGE[dtype])
    if dtype == BF16:
        gf = (g.astype(np.uint32) << 16).view(np.float32)
        wf = (w.astype(np.uint32) << 16).view(np.float32)
    else:
        gf, wf = g.astype(np.float32), w.astype(np.float32)
    gn, wn = np.isnan(gf), np.isnan(wf)
    assert np.array_equal(gn, wn), f"{what}: NaN positions differ"
    bits = np.uint32 if dtype == F32 else np.uint16
    gb, wb = g.view(bits)[~gn], w.view(bits)[~wn]
    bad = np.nonzero(gb != wb)[0]
    assert bad.size == 0, f"{what}: {bad.size} values differ, first at {bad[:5]}: {gb[bad[:3]]} vs {wb[bad[:3]]}"


def segment_bytes(buf: np.ndarray, p: int, which: int) -> np.ndarray:
    co = buf.size // p
    return buf[which * co:(which + 1) * co]


# ---------------------------------------------------------------- MinMax ----
def test_minmax_goldens(bc, goldens):
    n = int(goldens["counts"][0])
    for i in range(n):
        dtype, p, cs, target, _ = (int(v) for v in goldens[f"mm_meta_{i}"])
        x = goldens[f"mm_in_{i}"].view(STORAGE[dtype])
        t = bc.BaguaTensorPy(to_dev(x, dtype), f"g{i}")
        comp = t.compress("MinMaxUInt8", p, target)
        got = comp.to_numpy_u8()
        want = goldens[f"mm_comp_{i}"]
        assert got.size == want.size
        if target == -1:
            assert np.array_equal(got, want), f"case {i}: payload/header differs"
            out = torch.empty(p * cs, dtype=TORCH[dtype], device="cuda")
            bc.BaguaTensorPy(out, "o").decompress_from("MinMaxUInt8", p, comp)
            assert_float_bits_equal(to_host(out, dtype), goldens[f"mm_dec_{i}"], dtype, f"case {i} decode")
        else:
            assert np.array_equal(segment_bytes(got, p, target), segment_bytes(want, p, target)), f"case {i}"


@pytest.mark.parametrize("dtype", [F32, F16, BF16])
@pytest.mark.parametrize("p,cs,offset", [(1, 1, 0), (1, 3, 1), (1, 4096 * 4 + 3, 0), (2, 12345, 1), (3, 1001, 2),
                                         (4, 65536, 0), (8, 4099, 3), (5, 7, 0), (16, 2048, 1), (1, 1 << 20, 0)])
def test_minmax_random_shapes(bc, oracle_c, dtype, p, cs, offset):
    from oracle import oracle_np as NP
    rng = np.random.default_rng(p * 1000003 + cs + dtype)
    xf = (rng.standard_normal(p * cs) * 1e-2 + rng.standard_normal()).astype(np.float32)
    x = NP.from_f32(xf, dtype)
    want = oracle_c.compress_minmax_u8(x, dtype, p)
    t = bc.BaguaTensorPy(to_dev(x, dtype, offset), "x")
    comp = t.compress("MinMaxUInt8", p, -1)
    assert np.array_equal(comp.to_numpy_u8(), want)
    dec_want = np.zeros_like(x)
    oracle_c.decompress_minmax_u8(want, p, dec_want, dtype)
    out = to_dev(np.zeros_like(x), dtype, offset)
    bc.BaguaTensorPy(out, "o").decompress_from("MinMaxUInt8", p, comp)
    assert_float_bits_equal(to_host(out, dtype), dec_want, dtype, "decode")
    # target-chunk mode writes exactly that segment
    tgt = p - 1
    c2 = t.compress("MinMaxUInt8", p, tgt).to_numpy_u8()
    assert np.array_equal(segment_bytes(c2, p, tgt), segment_bytes(want, p, tgt))


def test_v1_abi_compress_decompress(bc, oracle_c):
    """The reference's exact extern "C" entry points (bagua_kernels.cu:661-689)."""
    K = bc._native.K
    rng = np.random.default_rng(11)
    p, cs = 4, 50000
    x = (rng.standard_normal(p * cs) * 1e-3).astype(np.float32)
    xt = to_dev(x, F32)
    S = K.bagua_minmax_u8_compressed_bytes(F32, cs, p)
    out = torch.empty(S, dtype=torch.uint8, device="cuda")
    tmp_bytes = K.array_min_max_size_f32_host(xt.data_ptr(), x.size, out.data_ptr(), None)
    tmp = torch.empty(tmp_bytes, dtype=torch.uint8, device="cuda")
    K.compress_f32_to_uint8_host(xt.data_ptr(), x.size, cs, p, out.data_ptr(), S, tmp.data_ptr(), tmp_bytes, -1, None)
    want = oracle_c.compress_minmax_u8(x, F32, p)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), want)
    dec = torch.empty(p * cs, dtype=torch.float32, device="cuda")
    K.decompress_uint8_to_f32_host(out.data_ptr(), S, cs, p, dec.data_ptr(), None)
    dw = np.zeros_like(x)
    oracle_c.decompress_minmax_u8(want, p, dw, F32)
    assert_float_bits_equal(to_host(dec, F32), dw, F32, "v1 decode")


@pytest.mark.parametrize("dtype,p,cs,pieces,offset", [(F32, 4, 65536 + 77, 3, 0), (BF16, 3, 40000, 4, 1),
                                                      (F16, 2, 1536, 4, 0), (F32, 1, 5000, 7, 2)])
def test_minmax_range_entry_points_misaligned(bc, oracle_c, dtype, p, cs, pieces, offset):
    """stage-1 partials + quantize_range per piece == one compress; decompress_range per piece == one decode
    (misaligned data pointers, F16, odd chunk sizes, ragged pieces at p = 1; K:455-500)."""
    from oracle import oracle_np as NP
    K = bc._native.K
    rng = np.random.default_rng(cs + pieces)
    x = NP.from_f32((rng.standard_normal(p * cs) * 1e-2 + 0.3).astype(np.float32), dtype)
    want = oracle_c.compress_minmax_u8(x, dtype, p)
    xt = to_dev(x, dtype, offset)
    S = K.bagua_minmax_u8_compressed_bytes(dtype, cs, p)
    out = torch.full((S,), 0xAB, dtype=torch.uint8, device="cuda")
    wsb = K.bagua_minmax_u8_workspace_bytes(cs, p)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    N = bc._native
    N.check(K.bagua_minmax_u8_compress_stage(1, dtype, xt.data_ptr(), x.size, cs, p, out.data_ptr(), S,
                                             ws.data_ptr(), wsb, -1, None), "stage 1")
    b, e = ctypes.c_int(), ctypes.c_int()
    ranges = []
    for q in range(pieces):
        N.check(K.bagua_minmax_u8_piece_range(cs, pieces, q, ctypes.byref(b), ctypes.byref(e)), "range")
        ranges.append((b.value, e.value))
    for q in reversed(range(pieces)):  # any order: pieces are disjoint
        N.check(K.bagua_minmax_u8_quantize_range(dtype, xt.data_ptr(), x.size, cs, p, out.data_ptr(), S, ws.data_ptr(),
                                                 wsb, -1, ranges[q][0], ranges[q][1], None), f"piece {q}")
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), want)
    dec_want = np.zeros_like(x)
    oracle_c.decompress_minmax_u8(want, p, dec_want, dtype)
    dec = to_dev(np.zeros_like(x), dtype, offset)
    for q in range(pieces):
        N.check(K.bagua_minmax_u8_decompress_range(dtype, out.data_ptr(), S, cs, p, dec.data_ptr(), ranges[q][0],
                                                   ranges[q][1], None), f"decode piece {q}")
    assert_float_bits_equal(to_host(dec, dtype), dec_want, dtype, "piecewise decode")


def test_invalid_arguments_are_reported(bc):
    t = bc.BaguaTensorPy(torch.zeros(10, device="cuda"), "x")
    with pytest.raises(RuntimeError):
        t.compress("MinMaxUInt8", 3, -1)  # 10 % 3 != 0 (datatypes/mod.rs:322-326)
    with pytest.raises(NotImplementedError):
        t.compress("TopK", 1, -1)
    K = bc._native.K
    assert K.bagua_minmax_u8_compress(F32, None, 0, 0, 0, None, 0, None, 0, -1, None) == 1
    assert K.bagua_minmax_u8_compress(F32, t.data_ptr(), 10, 10, 1, t.data_ptr(), 64, None, 0, -1, None) == 2
    assert K.bagua_minmax_u8_compress(F32, t.data_ptr(), 10, 10, 1, t.data_ptr(), 41, t.data_ptr(), 64, -1,
                                      None) == 1  # output smaller than chunk_size + 32


# ---------------------------------------------------------------- reduce ----
def test_reduce_goldens(bc, goldens):
    K = bc._native.K
    for i in range(int(goldens["counts"][1])):
        dtype, p, cs, target, avg = (int(v) for v in goldens[f"red_meta_{i}"])
        x = goldens[f"red_in_{i}"].view(STORAGE[dtype])
        xt = to_dev(x, dtype)
        assert K.bagua_reduce_chunks(dtype, xt.data_ptr(), cs, p, target, avg, None) == 0
        assert_float_bits_equal(to_host(xt, dtype), goldens[f"red_out_{i}"], dtype, f"reduce case {i}")


@pytest.mark.parametrize("dtype", [F32, F16, BF16])
@pytest.mark.parametrize("p,ragged", [(1, 0), (2, 0), (3, 0), (4, 0), (8, 0), (12, 0), (16, 0), (1, 3), (2, 5),
                                      (4, 1)])
@pytest.mark.parametrize("mode", ["store", "none", "final", "final_noseg"])
@pytest.mark.parametrize("average", [1, 0])
def test_fused_reduce_requantize(bc, oracle_c, dtype, p, ragged, mode, average):
    """bagua_minmax_u8_reduce_requantize == decompress_from + reduce_{mean,sum} + compress(target);
    with a NULL tensor (the reduced chunk recomputed, never stored) the same segment bytes and
    nothing of the tensor written; _final: the same bytes, and the own chunk of the tensor holds
    the decompressed requantised chunk (the op's final decompress there), nothing else written."""
    store = mode == "store"
    from oracle import oracle_np as NP
    rng = np.random.default_rng(100 + p + dtype)
    cs = 40000 + 8 * p + ragged  # ragged: a tail of < one 16-B vector of elements
    xs = [NP.from_f32((rng.standard_normal(p * cs) * 1e-3).astype(np.float32), dtype) for _ in range(p)]
    # the alltoall receive buffer of rank `r`: slot j = rank j's segment r
    r = p // 2
    comps = [oracle_c.compress_minmax_u8(x, dtype, p) for x in xs]
    S = comps[0].size
    co = S // p
    recv = np.concatenate([c[r * co:(r + 1) * co] for c in comps])
    # oracle: decompress, reduce into chunk r, compress target r
    t_want = np.zeros(p * cs, STORAGE[dtype])
    oracle_c.decompress_minmax_u8(recv, p, t_want, dtype)
    oracle_c.reduce_chunks(t_want, dtype, p, r, bool(average))
    send_want = np.zeros(S, np.uint8)
    oracle_c.compress_minmax_u8(t_want, dtype, p, r, out=send_want)
    # GPU (segments are poisoned: header gap and slack must be written as zeros)
    K = bc._native.K
    recv_d = torch.from_numpy(recv).cuda()
    t_d = torch.full((p * cs,), 7.0, dtype=TORCH[dtype], device="cuda")
    send_d = torch.full((S,), 0xA5, dtype=torch.uint8, device="cuda")
    ws = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
    if mode.startswith("final"):
        seg = mode == "final"
        rc = K.bagua_minmax_u8_reduce_requantize_final(dtype, recv_d.data_ptr(), S, cs, p, t_d.data_ptr(), average,
                                                       send_d.data_ptr() if seg else None, S if seg else 0, r,
                                                       ws.data_ptr(), ws.numel(), None)
    else:
        rc = K.bagua_minmax_u8_reduce_requantize(dtype, recv_d.data_ptr(), S, cs, p,
                                                 t_d.data_ptr() if store else None, average, send_d.data_ptr(), S, r,
                                                 ws.data_ptr(), ws.numel(), None)
    if mode != "none" and (r * cs * t_d.element_size()) % 16:
        assert rc == 4  # BAGUA_ERR_UNSUPPORTED: no vector path into a misaligned chunk (callers run unfused)
        return
    assert rc == 0
    got_t = to_host(t_d, dtype)
    untouched = np.ones(p * cs, bool)
    if store:
        assert_float_bits_equal(got_t[r * cs:(r + 1) * cs], t_want[r * cs:(r + 1) * cs], dtype, "reduced chunk")
        untouched[r * cs:(r + 1) * cs] = False
    elif mode.startswith("final"):
        final_want = np.zeros(p * cs, STORAGE[dtype])
        oracle_c.decompress_minmax_u8(send_want, p, final_want, dtype)
        assert_float_bits_equal(got_t[r * cs:(r + 1) * cs], final_want[r * cs:(r + 1) * cs], dtype, "final chunk")
        untouched[r * cs:(r + 1) * cs] = False
    rest = got_t[untouched]
    assert np.all(rest.astype(np.float32) == 7.0) if dtype != BF16 else np.all(rest == 0x40E0)
    got = send_d.cpu().numpy()
    if mode == "final_noseg":
        assert np.all(got == 0xA5), "no segment byte may be written without an output buffer"
        return
    assert np.array_equal(got[r * co:(r + 1) * co], send_want[r * co:(r + 1) * co])
    other = np.ones(S, bool)
    other[r * co:(r + 1) * co] = False
    assert np.all(got[other] == 0xA5), "bytes outside the target segment written"


def recompute_middle(K, dtype, recv_d, S, cs, p, r, pieces, ws, send_want, t_untouched=False, prefold=False):
    """bagua_minmax_u8_reduce_piece(tensor = NULL) per piece, then
    bagua_minmax_u8_reduce_requantize_piece per piece (reverse order; with `prefold` after
    bagua_minmax_u8_fold_piece_partials, as PIECES_FOLDED): segment r equals the
    oracle's decompress + reduce_mean + compress(target), no other byte is written."""
    co = S // p
    send_d = torch.full((S,), 0xA5, dtype=torch.uint8, device="cuda")
    n = pieces & 0xFFFF
    for q in range(n):
        assert K.bagua_minmax_u8_reduce_piece(dtype, recv_d.data_ptr(), S, cs, p, None, 1, r, pieces, q,
                                              ws.data_ptr(), ws.numel(), None) == 0
    rq = pieces
    if prefold:
        assert K.bagua_minmax_u8_fold_piece_partials(dtype, cs, pieces, ws.data_ptr(), ws.numel(), None) == 0
        rq = pieces | PIECES_FOLDED
    for q in reversed(range(n)):
        assert K.bagua_minmax_u8_reduce_requantize_piece(dtype, recv_d.data_ptr(), S, cs, p, 1, send_d.data_ptr(), S,
                                                         r, rq, q, ws.data_ptr(), ws.numel(), None) == 0
    got = send_d.cpu().numpy()
    assert np.array_equal(got[r * co:(r + 1) * co], send_want[r * co:(r + 1) * co]), (p, pieces)
    assert np.all(np.delete(got, np.s_[r * co:(r + 1) * co]) == 0xA5)


@pytest.mark.parametrize("dtype", [F32, F16, BF16])
@pytest.mark.parametrize("p,pieces", [(1, 3), (2, 4), (4, 2), (8, 5), (3, 3), (16, 4)])
def test_minmax_piecewise_building_blocks(bc, oracle_c, dtype, p, pieces):
    """The pipelined op's MinMax building blocks reproduce the unpieced bytes: quantize_range over
    every piece (after the stage-1 partials) == compress; reduce_piece + requantize_piece over every
    piece (requantised in reverse order) == decompress + reduce_mean + compress(target);
    decompress_range over every piece == decompress."""
    from oracle import oracle_np as NP
    K = bc._native.K
    rng = np.random.default_rng(700 + p + pieces + dtype)
    cs = 512 * 7 * pieces + 8 * p  # trailing pieces of different length, 16-B vectors throughout
    xs = [NP.from_f32((rng.standard_normal(p * cs) * 1e-3).astype(np.float32), dtype) for _ in range(p)]
    r = p - 1
    comps = [oracle_c.compress_minmax_u8(x, dtype, p) for x in xs]
    S = comps[0].size
    co = S // p
    ws = torch.empty(K.bagua_minmax_u8_pipeline_workspace_bytes(cs, pieces) + (1 << 20), dtype=torch.uint8,
                     device="cuda")
    # 1. compress, piece by piece
    x_d = to_dev(xs[0], dtype)
    out_d = torch.full((S,), 0xA5, dtype=torch.uint8, device="cuda")
    assert K.bagua_minmax_u8_compress_stage(5, dtype, x_d.data_ptr(), p * cs, cs, p, out_d.data_ptr(), S,
                                            ws.data_ptr(), ws.numel(), -1, None) == 0
    for q in range(pieces):
        b, e = ctypes.c_int(), ctypes.c_int()
        assert K.bagua_minmax_u8_piece_range(cs, pieces, q, ctypes.byref(b), ctypes.byref(e)) == 0
        if q == 0 or b.value < e.value:
            assert K.bagua_minmax_u8_quantize_range(dtype, x_d.data_ptr(), p * cs, cs, p, out_d.data_ptr(), S,
                                                    ws.data_ptr(), ws.numel(), -1, b.value, e.value, None) == 0
    assert np.array_equal(out_d.cpu().numpy(), comps[0])
    # 2. middle step, piece by piece
    recv = np.concatenate([c[r * co:(r + 1) * co] for c in comps])
    t_want = np.zeros(p * cs, STORAGE[dtype])
    oracle_c.decompress_minmax_u8(recv, p, t_want, dtype)
    oracle_c.reduce_chunks(t_want, dtype, p, r, True)
    send_want = np.zeros(S, np.uint8)
    oracle_c.compress_minmax_u8(t_want, dtype, p, r, out=send_want)
    recv_d = torch.from_numpy(recv).cuda()
    t_d = torch.zeros(p * cs, dtype=TORCH[dtype], device="cuda")
    send_d = torch.full((S,), 0xA5, dtype=torch.uint8, device="cuda")
    for q in range(pieces):
        assert K.bagua_minmax_u8_reduce_piece(dtype, recv_d.data_ptr(), S, cs, p, t_d.data_ptr(), 1, r, pieces, q,
                                              ws.data_ptr(), ws.numel(), None) == 0
    for q in reversed(range(pieces)):
        assert K.bagua_minmax_u8_requantize_piece(dtype, t_d.data_ptr(), cs, p, send_d.data_ptr(), S, r, pieces, q,
                                                  ws.data_ptr(), ws.numel(), None) == 0
    got = send_d.cpu().numpy()
    assert np.array_equal(got[r * co:(r + 1) * co], send_want[r * co:(r + 1) * co])
    assert np.all(np.delete(got, np.s_[r * co:(r + 1) * co]) == 0xA5)
    # 2b. the op's default middle step: partials-only reduce pieces, then every piece
    # requantised straight from the received segments (tensor untouched), same bytes
    recompute_middle(K, dtype, recv_d, S, cs, p, r, pieces, ws, send_want, t_untouched=True)
    recompute_middle(K, dtype, recv_d, S, cs, p, r, pieces, ws, send_want, prefold=True)
    # as the op runs it: later pieces and the requantise copy piece 0's tables
    recompute_middle(K, dtype, recv_d, S, cs, p, r, pieces | PIECES_TABLES, ws, send_want)
    if pieces >= 3:  # the tapered schedule (first and last piece half size)
        recompute_middle(K, dtype, recv_d, S, cs, p, r, pieces | bc._native.PIECES_TAPERED, ws, send_want)
    # the storing pair with the partials folded once (PIECES_FOLDED) and piece 0's tables
    # copied by the later pieces (PIECES_TABLES)
    t2 = torch.zeros(p * cs, dtype=TORCH[dtype], device="cuda")
    send2 = torch.full((S,), 0xA5, dtype=torch.uint8, device="cuda")
    for q in range(pieces):
        assert K.bagua_minmax_u8_reduce_piece(dtype, recv_d.data_ptr(), S, cs, p, t2.data_ptr(), 1, r,
                                              pieces | PIECES_TABLES, q, ws.data_ptr(), ws.numel(), None) == 0
    t2_want = np.zeros(p * cs, STORAGE[dtype])
    oracle_c.decompress_minmax_u8(recv, p, t2_want, dtype)
    oracle_c.reduce_chunks(t2_want, dtype, p, r, True)
    assert_float_bits_equal(to_host(t2, dtype)[r * cs:(r + 1) * cs], t2_want[r * cs:(r + 1) * cs], dtype,
                            "reduced chunk with copied tables")
    assert K.bagua_minmax_u8_fold_piece_partials(dtype, cs, pieces, ws.data_ptr(), ws.numel(), None) == 0
    for q in range(pieces):
        assert K.bagua_minmax_u8_requantize_piece(dtype, t2.data_ptr(), cs, p, send2.data_ptr(), S, r,
                                                  pieces | PIECES_FOLDED, q, ws.data_ptr(), ws.numel(), None) == 0
    got2 = send2.cpu().numpy()
    assert np.array_equal(got2[r * co:(r + 1) * co], send_want[r * co:(r + 1) * co])
    # 3. decompress, piece by piece
    y_d = torch.zeros(p * cs, dtype=TORCH[dtype], device="cuda")
    for q in range(pieces):
        b, e = ctypes.c_int(), ctypes.c_int()
        assert K.bagua_minmax_u8_piece_range(cs, pieces, q, ctypes.byref(b), ctypes.byref(e)) == 0
        if b.value < e.value:
            assert K.bagua_minmax_u8_decompress_range(dtype, out_d.data_ptr(), S, cs, p, y_d.data_ptr(), b.value,
                                                      e.value, None) == 0
    y_want = np.zeros(p * cs, STORAGE[dtype])
    oracle_c.decompress_minmax_u8(comps[0], p, y_want, dtype)
    assert_float_bits_equal(to_host(y_d, dtype), y_want, dtype, "piecewise decompress")


# ---------------------------------------------------------------- 1-bit -----
def test_onebit_goldens(bc, goldens):
    for i in range(int(goldens["counts"][2])):
        dtype, p, cs, _ = (int(v) for v in goldens[f"ob_meta_{i}"])
        if goldens[f"ob_in_{i}"].size == 0:
            continue
        x = goldens[f"ob_in_{i}"].view(STORAGE[dtype])
        t = bc.BaguaTensorPy(to_dev(x, dtype), "x")
        comp = t.compress("OneBitSignScale", p, -1)
        assert np.array_equal(comp.to_numpy_u8(), goldens[f"ob_comp_{i}"]), f"onebit case {i}"
        out = torch.empty(p * cs, dtype=TORCH[dtype], device="cuda")
        bc.BaguaTensorPy(out, "o").decompress_from("OneBitSignScale", p, comp)
        assert_float_bits_equal(to_host(out, dtype), goldens[f"ob_dec_{i}"], dtype, f"onebit decode {i}")


@pytest.mark.parametrize("dtype", [F32, F16, BF16])
@pytest.mark.parametrize("p", [1, 2, 3, 4, 5, 8, 16])
@pytest.mark.parametrize("store", [True, False])
def test_onebit_fused_reduce_requantize(bc, oracle_c, dtype, p, store):
    """bagua_onebit_reduce_requantize == decompress_from + reduce_mean + compress(target); with a
    NULL tensor the same segment is encoded and nothing of the tensor is written."""
    from oracle import oracle_np as NP
    rng = np.random.default_rng(300 + p + dtype)
    cs = 3 * 1024 + 8 * p + 5  # ragged last tile
    xs = [NP.from_f32((rng.standard_normal(p * cs) * 1e-3 + 1e-4).astype(np.float32), dtype) for _ in range(p)]
    r = p - 1
    comps = [oracle_c.compress_onebit(x, dtype, p) for x in xs]
    S = comps[0].size
    co = S // p
    recv = np.concatenate([c[r * co:(r + 1) * co] for c in comps])
    t_want = np.zeros(p * cs, STORAGE[dtype])
    oracle_c.decompress_onebit(recv, p, t_want, dtype)
    oracle_c.reduce_chunks(t_want, dtype, p, r, True)
    send_want = np.zeros(S, np.uint8)
    oracle_c.compress_onebit(t_want, dtype, p, r, out=send_want)
    K = bc._native.K
    recv_d = torch.from_numpy(recv).cuda()
    t_d = torch.full((p * cs,), 7.0, dtype=TORCH[dtype], device="cuda")
    send_d = torch.zeros(S, dtype=torch.uint8, device="cuda")
    ws = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
    rc = K.bagua_onebit_reduce_requantize(dtype, recv_d.data_ptr(), S, cs, p, t_d.data_ptr() if store else None,
                                          1, send_d.data_ptr(), S, r, ws.data_ptr(), ws.numel(), None)
    assert rc == 0
    got_t = to_host(t_d, dtype)
    if store:
        assert_float_bits_equal(got_t[r * cs:(r + 1) * cs], t_want[r * cs:(r + 1) * cs], dtype, "reduced chunk")
    else:
        assert np.all(got_t.astype(np.float32) == 7.0) if dtype != BF16 else np.all(got_t == 0x40E0)
    assert np.array_equal(segment_bytes(send_d.cpu().numpy(), p, r), segment_bytes(send_want, p, r))


@pytest.mark.parametrize("dtype", [F32, F16, BF16])
@pytest.mark.parametrize("p", [1, 2, 3, 4])
@pytest.mark.parametrize("kind", ["zeros", "signed_zeros", "huge", "nan_inf", "one_side"])
def test_onebit_fused_reduce_requantize_special(bc, oracle_c, dtype, p, kind):
    """The p <= 2 middle step's group-table path (full tiles: a 256-entry table of each
    sub-tile's |x| tree part, sign bits from the fields) and the 2 < p <= 4 pair-table path
    (each element pair's |x| sum and sign bits) on inputs whose reduced values are
    +-0, overflow to +-inf, are NaN or all one sign: the same bytes as the oracle's
    decompress + reduce_mean + compress(target)."""
    from oracle import oracle_np as NP
    rng = np.random.default_rng(500 + p + dtype)
    cs = 4 * 1024 + 3  # four full tiles (the table path) and a ragged one (the per-element path)
    base = (rng.standard_normal((p, p * cs)) * 1e-3).astype(np.float32)
    if kind == "zeros":
        base[:] = 0.0
    elif kind == "signed_zeros":
        base[:] = np.where(rng.random(base.shape) < 0.5, np.float32(-0.0), np.float32(0.0))
    elif kind == "huge":
        base = (np.sign(base) * np.float32(3e38)).astype(np.float32)
        if dtype != F32:
            base = np.sign(base).astype(np.float32) * np.float32(6e4)
    elif kind == "nan_inf":
        base[:, ::7] = np.inf
        base[:, 3::11] = np.nan
    else:
        base = np.abs(base) + np.float32(1e-4)
    xs = [NP.from_f32(base[r], dtype) for r in range(p)]
    r = p - 1
    comps = [oracle_c.compress_onebit(x, dtype, p) for x in xs]
    S = comps[0].size
    co = S // p
    recv = np.concatenate([c[r * co:(r + 1) * co] for c in comps])
    t_want = np.zeros(p * cs, STORAGE[dtype])
    oracle_c.decompress_onebit(recv, p, t_want, dtype)
    oracle_c.reduce_chunks(t_want, dtype, p, r, True)
    send_want = np.zeros(S, np.uint8)
    oracle_c.compress_onebit(t_want, dtype, p, r, out=send_want)
    K = bc._native.K
    recv_d = torch.from_numpy(recv).cuda()
    send_d = torch.zeros(S, dtype=torch.uint8, device="cuda")
    ws = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
    assert K.bagua_onebit_reduce_requantize(dtype, recv_d.data_ptr(), S, cs, p, None, 1, send_d.data_ptr(), S, r,
                                            ws.data_ptr(), ws.numel(), None) == 0
    assert np.array_equal(segment_bytes(send_d.cpu().numpy(), p, r), segment_bytes(send_want, p, r)), kind


@pytest.mark.parametrize("dtype", [F32, F16, BF16])
@pytest.mark.parametrize("p,cs,pieces,offset", [(1, 5 * 1024 + 17, 3, 0), (3, 4096, 5, 1), (2, 100000, 4, 0),
                                                (4, 700, 2, 0)])
def test_onebit_piecewise_building_blocks(bc, oracle_c, dtype, p, cs, pieces, offset):
    """encode_range over every piece + finalize == bagua_onebit_compress; decompress_range over
    every piece == bagua_onebit_decompress (the pipelined op's building blocks)."""
    from oracle import oracle_np as NP
    rng = np.random.default_rng(cs + p + pieces)
    x = NP.from_f32((rng.standard_normal(p * cs) * 1e-3).astype(np.float32), dtype)
    want = oracle_c.compress_onebit(x, dtype, p)
    K = bc._native.K
    xt = to_dev(x, dtype, offset)
    S = K.bagua_onebit_compressed_bytes(cs, p)
    assert S == want.size
    out = torch.full((S,), 0x5A, dtype=torch.uint8, device="cuda")
    wsb = K.bagua_onebit_workspace_bytes(cs, p)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    b, e = ctypes.c_int(), ctypes.c_int()
    ranges = []
    for q in range(pieces):
        assert K.bagua_onebit_piece_range(cs, pieces, q, ctypes.byref(b), ctypes.byref(e)) == 0
        ranges.append((b.value, e.value))
        assert K.bagua_onebit_encode_range(dtype, xt.data_ptr(), p * cs, cs, p, out.data_ptr(), S, ws.data_ptr(), wsb,
                                           b.value, e.value, None) == 0
    tiles = (cs + 1023) // 1024
    assert ranges[0][0] == 0 and ranges[-1][1] == tiles
    assert all(ranges[i][1] == ranges[i + 1][0] for i in range(pieces - 1))
    assert K.bagua_onebit_finalize(ws.data_ptr(), wsb, p * cs, cs, p, out.data_ptr(), S, None) == 0
    assert np.array_equal(out.cpu().numpy(), want)
    dec = torch.zeros(p * cs, dtype=TORCH[dtype], device="cuda")
    for tb, te in ranges:
        assert K.bagua_onebit_decompress_range(dtype, out.data_ptr(), S, cs, p, dec.data_ptr(), tb, te, None) == 0
    dw = np.zeros(p * cs, STORAGE[dtype])
    oracle_c.decompress_onebit(want, p, dw, dtype)
    assert_float_bits_equal(to_host(dec, dtype), dw, dtype, "pieced 1-bit decode")


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("p,cs,offset", [(1, 3 * 1024 * 1024 + 17, 0), (2, 1500, 1), (1, 1024 * 1100, 2),
                                         (1, 65 * (1 << 20) + 5 * 1024 + 3, 0), (8, 4 * (1 << 20) + 7, 0)])
def test_onebit_vs_oracle(bc, oracle_c, dtype, p, cs, offset):
    """The last two shapes drive the finalize's scale tree through its batch paths: 66 groups of
    1,024 tile partials (one full batch of 64, then a batch of one full group, one ragged group
    and empty ones) and 8 chunks of 5 groups (a ragged batch each)."""
    from oracle import oracle_np as NP
    rng = np.random.default_rng(cs + p)
    x = NP.from_f32((rng.standard_normal(p * cs) * 1e-3).astype(np.float32), dtype)
    want = oracle_c.compress_onebit(x, dtype, p)
    comp = bc.BaguaTensorPy(to_dev(x, dtype, offset), "x").compress("OneBitSignScale", p, -1)
    assert np.array_equal(comp.to_numpy_u8(), want)


# ---------------------------------------------------------- elementwise -----
@pytest.mark.parametrize("dtype", [F32, F16, BF16])
def test_add_addmul(bc, oracle_c, dtype):
    from oracle import oracle_np as NP
    rng = np.random.default_rng(5 + dtype)
    n = 100003
    x = NP.from_f32(rng.standard_normal(n).astype(np.float32), dtype)
    y = NP.from_f32(rng.standard_normal(n).astype(np.float32), dtype)
    xd, yd = to_dev(x, dtype), to_dev(y, dtype)
    tx, ty = bc.BaguaTensorPy(xd, "x"), bc.BaguaTensorPy(yd, "y")
    want = x.copy()
    for f in (float(np.float32(1.0 / 3.0)), float(np.float32(-5.0 / 3.0))):
        tx.addmul_inplace(ty, f)
        oracle_c.addmul_inplace(want, y, dtype, f)
    tx.add_inplace(ty)
    oracle_c.add_inplace(want, y, dtype)
    assert_float_bits_equal(to_host(xd, dtype), want, dtype, "add/addmul")


# ------------------------------------------------------- full size (cfg 2) --
def test_full_size_256mib_parity(bc, oracle_c):
    """Config 2 at its real size: 256 MiB fp32 bucket, p = 1, against the C oracle."""
    n = 1 << 26
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    x = torch.randn(n, device="cuda", generator=g) * 1e-3
    t = bc.BaguaTensorPy(x, "bucket")
    comp = t.compress("MinMaxUInt8", 1, -1)
    out = torch.empty_like(x)
    bc.BaguaTensorPy(out, "o").decompress_from("MinMaxUInt8", 1, comp)
    xh = x.cpu().numpy()
    want = oracle_c.compress_minmax_u8(xh, F32, 1)
    got = comp.to_numpy_u8()
    assert np.array_equal(got, want)
    dw = np.empty_like(xh)
    oracle_c.decompress_minmax_u8(want, 1, dw, F32)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), dw.view(np.uint32))
    bound = 0.5 * (float(xh.max()) - float(xh.min()) + 1e-7) / 255 * (1 + 1e-4) + 2 * float(np.spacing(np.float32(
        np.abs(xh).max())))
    assert float(np.abs(dw.astype(np.float64) - xh).max()) <= bound


def test_maximum_size_bucket_parity(bc, oracle_c):
    """The largest bucket the reference's int32 ABI can describe (K:573-691 take
    `int` element counts): n = 2^31 - 32 fp32 elements (8 GiB) in p = 4 chunks,
    so every 64-bit offset path of the kernels is exercised.  Payload, headers
    and the decoded tensor must equal the C oracle bit-for-bit."""
    n, p = (1 << 31) - 32, 4
    g = torch.Generator(device="cuda").manual_seed(31)
    x = torch.randn(n, device="cuda", generator=g)
    x[n - 1] = 7.5  # the maximum sits in the very last element of the last chunk
    t = bc.BaguaTensorPy(x, "max_bucket")
    comp = t.compress("MinMaxUInt8", p, -1)
    got = comp.to_numpy_u8()
    xh = x.cpu().numpy()
    want = oracle_c.compress_minmax_u8(xh, F32, p)
    assert got.size == want.size
    assert np.array_equal(got, want)
    del got
    out = torch.empty_like(x)
    bc.BaguaTensorPy(out, "o").decompress_from("MinMaxUInt8", p, comp)
    del x
    dw = np.empty_like(xh)
    del xh
    oracle_c.decompress_minmax_u8(want, p, dw, F32)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), dw.view(np.uint32))


def test_time_next_kernel_records_one_launch(bc):
    """The measurement hook: the next launch records its own start/stop events; one-shot."""
    K, N = bc._native.K, bc._native
    n = 1 << 24
    x = torch.randn(n, device="cuda")
    S = K.bagua_minmax_u8_compressed_bytes(F32, n, 1)
    out = torch.empty(S, dtype=torch.uint8, device="cuda")
    wsb = K.bagua_minmax_u8_workspace_bytes(n, 1)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    b.record(st)
    torch.cuda.synchronize()
    N.check(K.bagua_time_next_kernel(a.cuda_event, b.cuda_event), "hook")
    N.check(K.bagua_minmax_u8_compress_stage(1, F32, x.data_ptr(), n, n, 1, out.data_ptr(), S, ws.data_ptr(), wsb, -1,
                                             ctypes.c_void_p(st.cuda_stream)), "partials")
    torch.cuda.synchronize()
    t1 = a.elapsed_time(b)
    assert 0.0 < t1 < 50.0  # ms: one 64 MiB read
    # disarmed: a second launch leaves the events alone
    N.check(K.bagua_minmax_u8_compress_stage(2, F32, x.data_ptr(), n, n, 1, out.data_ptr(), S, ws.data_ptr(), wsb, -1,
                                             ctypes.c_void_p(st.cuda_stream)), "quantise")
    torch.cuda.synchronize()
    assert a.elapsed_time(b) == t1


@pytest.mark.parametrize("dtype", [F32, F16, BF16])
@pytest.mark.parametrize("case", ["normal", "offset", "nan_mixed", "pos_inf", "both_inf", "all_nan", "constant",
                                  "huge_range", "tiny"])
@pytest.mark.parametrize("offset", [0, 1])
def test_one_rank_op_matches_sequence(bc, oracle_c, dtype, case, offset):
    """bagua_minmax_u8_centralized_one_rank (min/max pass + one table-driven pass) ==
    the reference op sequence at p = 1 (centralized_low_precision_synchronous.rs:30-71:
    compress, decompress, reduce, compress, decompress), regular and degenerate regimes,
    aligned and misaligned tensors, mean and sum."""
    from oracle import oracle_np as NP
    from oracle import simulate
    K = bc._native.K
    rng = np.random.default_rng(len(case) * 7 + dtype + offset)
    n = 5 if case == "tiny" else (1 << 20) + 37
    big = {F32: 3e38, F16: 6e4, BF16: 3e38}[dtype]
    v = (rng.standard_normal(n) * 1e-3).astype(np.float32)
    if case == "offset":
        v += 7.5
    elif case == "nan_mixed":
        v[::7] = np.nan
    elif case == "pos_inf":
        v[5] = np.inf
    elif case == "both_inf":
        v[3], v[4] = np.inf, -np.inf
    elif case == "all_nan":
        v[:] = np.nan
    elif case == "constant":
        v[:] = 0.25
    elif case == "huge_range":
        v[0], v[1] = big, -big
    x = NP.from_f32(v, dtype)
    wsb = K.bagua_minmax_u8_workspace_bytes(n, 1)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    for average in (1, 0):
        want = simulate.centralized_low_precision(oracle_c, [x.copy()], dtype, bool(average))[0]
        xt = to_dev(x, dtype, offset)
        assert K.bagua_minmax_u8_centralized_one_rank(dtype, xt.data_ptr(), n, average, ws.data_ptr(), wsb, None) == 0
        assert_float_bits_equal(to_host(xt, dtype), want, dtype, f"one rank {case} average={average}")


@pytest.mark.parametrize("keep_mib", ["0", "1"])
@pytest.mark.parametrize("dtype", [F32, BF16])
def test_one_rank_op_load_policy_split(bc, oracle_c, dtype, keep_mib, monkeypatch):
    """The one-rank op's min/max pass with non-temporal loads below the kept tail
    (BAGUA_ONE_RANK_KEEP_MIB: all of it at 0, all but the last MiB at 1) gives the
    same bits as the reference sequence: the load policy moves no value."""
    from oracle import oracle_np as NP
    from oracle import simulate
    K = bc._native.K
    monkeypatch.setenv("BAGUA_ONE_RANK_KEEP_MIB", keep_mib)
    rng = np.random.default_rng(int(keep_mib) * 3 + dtype)
    n = (3 << 20) + 4099
    v = (rng.standard_normal(n) * 1e-3).astype(np.float32)
    v[n // 2] = 0.75  # the max inside the non-temporal part
    v[n - 9] = -0.5   # the min inside the kept tail
    x = NP.from_f32(v, dtype)
    wsb = K.bagua_minmax_u8_workspace_bytes(n, 1)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    want = simulate.centralized_low_precision(oracle_c, [x.copy()], dtype, True)[0]
    xt = to_dev(x, dtype, 0)
    assert K.bagua_minmax_u8_centralized_one_rank(dtype, xt.data_ptr(), n, 1, ws.data_ptr(), wsb, None) == 0
    assert_float_bits_equal(to_host(xt, dtype), want, dtype, f"one rank keep={keep_mib}")


@pytest.mark.parametrize("dtype", [F32, F16, BF16])
@pytest.mark.parametrize("case", ["normal", "ragged", "offset", "nan_mixed", "pos_inf", "both_inf", "all_nan",
                                  "zeros", "neg_zeros", "constant", "huge", "tiny", "one"])
@pytest.mark.parametrize("offset", [0, 1])
def test_onebit_one_rank_op_matches_sequence(bc, oracle_c, dtype, case, offset):
    """bagua_onebit_centralized_one_rank (encode pass, one workgroup for both scales, one pass
    writing +-scale2 from the bits) == the 1-bit op's sequence at p = 1 (encode, decode +
    reduce + re-encode, decode; centralized_low_precision_synchronous.rs:30-71 with the
    1-bit codec), bit for bit: regular, ragged last tile, +-0, NaN / Inf, overflowing
    scale sums, tiny tensors; aligned and misaligned; mean and sum."""
    from oracle import oracle_np as NP
    from oracle import simulate
    K = bc._native.K
    rng = np.random.default_rng(len(case) * 11 + dtype + offset)
    n = {"tiny": 5, "one": 1, "ragged": (1 << 20) + 37}.get(case, 1 << 20)
    big = {F32: 3e38, F16: 6e4, BF16: 3e38}[dtype]
    v = (rng.standard_normal(n) * 1e-3).astype(np.float32)
    if case == "offset":
        v += 7.5
    elif case == "nan_mixed":
        v[::7] = np.nan
    elif case == "pos_inf":
        v[5] = np.inf
    elif case == "both_inf":
        v[3], v[4] = np.inf, -np.inf
    elif case == "all_nan":
        v[:] = np.nan
    elif case == "zeros":
        v[:] = 0.0
    elif case == "neg_zeros":
        v[:] = -0.0
        v[::3] = 0.0
    elif case == "constant":
        v[:] = -0.25
    elif case == "huge":
        v[:] = big  # the |x| tree overflows to inf
        v[1::2] = -big
    x = NP.from_f32(v, dtype)
    wsb = K.bagua_onebit_one_rank_workspace_bytes(n)
    ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
    for average in (1, 0):
        want = simulate.centralized_low_precision(oracle_c, [x.copy()], dtype, bool(average),
                                                  method="OneBitSignScale")[0]
        xt = to_dev(x, dtype, offset)
        assert K.bagua_onebit_centralized_one_rank(dtype, xt.data_ptr(), n, average, ws.data_ptr(), wsb, None) == 0
        assert_float_bits_equal(to_host(xt, dtype), want, dtype, f"1-bit one rank {case} average={average}")


@pytest.mark.parametrize("fused", ["1", "0"])
def test_onebit_one_rank_through_the_op(bc, oracle_c, fused, monkeypatch):
    """The centralized op at one rank with the 1-bit codec takes the two-pass path
    (BAGUA_ONE_RANK_FUSED=1, the default) or the full sequence (0): same bytes, the oracle's."""
    from bagua_core.communicator import loopback_communicators
    from oracle import simulate
    monkeypatch.setenv("BAGUA_ONE_RANK_FUSED", fused)
    N = bc._native
    n = (1 << 21) + 1000
    x = (np.random.default_rng(5).standard_normal(n) * 1e-3).astype(np.float32)
    want = simulate.centralized_low_precision(oracle_c, [x.copy()], F32, True, method="OneBitSignScale")[0]
    comm = loopback_communicators(1, 0)[0]
    t = torch.from_numpy(x.copy()).cuda()
    torch.cuda.synchronize()
    raw = bc.BaguaTensorPy(t, "g").raw()
    N.check(N.C.bagua_centralized_low_precision_synchronous(comm.handle, ctypes.byref(raw), 1, N.COMPRESSION_ONEBIT),
            "1-bit op")
    comm.synchronize()
    assert_float_bits_equal(t.cpu().numpy(), want, F32, f"fused={fused}")
