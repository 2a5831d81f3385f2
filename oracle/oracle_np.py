"""Independent numpy restatement of the bagua-core codec hot path.

TEST INFRASTRUCTURE ONLY.  Written separately from the C oracle
(oracle/bagua_oracle.c); the two must agree bit-for-bit on every fixture
(tests/test_oracle.py).  Citations (reference repo paths):
  K  = bagua-core-internal/kernels/bagua_kernels.cu
  DT = bagua-core-internal/src/datatypes/mod.rs
All arithmetic is numpy float32 elementwise (one IEEE op per ufunc, RNE),
so expression order below mirrors the CUDA source exactly.
"""
from __future__ import annotations

import numpy as np

F32, F16, BF16 = 0, 1, 2
EPS = np.float32(1e-7)  # K:10 `const float eps = 1e-7;`
INIT_MAX = {F32: np.float32(np.finfo(np.float32).max), F16: np.float32(65504.0),
            BF16: np.uint32(0x7F7F0000).view(np.float32)}


# ---------------------------------------------------------------- dtypes ----
def to_f32(x: np.ndarray, dtype: int) -> np.ndarray:
    if dtype == F32:
        return x.astype(np.float32, copy=False)
    if dtype == F16:
        return x.astype(np.float16, copy=False).astype(np.float32)
    return (x.astype(np.uint32) << 16).view(np.float32)


def from_f32(v: np.ndarray, dtype: int) -> np.ndarray:
    v = np.asarray(v, dtype=np.float32)
    if dtype == F32:
        return v.copy()
    if dtype == F16:
        return v.astype(np.float16)
    u = v.view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def raw_bytes(v: float, dtype: int) -> bytes:
    return from_f32(np.array([v], np.float32), dtype).tobytes()


def from_raw(b: bytes, dtype: int) -> np.float32:
    if dtype == F32:
        return np.frombuffer(b[:4], np.float32)[0]
    if dtype == F16:
        return np.float32(np.frombuffer(b[:2], np.float16)[0])
    return to_f32(np.frombuffer(b[:2], np.uint16), BF16)[0]


def esize(dtype: int) -> int:
    return 4 if dtype == F32 else 2


# ----------------------------------------------------------------- sizes ----
def _align(x: int, a: int) -> int:
    return (x + a - 1) // a * a


def minmax_compressed_size(n_chunks: int, chunk_size: int, dtype: int) -> int:
    # DT:679-693
    return _align(chunk_size * n_chunks, 32) + _align(2 * esize(dtype), 32) * n_chunks


# ---------------------------------------------------------------- minmax ----
def minmax(xf: np.ndarray, dtype: int) -> tuple[np.float32, np.float32]:
    """cub Min/Max with init +-T_MAX (K:312-371); NaN skipped, -0 < +0."""
    init = INIT_MAX[dtype]
    v = np.ascontiguousarray(xf[~np.isnan(xf)], np.float32)

    def keys(a):
        i = a.view(np.int32)
        return i ^ ((i >> 31) & 0x7FFFFFFF)
    kmin = keys(np.concatenate([v, np.array([init], np.float32)])).min()
    kmax = keys(np.concatenate([v, np.array([-init], np.float32)])).max()

    def back(k):
        k = np.int32(k)
        return np.array([k ^ ((k >> 31) & 0x7FFFFFFF)], np.int32).view(np.float32)[0]
    return back(kmin), back(kmax)


def qparams(mn: np.float32, mx: np.float32):
    # K:465-467: scale = 255.0 / (max - min + eps) in double, stored as float
    d = np.float32(np.float32(mx - mn) + EPS)
    scale = np.float32(np.float64(255.0) / np.float64(d))
    ub = np.float32(np.rint(np.float32(mx * scale)))
    lb = np.float32(np.float64(ub) - 255.0)
    return scale, lb, ub


def quantize(xf: np.ndarray, scale, lb, ub) -> np.ndarray:
    # K:410-422
    with np.errstate(all="ignore"):
        level = np.rint(xf * scale)
        level = np.fmin(level, ub)
        v = level - lb
        v = np.fmin(np.fmax(v, np.float32(0)), np.float32(255))
    return v.astype(np.uint8)


def dequantize(q: np.ndarray, scale, lb) -> np.ndarray:
    # K:424-432
    with np.errstate(all="ignore"):
        return (q.astype(np.float32) + lb) / scale


def compress_minmax_u8(x: np.ndarray, dtype: int, n_chunks: int, target_chunk: int = -1,
                       out: np.ndarray | None = None, num_elem: int | None = None) -> np.ndarray:
    """K:533-560 + K:455-479 (+ zeroed header gap / slack).

    `num_elem` = the tensor's num_elements() (DT:339, default x.size).  The
    host loop K:538-545 hands cub `min(remaining, chunk_size)` elements per
    chunk (remaining may go negative: an empty range, header = init), while
    the quantise kernel K:468-472 runs i over the whole chunk_size -- so the
    elements past num_elem are outside the min/max but still quantised."""
    assert x.size % n_chunks == 0
    cs = x.size // n_chunks
    size = minmax_compressed_size(n_chunks, cs, dtype)
    if out is None:
        out = np.zeros(size, np.uint8)
    co = size // n_chunks
    es = esize(dtype)
    xf = to_f32(x, dtype)
    remaining = x.size if num_elem is None else int(num_elem)
    for c in range(n_chunks):
        n_valid = max(0, min(remaining, cs))
        remaining -= cs
        if target_chunk != -1 and c != target_chunk:
            continue
        seg = xf[c * cs:(c + 1) * cs]
        mn, mx = minmax(seg[:n_valid], dtype)
        head = np.zeros(32, np.uint8)
        head[:es] = np.frombuffer(raw_bytes(mn, dtype), np.uint8)
        head[es:2 * es] = np.frombuffer(raw_bytes(mx, dtype), np.uint8)
        base = c * co
        out[base:base + 32] = head
        scale, lb, ub = qparams(from_raw(head[:es].tobytes(), dtype), from_raw(head[es:2 * es].tobytes(), dtype))
        out[base + 32:base + 32 + cs] = quantize(seg, scale, lb, ub)
        out[base + 32 + cs:base + co] = 0
    if target_chunk == -1:
        out[n_chunks * co:] = 0
    return out


def decompress_minmax_u8(buf: np.ndarray, n_chunks: int, out: np.ndarray, dtype: int) -> np.ndarray:
    cs = out.size // n_chunks
    co = buf.size // n_chunks
    es = esize(dtype)
    for c in range(n_chunks):
        base = c * co
        scale, lb, _ = qparams(from_raw(buf[base:base + es].tobytes(), dtype),
                               from_raw(buf[base + es:base + 2 * es].tobytes(), dtype))
        out[c * cs:(c + 1) * cs] = from_f32(dequantize(buf[base + 32:base + 32 + cs], scale, lb), dtype)
    return out


# ---------------------------------------------------------------- reduce ----
def reduce_chunks(x: np.ndarray, dtype: int, n_chunks: int, target_chunk: int, average: bool) -> np.ndarray:
    """K:373-400 with the K:171-194 tree and K:502-531 block_dim_y table."""
    p = n_chunks
    cs = x.size // p
    by = 2 if p <= 4 else 4 if p <= 8 else 8 if p <= 16 else 16 if p <= 32 else 32
    xf = to_f32(x, dtype).reshape(p, cs)
    s = []
    for y in range(by):
        acc = np.zeros(cs, np.float32)
        for i in range(y, p, by):
            acc = acc + xf[i]
        s.append(acc)
    h = by // 2
    while h >= 1:
        for y in range(h):
            s[y] = s[y] + s[y + h]
        h //= 2
    r = s[0] / np.float32(p) if average else s[0]
    x[target_chunk * cs:(target_chunk + 1) * cs] = from_f32(r, dtype)
    return x


# ----------------------------------------------------------- elementwise ----
def add_inplace(x: np.ndarray, y: np.ndarray, dtype: int) -> np.ndarray:
    x[...] = from_f32(to_f32(x, dtype) + to_f32(y, dtype), dtype)
    return x


def addmul_inplace(x: np.ndarray, y: np.ndarray, dtype: int, factor: float) -> np.ndarray:
    if dtype == F32:
        # nvcc -fmad=true contracts `x += y*factor` into fmaf(y, factor, x)
        x[...] = fma_f32(y, np.float32(factor), x)
        return x
    fh = to_f32(from_f32(np.array([factor], np.float32), dtype), dtype)[0]
    prod = to_f32(from_f32(to_f32(y, dtype) * fh, dtype), dtype)
    x[...] = from_f32(to_f32(x, dtype) + prod, dtype)
    return x


def fma_f32(y: np.ndarray, f: np.float32, x: np.ndarray) -> np.ndarray:
    """Correctly rounded fmaf(y, f, x) for float32 arrays.  y*f is exact in
    float64; the float64 sum s has an exact error term (TwoSum).  Rounding s to
    float32 is correct unless s sits exactly on a float32 midpoint with a
    nonzero error, in which case the error decides the direction."""
    a = x.astype(np.float64)
    b = y.astype(np.float64) * np.float64(f)
    s = a + b
    bb = s - a
    err = (a - (s - bb)) + (b - bb)
    with np.errstate(over="ignore", invalid="ignore"):
        r = s.astype(np.float32)
        up = np.nextafter(r, np.float32(np.inf))
        dn = np.nextafter(r, np.float32(-np.inf))
        m_up = (r.astype(np.float64) + up.astype(np.float64)) / 2
        m_dn = (r.astype(np.float64) + dn.astype(np.float64)) / 2
        r = np.where((s == m_up) & (err > 0), up, r)
        r = np.where((s == m_dn) & (err < 0), dn, r)
    return r.astype(np.float32)


# ----------------------------------------------------------------- 1-bit ----
OB_TILE, OB_TILE_BYTES = 1024, 128


def onebit_compressed_size(n_chunks: int, chunk_size: int) -> int:
    tiles = (chunk_size + OB_TILE - 1) // OB_TILE
    return n_chunks * (32 + tiles * OB_TILE_BYTES)


def _tile_partials(v: np.ndarray) -> np.ndarray:
    nt = (v.size + OB_TILE - 1) // OB_TILE
    a = np.zeros(nt * OB_TILE, np.float32)
    a[:v.size] = v
    a = a.reshape(nt, 4, 64, 4)                        # [tile][sub][lane][e]
    q = (a[..., 0] + a[..., 1]) + (a[..., 2] + a[..., 3])  # [tile][sub][lane]
    s = (q[:, 0] + q[:, 1]) + (q[:, 2] + q[:, 3])      # [tile][lane]
    h = 32
    while h >= 1:
        s = s[:, :h] + s[:, h:2 * h]
        h //= 2
    return s[:, 0]


def onebit_tree_sum(v: np.ndarray) -> np.float32:
    v = np.asarray(v, np.float32)
    if v.size == 0:
        return np.float32(0)
    while True:
        p = _tile_partials(v)
        if v.size <= OB_TILE:
            return p[0]
        v = p


def compress_onebit(x: np.ndarray, dtype: int, n_chunks: int, target_chunk: int = -1,
                    out: np.ndarray | None = None) -> np.ndarray:
    assert x.size % n_chunks == 0
    cs = x.size // n_chunks
    size = onebit_compressed_size(n_chunks, cs)
    if out is None:
        out = np.zeros(size, np.uint8)
    co = size // n_chunks
    tiles = (cs + OB_TILE - 1) // OB_TILE
    xf = to_f32(x, dtype)
    for c in range(n_chunks):
        if target_chunk != -1 and c != target_chunk:
            continue
        seg = xf[c * cs:(c + 1) * cs]
        with np.errstate(all="ignore"):
            total = onebit_tree_sum(np.abs(seg))
            scale = np.float32(total / np.float32(cs)) if cs > 0 else np.float32(0)
        base = c * co
        head = np.zeros(32, np.uint8)
        head[:4] = np.frombuffer(np.float32(scale).tobytes(), np.uint8)
        head[4:8] = np.frombuffer(np.uint32(cs).tobytes(), np.uint8)
        out[base:base + 32] = head
        neg = np.zeros(tiles * OB_TILE, np.uint8)
        neg[:cs] = seg < 0
        # [tile][sub][lane][e] -> per lane a 16-bit field [tile][lane][sub*4+e]
        b = neg.reshape(tiles, 4, 64, 4).transpose(0, 2, 1, 3).reshape(tiles, 64, 16)
        packed = np.packbits(b, axis=-1, bitorder="little")  # [tile][64][2] bytes
        out[base + 32:base + 32 + tiles * OB_TILE_BYTES] = packed.reshape(-1)
        out[base + 32 + tiles * OB_TILE_BYTES:base + co] = 0
    if target_chunk == -1:
        out[n_chunks * co:] = 0
    return out


def decompress_onebit(buf: np.ndarray, n_chunks: int, out: np.ndarray, dtype: int) -> np.ndarray:
    cs = out.size // n_chunks
    co = buf.size // n_chunks
    tiles = (cs + OB_TILE - 1) // OB_TILE
    for c in range(n_chunks):
        base = c * co
        scale = np.frombuffer(buf[base:base + 4].tobytes(), np.float32)[0]
        packed = buf[base + 32:base + 32 + tiles * OB_TILE_BYTES].reshape(tiles, 64, 2)
        b = np.unpackbits(packed, axis=-1, bitorder="little")  # [tile][lane][sub*4+e]
        b = b.reshape(tiles, 64, 4, 4).transpose(0, 2, 1, 3).reshape(-1)[:cs]
        vals = np.where(b.astype(bool), -scale, scale).astype(np.float32)
        out[c * cs:(c + 1) * cs] = from_f32(vals, dtype)
    return out
