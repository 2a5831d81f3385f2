"""ctypes wrapper of the C oracle (oracle/bagua_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the parity checker; the product path never
imports anything under oracle/.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libbagua_oracle.so")

F32, F16, BF16 = 0, 1, 2
DTYPE_CODE = {"f32": F32, "f16": F16, "bf16": BF16}
# numpy storage dtype per code (bf16 is carried as raw uint16 bits)
NP_STORAGE = {F32: np.float32, F16: np.float16, BF16: np.uint16}

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, sz, i32, i64, f32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int64, ctypes.c_float
        L.orc_minmax_compressed_size.argtypes = [i32, sz, i32]
        L.orc_minmax_compressed_size.restype = sz
        L.orc_minmax.argtypes = [vp, i32, i64, ctypes.POINTER(f32), ctypes.POINTER(f32)]
        L.orc_compress_minmax_u8.argtypes = [vp, i32, i32, i32, i32, vp, sz, i32]
        L.orc_decompress_minmax_u8.argtypes = [vp, sz, i32, i32, vp, i32]
        L.orc_reduce_chunks.argtypes = [vp, i32, i32, i32, i32, i32]
        L.orc_add_inplace.argtypes = [vp, vp, i32, i64]
        L.orc_addmul_inplace.argtypes = [vp, vp, i32, i64, f32]
        L.orc_onebit_compressed_size.argtypes = [i32, sz]
        L.orc_onebit_compressed_size.restype = sz
        L.orc_onebit_tree_sum.argtypes = [vp, i64]
        L.orc_onebit_tree_sum.restype = f32
        L.orc_compress_onebit.argtypes = [vp, i32, i32, i32, i32, vp, sz, i32]
        L.orc_decompress_onebit.argtypes = [vp, sz, i32, i32, vp, i32]
        L.orc_half_to_float.argtypes = [ctypes.c_uint16]
        L.orc_half_to_float.restype = f32
        L.orc_float_to_half.argtypes = [f32]
        L.orc_float_to_half.restype = ctypes.c_uint16
        L.orc_bf16_to_float.argtypes = [ctypes.c_uint16]
        L.orc_bf16_to_float.restype = f32
        L.orc_float_to_bf16.argtypes = [f32]
        L.orc_float_to_bf16.restype = ctypes.c_uint16
        L.orc_num_threads.restype = i32
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def num_threads() -> int:
    return lib().orc_num_threads()


def set_num_threads(n: int) -> int:
    """OpenMP threads for later calls; returns the team size now in effect"""
    f = lib().orc_set_num_threads
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_int]
    return f(int(n))


def minmax_compressed_size(n_chunks: int, chunk_size: int, dtype: int) -> int:
    return lib().orc_minmax_compressed_size(n_chunks, chunk_size, dtype)


def onebit_compressed_size(n_chunks: int, chunk_size: int) -> int:
    return lib().orc_onebit_compressed_size(n_chunks, chunk_size)


def minmax(x: np.ndarray, dtype: int) -> tuple[float, float]:
    mn, mx = ctypes.c_float(), ctypes.c_float()
    lib().orc_minmax(_ptr(x), dtype, x.size, ctypes.byref(mn), ctypes.byref(mx))
    return mn.value, mx.value


def compress_minmax_u8(x: np.ndarray, dtype: int, n_chunks: int, target_chunk: int = -1,
                       out: np.ndarray | None = None, num_elem: int | None = None) -> np.ndarray:
    """BaguaTensor.compress("MinMaxUInt8", n_chunks, target_chunk) on a host array.
    `num_elem` (default x.size) is the tensor's num_elements() (DT:339): elements
    past it are left out of the chunk's min/max (K:538-545, min(remaining, cs))
    but still quantised with that chunk's parameters (K:468-472 loops over every
    i < chunk_size).  An empty chunk gets the init header (+-T_MAX) and, for
    f32/bf16, scale = -0 and every byte 255 (decodes to NaN)."""
    assert x.size % n_chunks == 0, "compression tensor size % n_chunks must be 0"
    cs = x.size // n_chunks
    size = minmax_compressed_size(n_chunks, cs, dtype)
    if out is None:
        out = np.zeros(size, dtype=np.uint8)
    n = x.size if num_elem is None else int(num_elem)
    rc = lib().orc_compress_minmax_u8(_ptr(x), dtype, n, cs, n_chunks, _ptr(out), size, target_chunk)
    assert rc == 0, rc
    return out


def decompress_minmax_u8(buf: np.ndarray, n_chunks: int, out: np.ndarray, dtype: int) -> np.ndarray:
    cs = out.size // n_chunks
    rc = lib().orc_decompress_minmax_u8(_ptr(buf), buf.size, cs, n_chunks, _ptr(out), dtype)
    assert rc == 0, rc
    return out


def reduce_chunks(x: np.ndarray, dtype: int, n_chunks: int, target_chunk: int, average: bool) -> np.ndarray:
    cs = x.size // n_chunks
    rc = lib().orc_reduce_chunks(_ptr(x), dtype, cs, n_chunks, target_chunk, int(bool(average)))
    assert rc == 0, rc
    return x


def add_inplace(x: np.ndarray, y: np.ndarray, dtype: int) -> np.ndarray:
    lib().orc_add_inplace(_ptr(x), _ptr(y), dtype, x.size)
    return x


def addmul_inplace(x: np.ndarray, y: np.ndarray, dtype: int, factor: float) -> np.ndarray:
    lib().orc_addmul_inplace(_ptr(x), _ptr(y), dtype, x.size, factor)
    return x


def onebit_tree_sum(v: np.ndarray) -> float:
    v = np.ascontiguousarray(v, dtype=np.float32)
    return lib().orc_onebit_tree_sum(_ptr(v), v.size)


def compress_onebit(x: np.ndarray, dtype: int, n_chunks: int, target_chunk: int = -1,
                    out: np.ndarray | None = None) -> np.ndarray:
    assert x.size % n_chunks == 0
    cs = x.size // n_chunks
    size = onebit_compressed_size(n_chunks, cs)
    if out is None:
        out = np.zeros(size, dtype=np.uint8)
    rc = lib().orc_compress_onebit(_ptr(x), dtype, x.size, cs, n_chunks, _ptr(out), size, target_chunk)
    assert rc == 0, rc
    return out


def decompress_onebit(buf: np.ndarray, n_chunks: int, out: np.ndarray, dtype: int) -> np.ndarray:
    cs = out.size // n_chunks
    rc = lib().orc_decompress_onebit(_ptr(buf), buf.size, cs, n_chunks, _ptr(out), dtype)
    assert rc == 0, rc
    return out
